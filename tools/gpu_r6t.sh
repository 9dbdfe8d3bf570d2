#!/bin/bash
# round 6 T: the wider context warm-up -- cold first queries of C2 / C3 / C4, context creation time, a test subset
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6t}
mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c3 c4; do
timeout -k 10 200 python tools/cold_probe.py $c > $OUT/cold_$c.json 2> $OUT/cold_$c.err || { tail -20 $OUT/cold_$c.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/cold_$c.json'));print('$c', 'context %.1f ms' % d['context_ms'], 'first', d['first'], 'second', d['second'])"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_jit_async.py tests/test_gpu_parity.py -k "memory_budget or engine_options or async or jit_wait or specialised" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
