#!/bin/bash
# round 6 A: new tests (async JIT swap, code copies without narrow codes, hang handling), C2 bench line with cold start
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jit_async.py tests/test_gpu_parity.py -k "async or jit_wait or code_copies or specialised or compact" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_c2.json')); r=d['roofline']
print('c2', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['frac']); print('cold', json.dumps(d['cold_start'])); print('c5', {k: d['c5'].get(k) for k in ('value','ms_per_step','error')})"
