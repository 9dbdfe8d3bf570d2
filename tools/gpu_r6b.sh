#!/bin/bash
# round 6 B: cold first query after the context warm-up and background module loads
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/cold_probe.py > $OUT/cold_probe.json 2> $OUT/cold_probe.err || { tail -20 $OUT/cold_probe.err; exit 1; }
cat $OUT/cold_probe.json
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jit_async.py tests/test_gpu_dist.py tests/test_gpu_merge.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -2 $OUT/smoke.txt
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_c2.json')); r=d['roofline']
print('c2', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['frac']); print('cold', json.dumps(d['cold_start']))"
