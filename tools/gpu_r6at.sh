#!/bin/bash
# round 6 AT: C4's fused pass with its zeroed buffers cleared by one kernel: parity (parity and
# full-size suites) and the C4 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6at}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for v in "" "--sorted"; do
timeout -k 10 300 python bench.py --config c4 $v --steps 20 --warmup 3 --no-cpu-baseline --no-compact-record --no-cold-record > $OUT/bench_c4$v.json 2> $OUT/bench_c4$v.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_c4$v.json')); r=d['roofline']
print('c4 $v', round(d['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in r.items() if 'ms' in k or k == 'frac'})"
done
