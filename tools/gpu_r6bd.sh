#!/bin/bash
# round 6 BD: C4 combine at 16 chunks a run: distinct / scd parity (parity + full-size suites), C4 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6bd}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for v in "" "--sorted"; do
timeout -k 10 300 python bench.py --config c4 $v --steps 20 --warmup 3 --no-cpu-baseline --no-compact-record --no-cold-record > $OUT/bench_c4$v.json 2> $OUT/bench_c4$v.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_c4$v.json')); r=d['roofline']
print('c4 $v', round(d['ms_per_step'],4), 'kernel', round(r['kernel_avg_ms'],4), 'frac', round(r['frac'],4), 'device', round(r['device_ms_per_query'],4))"
done
