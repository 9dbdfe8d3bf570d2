#!/bin/bash
# round 6 AS: ABI 10 (bqg_timing.copy_ms, roofline.frac_all_kernels): host / timing tests, the
# slot-emit parity, C3 and C2 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6as}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "slot_emit or timing or remaining_engine_options" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for c in c3 c2; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-compact-record --no-cold-record > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_$c.json')); r=d['roofline']
print('$c', round(d['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in r.items() if 'ms' in k or 'frac' in k})"
done
