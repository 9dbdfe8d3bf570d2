#!/bin/bash
# round 6 M: C2 step with / without an explicit dispatch flush after the scan launch (A/B on one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6m}
mkdir -p $OUT
for r in 1 2 3; do
for x in 0 1; do
BQGPU_EXP=$x timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/x${x}_$r.json 2> $OUT/x${x}_$r.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/x${x}_$r.json'));print('exp=$x', round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4))"
done
done
