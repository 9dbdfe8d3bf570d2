#!/bin/bash
# round 6 P: C2 step with the HIP runtime spinning on completion (hipDeviceScheduleSpin) vs the default (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6p}
mkdir -p $OUT
for r in 1 2 3; do
for x in 0 2; do
BQGPU_EXP=$x timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/x${x}_$r.json 2> $OUT/x${x}_$r.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/x${x}_$r.json'));print('exp=$x', round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4))"
done
done
grep EXP $OUT/x2_1.err | head -2
for x in 0 2; do
BQGPU_EXP=$x timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/c3_x${x}.json 2> $OUT/c3_x${x}.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_x${x}.json'));print('c3 exp=$x', round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4))"
done
