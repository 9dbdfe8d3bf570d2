#!/bin/bash
# round 6 AU: C5 step timeline (world 1) (kernels, copies, HIP calls)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6au}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $OUT/tl -o tl --output-format csv -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 tools/step_timeline.py $OUT/tl bq_jit_part_scatter > $OUT/timeline.txt
