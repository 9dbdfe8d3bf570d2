#!/bin/bash
# round 6 L: where C2's step time goes beside the scan (HIP API + kernel trace of the timed loop)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6l}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/tr -o tr -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/tr.json 2> $OUT/tr.err || { tail -20 $OUT/tr.err; exit 1; }
ls -R $OUT/tr | head -20
python3 tools/step_timeline.py $OUT/tr > $OUT/timeline.txt && cat $OUT/timeline.txt
