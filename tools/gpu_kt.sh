# usage: bash tools/gpu_kt.sh TAG CONFIG [ENV=VAL ...] -- rocprofv3 kernel-trace summary of one bench config
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; shift 2
for kv in "$@"; do export "$kv"; done
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$CFG -o kt -- python3 bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_$CFG.json 2> $OUT/kt_$CFG.err || exit $?
f=$(find $OUT/kt_$CFG -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('%-40s calls %5s avg %9.1f us  total %8.3f ms' % (r['Name'][:40], r['Calls'], float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e6))
PY
