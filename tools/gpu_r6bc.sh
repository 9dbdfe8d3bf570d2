#!/bin/bash
# round 6 BC: C4 chunk-combine run length sweep (temporary BQG_SCD_PER override)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6bc}
mkdir -p $OUT
export TMPDIR=/tmp
for per in 32 16 8 64; do
BQG_SCD_PER=$per timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$per -o kt --output-format csv -- python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/p$per.json 2> $OUT/p$per.err || exit 1
python3 - $OUT/p$per $per <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
t = 0
for r in csv.DictReader(open(f)):
    if 'scd_combine' in r['Name']:
        t += float(r['AverageNs']) / 1e3
        print('per', sys.argv[2], r['Name'][:40], round(float(r['AverageNs']) / 1e3, 1))
print('per', sys.argv[2], 'combine total', round(t, 1))
PY
done
