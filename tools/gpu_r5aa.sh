# C3 aggregate launch sweep at HEAD: splits and window
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5aa}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for o in "" "part_splits=1" "part_splits=3" "part_splits=4" "part_win=1024" "part_win=2048"; do
i=$((i+1))
BQGPU_OPTIONS="$o" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$i -o kt -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record > $OUT/kt$i.json 2> $OUT/kt$i.err || exit $?
echo "== opts [$o]"; python3 -c "
import csv
tot=0
for r in csv.DictReader(open('$OUT/kt$i/kt_kernel_stats.csv')):
    if 'part' in r['Name']:
        print('  %-40s %8.1f us' % (r['Name'][:40], float(r['AverageNs'])/1000)); tot+=float(r['AverageNs'])/1000
print('  total %.1f' % tot)"
done
