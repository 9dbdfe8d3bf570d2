#!/bin/bash
# late-first mode (part_first=3): parity tests, then C3 kernel times default vs part_first=3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5ai}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "first_rows or partitioned" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
i=0
for o in "" "part_first=3"; do
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
