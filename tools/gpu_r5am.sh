#!/bin/bash
# windows past the row-record tiles load no row records: parity (partitioned, first rows, fuzz), C3 kernel times, C3/C5 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5am}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py -m gpu -k "first_rows or partitioned or random or c3 or c5 or C3 or C5" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt1 -o kt -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record > $OUT/kt1.json 2> $OUT/kt1.err || exit $?
python3 -c "
import csv
tot=0
for r in csv.DictReader(open('$OUT/kt1/kt_kernel_stats.csv')):
    if 'part' in r['Name']:
        print('  %-40s %8.1f us' % (r['Name'][:40], float(r['AverageNs'])/1000)); tot+=float(r['AverageNs'])/1000
print('  total %.1f' % tot)"
for cfg in c3 c5; do
timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_$cfg.json')); r=d['roofline'] or {}; c=d.get('c5') or {}
print('$cfg', d['value'], round(d['ms_per_step'],4), r.get('kernel_avg_ms'), r.get('frac'), c.get('roofline_frac_of_the_shard_pass'))"
done
