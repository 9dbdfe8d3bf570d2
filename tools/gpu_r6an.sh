#!/bin/bash
# round 6 AN: final measurements at HEAD -- bench lines (C2 full line, C3, C4, C4 sorted, C5), kernel traces,
# HBM traffic passes, the C5 full shape on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6an}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
for c in c3 c4 c5; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
done
timeout -k 10 300 python bench.py --config c4 --sorted --no-cpu-baseline > $OUT/bench_c4_sorted.json 2> $OUT/bench_c4_sorted.err || exit $?
python3 - <<PY
import json
for c in ['c2','c3','c4','c4_sorted','c5']:
    d=json.load(open('$OUT/bench_%s.json' % c)); r=d.get('roofline') or {}
    print(c, '%.3e rows/s' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel %s' % r.get('kernel_avg_ms'), 'frac %s' % r.get('frac'), 'dev/query %s' % r.get('device_ms_per_query'))
d=json.load(open('$OUT/bench_c2.json'))
print('cold', d['cold_first_query_ms'], d['cold_start']['first_over_generic_steady'])
print('c5 sub', {k: d['c5'].get(k) for k in ('value','ms_per_step','merge_ms_max_over_ranks','roofline_frac_of_the_shard_pass')})
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
PY
B="--no-cpu-baseline --no-c5 --no-compact-record --no-cold-record"
for c in c2 c3 c4; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$c -o kt -- python3 bench.py --config $c --steps 10 --warmup 3 $B > $OUT/kt_$c.json 2> $OUT/kt_$c.err || exit $?
done
for c in c2 c3 c5; do
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 $B > /dev/null 2> $OUT/pf_$c.err || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 $B > /dev/null 2> $OUT/pw_$c.err || exit $?
done
python3 tools/pmc_to_json.py $OUT/pf_c2 $OUT/pw_c2 c2 100000000 $OUT/pmc_c2.json bq_jit_scan_private || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c3 $OUT/pw_c3 c3 100000000 $OUT/pmc_c3.json bq_jit_part_scatter k_part_aggregate k_part_combine bq_jit_part_first_rows || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c5 $OUT/pw_c5 c5 125000000 $OUT/pmc_c5.json bq_jit_part_scatter k_part_aggregate k_part_combine bq_jit_part_first_rows || exit $?
for c in c2 c3 c4; do echo "== $c"; python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kt_$c/kt_kernel_stats.csv')):
    print('  %-50s %6s %8.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1000))" | head -8; done
timeout -k 10 500 python bench.py --config c5 --local-ranks 8 --steps 5 --warmup 2 > $OUT/bench_c5_8ranks.json 2> $OUT/bench_c5_8ranks.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_c5_8ranks.json')); c=d['config']; p=c['projected_node']
print('c5 8 ranks', d['value'], d['ms_per_step'], 'proj', p['ms_per_step'], p['x_over_one_gpu'], 'merge crit', c['merge_ms_critical_path'])"
