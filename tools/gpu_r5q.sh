# round-5 final B: kernel traces (C2 as stored, C3, C4 random) and HBM traffic passes (C2, C3, C5) at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5q}
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-c5 --no-compact-record"
for c in c2 c3 c4; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$c -o kt -- python3 bench.py --config $c --steps 10 --warmup 3 $B > $OUT/kt_$c.json 2> $OUT/kt_$c.err || exit $?
done
for c in c2 c3 c5; do
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 $B > /dev/null 2> $OUT/pf_$c.err || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 $B > /dev/null 2> $OUT/pw_$c.err || exit $?
done
python3 tools/pmc_to_json.py $OUT/pf_c2 $OUT/pw_c2 c2 100000000 $OUT/pmc_c2.json scan_private || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c3 $OUT/pw_c3 c3 100000000 $OUT/pmc_c3.json bq_jit_part_scatter k_part_aggregate k_part_combine bq_jit_part_first_rows || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c5 $OUT/pw_c5 c5 125000000 $OUT/pmc_c5.json bq_jit_part_scatter k_part_aggregate k_part_combine bq_jit_part_first_rows || exit $?
for c in c2 c3 c4; do echo "== $c"; python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kt_$c/kt_kernel_stats.csv')):
    print('  %-50s %6s %8.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1000))" | head -8; done
