# usage: bash tools/gpu_c3_prof.sh TAG -- C3 and C5 bench lines, kernel-trace summary and HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes, gfx950 correction) of the partitioned path -> profiles-ready files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  cat $OUT/bench_$c.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3 -o kt -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> $OUT/kt_c3.err || exit $?
for c in c3 c5; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pf_$c.err || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pw_$c.err || exit $?
done
python3 tools/pmc_to_json.py $OUT/pf_c3 $OUT/pw_c3 c3 100000000 $OUT/pmc_c3.json bq_jit_part_scatter k_part_aggregate k_part_combine bq_jit_part_first_rows || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c5 $OUT/pw_c5 c5 125000000 $OUT/pmc_c5.json bq_jit_part_scatter k_part_aggregate k_part_combine bq_jit_part_first_rows || exit $?
cat $OUT/pmc_c3.json | tail -4
f=$(find $OUT/kt_c3 -name '*kernel_stats.csv' | head -1); head -8 "$f"
