# usage: bash tools/gpu_c4_prof.sh TAG -- C4 bench lines (random and sorted order), kernel-trace
# summary and HBM traffic (FETCH_SIZE / WRITE_SIZE passes, gfx950 correction) of the fused
# distinct pass -> profiles-ready files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-c4prof}
mkdir -p $OUT
export TMPDIR=/tmp
for v in "" "--sorted"; do
  timeout -k 10 300 python bench.py --config c4 $v --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4$v.json 2> $OUT/bench_c4$v.err || exit $?
  cat $OUT/bench_c4$v.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c4 -o kt -- python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> $OUT/kt_c4.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_c4 -o pmc -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pf_c4.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_c4 -o pmc -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pw_c4.err || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c4 $OUT/pw_c4 c4 200000000 $OUT/pmc_c4.json bq_jit_scd_fused32 || exit $?
tail -4 $OUT/pmc_c4.json
f=$(find $OUT/kt_c4 -name '*kernel_stats.csv' | head -1); head -8 "$f"
