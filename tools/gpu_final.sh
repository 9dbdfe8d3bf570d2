# usage: bash tools/gpu_final.sh TAG -- round profiles: PMC traffic for C3/C5, kernel traces and
# bench lines for C2 (default command, with the CPU baseline), C4, C5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in c3 c5; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pf_$c.err || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pw_$c.err || exit $?
done
python3 tools/pmc_to_json.py $OUT/pf_c3 $OUT/pw_c3 c3 100000000 $OUT/pmc_c3.json bq_jit_part_count bq_jit_part_scatter k_part_aggregate || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c5 $OUT/pw_c5 c5 125000000 $OUT/pmc_c5.json bq_jit_part_count bq_jit_part_scatter k_part_aggregate || exit $?
for c in c2 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$c -o kt -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_$c.json 2> $OUT/kt_$c.err || exit $?
done
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
cat $OUT/bench_c4.json
