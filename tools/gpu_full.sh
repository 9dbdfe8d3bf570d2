# usage: bash tools/gpu_full.sh TAG
# GPU tests, C2 bench + kernel trace, PMC traffic passes (FETCH_SIZE / WRITE_SIZE separately,
# per MI355X_MICROARCH.md), and C3/C4 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -rf > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err || exit $?
for c in c3 c4; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  cat $OUT/bench_$c.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o kt -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/prof_$c.err || exit $?
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_torchrun.json 2> $OUT/bench_torchrun.err || exit $?
cat $OUT/bench_torchrun.json
