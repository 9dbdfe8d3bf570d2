# usage: bash tools/gpu_c5e2e.sh TAG -- C5 (multi-shard + merge) bench and C1 end-to-end legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e.py -q -m gpu -x -k "distinct or c4 or golden" > $OUT/pytest_k.log 2>&1 || { tail -30 $OUT/pytest_k.log; exit 1; }
tail -2 $OUT/pytest_k.log
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
cat $OUT/bench_c4.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o kt -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/prof_c4.err || exit $?
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
cat $OUT/bench_c5.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --config c5 --steps 5 --warmup 2 > $OUT/bench_c5_torchrun.json 2> $OUT/bench_c5_torchrun.err || exit $?
cat $OUT/bench_c5_torchrun.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o kt -- python3 bench.py --config c5 --steps 3 --warmup 1 > /dev/null 2> $OUT/prof_c5.err || exit $?
timeout -k 10 400 python tools/bench_e2e.py --reps 5 > $OUT/e2e_c1.json 2> $OUT/e2e_c1.err || exit $?
cat $OUT/e2e_c1.json
