# usage: bash tools/gpu_c5.sh TAG -- merge/dist parity tests, C5 bench fused vs per-shard
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -rf -x -k "merge or colocated or dist" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
cat $OUT/bench_c5.json
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --c5-per-shard > $OUT/bench_c5_per_shard.json 2> $OUT/bench_c5_per_shard.err || exit $?
cat $OUT/bench_c5_per_shard.json
