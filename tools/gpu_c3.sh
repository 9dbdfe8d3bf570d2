# usage: bash tools/gpu_c3.sh TAG -- partition parity tests, C3 bench, C3 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -rf -x -k "part or c3 or merge or limits or dist" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o kt -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_c3.json 2> $OUT/prof_c3.err || exit $?
cut -d, -f1-4 $OUT/prof_c3/kt_kernel_stats.csv | head -5
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
cat $OUT/bench_c3.json
