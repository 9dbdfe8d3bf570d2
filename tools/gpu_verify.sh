# usage: bash tools/gpu_verify.sh TAG -- GPU parity tests, then C2..C5 bench lines + C2 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-verify}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -q -m gpu -rf -x --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_c2.json 2> $OUT/prof_c2.err || exit $?
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  cat $OUT/bench_$c.json
done
