# usage: bash tools/gpu_run.sh TAG [pytest-args...]
# The round's GPU check: every -m gpu test (full-size parity included), the default bench line
# (C2 with the CPU baselines), C3 / C4 / C5 bench lines and a rocprofv3 kernel-trace summary of
# the default bench command.  Every GPU step has its own time limit; the script stops at the
# first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  cat $OUT/bench_$c.json
done
timeout -k 10 400 python bench.py --config c5 --local-ranks 8 --steps 5 --warmup 2 > $OUT/bench_c5_8ranks.json 2> $OUT/bench_c5_8ranks.err || exit $?
cat $OUT/bench_c5_8ranks.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_c2.json 2> $OUT/prof_c2.err || exit $?
find $OUT/prof_c2 -name '*kernel_stats.csv' -exec head -6 {} \;
