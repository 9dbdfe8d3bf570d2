# usage: bash tools/gpu_c3d.sh TAG -- partition parity tests, C3 bench + kernel trace, C5 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -rf -x -k "part or c3 or merge or limits or colocated" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3 -o kt -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_c3.json 2> $OUT/kt_c3.err || exit $?
head -4 $OUT/kt_c3/kt_kernel_stats.csv | cut -c1-110
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
done
