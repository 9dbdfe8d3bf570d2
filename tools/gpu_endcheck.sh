# usage: bash tools/gpu_endcheck.sh TAG -- the driver's round-end sequence: GPU suite, smoke,
# default bench line; plus the host-overhead breakdown and a C2 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-round_end}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -q -m gpu -rf -x --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
timeout -k 10 200 python tools/host_overhead.py > $OUT/host_overhead.txt 2>&1 || exit $?
cat $OUT/host_overhead.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c2 -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/kt_c2.json 2> $OUT/kt_c2.err || exit $?
head -3 $OUT/kt_c2/kt_kernel_stats.csv | cut -c1-120
