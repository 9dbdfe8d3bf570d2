# usage: bash tools/gpu_measure_a.sh TAG -- GPU tests, then C2 and C3: bench line, kernel trace,
# FETCH_SIZE / WRITE_SIZE passes (separate runs) -> profiles/pmc_<cfg>.json inputs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ma}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
for c in c2 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$c -o kt -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_$c.json 2> $OUT/kt_$c.err || exit $?
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pf_$c.err || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pw_$c.err || exit $?
done
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
cat $OUT/bench_c3.json
