# usage: bash tools/gpu_c4_check.sh TAG -- distinct-pass GPU tests, then C4 bench lines (random and sorted order)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-c4check}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_limits.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c4 or distinct or scd" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in "" "--sorted"; do
  timeout -k 10 300 python bench.py --config c4 $v --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4$v.json 2> $OUT/bench_c4$v.err || exit $?
  python3 -c "import json;d=json.load(open('$OUT/bench_c4$v.json'));print('c4$v',d['ms_per_step'],d['roofline']['kernel_avg_ms'],d['roofline']['frac'])"
done
