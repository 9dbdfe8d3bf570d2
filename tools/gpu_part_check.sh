cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/part
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "partition" -x -q --timeout 120 --timeout-method thread > gpurun_out/part/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/part/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/part/bench_c3.json 2> gpurun_out/part/bench_c3.err || exit $?
cat gpurun_out/part/bench_c3.json
