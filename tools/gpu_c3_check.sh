set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c3flush
bash tools/micro/run_part_micro.sh 100000000 3 0 > gpurun_out/c3flush/micro.log 2>&1 || exit $?
grep -v "slot [0-9]" gpurun_out/c3flush/micro.log | head -6
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "partition or c3 or multikey" > gpurun_out/c3flush/pytest.log 2>&1 || { tail -30 gpurun_out/c3flush/pytest.log; exit 1; }
tail -2 gpurun_out/c3flush/pytest.log
for c in c3 c5; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3flush/bench_$c.json 2>gpurun_out/c3flush/bench_$c.err || exit $?; python3 -c "import json;d=json.load(open('gpurun_out/c3flush/bench_$c.json'));print('$c',d['ms_per_step'],d['roofline']['kernel_avg_ms'],d['roofline']['frac'])"; done
