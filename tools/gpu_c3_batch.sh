# usage: bash tools/gpu_c3_batch.sh TAG -- C3 step time vs partition row batch (Infinity Cache residency)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-c3batch}
mkdir -p $OUT
for b in 0 4194304 8388608 16777216 33554432; do
  if [ $b -eq 0 ]; then unset BQGPU_PART_BATCH; else export BQGPU_PART_BATCH=$b; fi
  timeout -k 10 200 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3_$b.json 2> $OUT/c3_$b.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$OUT/c3_$b.json')); print($b, 'ms/step %.3f kernel %.3f frac %.3f' % (d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac']))"
done
export BQGPU_PART_BATCH=8388608
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k c3 -x -q --timeout 240 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
