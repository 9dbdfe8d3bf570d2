set -o pipefail
cd "$GRAFT_REPO_ROOT"
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
if [ $rc -le 1 ]; then
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b1.json 2> gpurun_out/b1.err
  echo "bench rc=$?" >> gpurun_out/b1.err
fi
