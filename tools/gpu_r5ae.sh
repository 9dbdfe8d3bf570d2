#!/bin/bash
# per-slot fixed-point shifts: the fixed-point tests, then the float-sum / moments subset
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "fixed_point or float_sums or moments or nonfinite or fuzz" > gpurun_out/r5ae_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5ae_tests.log; exit $rc
