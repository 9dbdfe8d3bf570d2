#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -m gpu > gpurun_out/r5ag_fuzz.log 2>&1
rc=$?; tail -3 gpurun_out/r5ag_fuzz.log; exit $rc
