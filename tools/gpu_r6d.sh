#!/bin/bash
# round 6 D: RCCL at world 2 on one GPU (socket transport between two "hosts")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6d}
mkdir -p $OUT
export TMPDIR=/tmp
export BQGPU_DIST_ONE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 tools/dist_check.py > $OUT/dist2.log 2>&1; rc=$?
grep -E "dist_check|Error|error|Duplicate" $OUT/dist2.log | head -20
tail -5 $OUT/dist2.log
exit $rc
