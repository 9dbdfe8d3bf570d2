#!/bin/bash
# round 6 G: the shared-host merge (bqg_merge_shared_host) at world 1-4 on one GPU, bench c5 with it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6g}
mkdir -p $OUT
export TMPDIR=/tmp
df -h /dev/shm | tail -1
for w in 1 2 4; do
BQGPU_DIST_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2953$w tools/dist_check.py > $OUT/dist$w.log 2>&1 || { tail -30 $OUT/dist$w.log; exit 1; }
grep dist_check $OUT/dist$w.log
done
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > $OUT/bench_c5_w1.json 2> $OUT/bench_c5_w1.err || { tail -30 $OUT/bench_c5_w1.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c5_w1.json'));c=d['c5'];print('c5 world 1', {k: c.get(k) for k in ('value','ms_per_step','shard_pass_ms_max_over_ranks','merge_ms_max_over_ranks','merged_rows','merged_row_count_check','error')})"
for w in 2 4; do
BQGPU_BENCH_DEVICE=0 BQGPU_BENCH_ONE_GPU_RCCL=1 timeout -k 10 400 python bench.py --gpus $w --config c5 --steps 5 --warmup 2 > $OUT/bench_c5_w$w.json 2> $OUT/bench_c5_w$w.err || { tail -30 $OUT/bench_c5_w$w.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c5_w$w.json'));c=d['c5'];print('c5 world $w', {k: c.get(k) for k in ('value','ms_per_step','merge_ms_max_over_ranks','merged_rows','merged_row_count_check','error')})"
done
