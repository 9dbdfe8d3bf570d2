# usage: bash tools/gpu_measure_b.sh TAG -- C4 (bench, trace, PMC), C5 bench, torchrun N=1,
# C1 end-to-end and the cold-path ingest measurement
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-mb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
c=c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$c -o kt -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_$c.json 2> $OUT/kt_$c.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pf_$c.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pw_$c.err || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
cat $OUT/bench_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c5 -o kt -- python3 bench.py --config c5 --steps 5 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
cat $OUT/bench_c5.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c2_torchrun.json 2> $OUT/bench_c2_torchrun.err || exit $?
cat $OUT/bench_c2_torchrun.json
timeout -k 10 400 python tools/bench_e2e.py --reps 3 > $OUT/e2e_c1.json 2> $OUT/e2e_c1.err || exit $?
cat $OUT/e2e_c1.json
timeout -k 10 400 python tools/bench_ingest.py --reps 3 > $OUT/ingest_c2.json 2> $OUT/ingest_c2.err || exit $?
cat $OUT/ingest_c2.json
