# usage: bash tools/gpu_prof.sh TAG CONFIG [extra bench args]
# kernel trace + FETCH_SIZE / WRITE_SIZE PMC passes of one bench config (separate runs, per
# MI355X_MICROARCH.md: FETCH_SIZE x2 on gfx950 for wide streaming reads)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-prof}; CFG=${2:-c3}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || exit $?
cat $OUT/bench_$CFG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$CFG -o kt -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> $OUT/kt_$CFG.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$CFG -o pmc -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> $OUT/pf_$CFG.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$CFG -o pmc -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> $OUT/pw_$CFG.err || exit $?
python3 tools/pmc_kernels.py $OUT/pf_$CFG $OUT/pw_$CFG > $OUT/pmc_$CFG.txt 2>&1 || true
cat $OUT/pmc_$CFG.txt
