# usage: bash tools/micro/pmc_part_micro.sh -- PMC passes (FETCH/WRITE bytes, SQ instruction mix) over the partition micro-benchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/micro_pmc
mkdir -p $OUT
export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I bqueryd_amd/csrc -I include tools/micro/part_micro.hip -o $OUT/part_micro || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- $OUT/part_micro 100000000 1 0 > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- $OUT/part_micro 100000000 1 0 > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY -d $OUT/sq -o pmc --output-format csv -- $OUT/part_micro 100000000 1 0 > $OUT/sq.log 2>&1 || exit $?
python3 tools/pmc_sq.py $OUT/fetch
python3 tools/pmc_sq.py $OUT/write
python3 tools/pmc_sq.py $OUT/sq
