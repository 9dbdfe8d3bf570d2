# usage: bash tools/gpu_c3_sq.sh TAG -- SQ instruction-mix / wait counters of the C3 partition kernels (two PMC passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-c3sq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY --output-format csv -d $OUT/sq1 -o pmc -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-c5 --no-compact-record > /dev/null 2> $OUT/sq1.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $OUT/sq2 -o pmc -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-c5 --no-compact-record > /dev/null 2> $OUT/sq2.err || exit $?
python3 tools/pmc_sq.py $OUT/sq1 part_ > $OUT/sq.txt && python3 tools/pmc_sq.py $OUT/sq2 part_ >> $OUT/sq.txt && cat $OUT/sq.txt
