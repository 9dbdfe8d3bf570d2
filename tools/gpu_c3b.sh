# usage: bash tools/gpu_c3b.sh TAG -- C3 SQ/LDS PMC pass, nt-store scatter variant vs default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in default BQ_NT_STORE; do
  if [ $v = default ]; then unset BQGPU_JIT_DEFS; else export BQGPU_JIT_DEFS=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o kt -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit $?
  echo $v; cut -d, -f1-4 $OUT/kt_$v/kt_kernel_stats.csv | head -4
done
unset BQGPU_JIT_DEFS
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o pmc -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_sq.err || exit $?
python3 tools/pmc_any.py $OUT/pmc_sq > $OUT/pmc_sq.txt
grep -A 10 "part_aggregate\|part_scatter" $OUT/pmc_sq.txt
