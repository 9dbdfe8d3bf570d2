# usage: bash tools/gpu_c4sweep.sh TAG -- distinct-pass parity with the peel variant, C4 variant
# sweep, C5 PMC traffic + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c4sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BQGPU_JIT_DEFS=BQ_SCD_PEEL=2 timeout -k 10 400 python -u -m pytest tests -q -m gpu -rf -x -k "distinct or scd or jit or c4" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/c4_sweep.py > $OUT/sweep.txt 2> $OUT/sweep.err || exit $?
cat $OUT/sweep.txt
c=c5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pf_$c.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$c -o pmc -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pw_$c.err || exit $?
python3 tools/pmc_to_json.py $OUT/pf_c5 $OUT/pw_c5 c5 125000000 $OUT/pmc_c5.json bq_jit_part_count bq_jit_part_scatter k_part_aggregate > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c5 -o kt -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_c5.json 2> $OUT/kt_c5.err || exit $?
head -4 $OUT/kt_c5/kt_kernel_stats.csv | cut -c1-120
