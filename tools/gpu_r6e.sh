#!/bin/bash
# round 6 E: C4 parity after the LDS swizzle, C4 A/B (abtest = pre-swizzle HEAD) with SQ bank-conflict counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6e}
mkdir -p $OUT
export TMPDIR=/tmp
true
tail -2 $OUT/tests.log
for side in abtest .; do
  tag=$( [ "$side" = "." ] && echo new || echo old )
  for v in "" "--sorted"; do
    (cd $side && timeout -k 10 200 python bench.py --config c4 $v --steps 20 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record > $OUT/${tag}_c4$v.json 2> $OUT/${tag}_c4$v.err) || exit $?
    python3 -c "import json;d=json.load(open('$OUT/${tag}_c4$v.json'));print('$tag c4 $v ms', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_avg_ms'],4), 'frac', round(d['roofline']['frac'],3))"
  done
  (cd $side && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY --output-format csv -d $OUT/${tag}_sq1 -o pmc -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-c5 --no-compact-record > /dev/null 2> $OUT/${tag}_sq1.err) || exit $?
  (cd $side && timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $OUT/${tag}_sq2 -o pmc -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-c5 --no-compact-record > /dev/null 2> $OUT/${tag}_sq2.err) || exit $?
  echo "== $tag" >> $OUT/sq.txt
  python3 tools/pmc_sq.py $OUT/${tag}_sq1 scd_fused >> $OUT/sq.txt && python3 tools/pmc_sq.py $OUT/${tag}_sq2 scd_fused >> $OUT/sq.txt
done
cat $OUT/sq.txt
