#!/bin/bash
# round 6 AE: SQ counters of the large-result emit kernels (C3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6ae}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d $OUT/sq -o sq --output-format csv -- $B > /dev/null 2> $OUT/sq.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/sq2 -o sq2 --output-format csv -- $B > /dev/null 2> $OUT/sq2.err || exit 1
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for d in ('sq', 'sq2'):
    f = glob.glob(out + '/' + d + '/**/*counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if not any(k in n for k in ('k_rank_emit_slots', 'k_setbits_slots', 'k_word_scan_pairs', 'k_part_combine')):
            continue
        agg[n[:40]][r['Counter_Name']].append(float(r['Counter_Value']))
    for n, cs in agg.items():
        print(d, n, {c: round(sum(v) / len(v), 1) for c, v in cs.items()})
PY
