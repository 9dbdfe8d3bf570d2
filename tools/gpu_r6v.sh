#!/bin/bash
# round 6 V: A/B of a scatter change (abtest = HEAD worktree, . = working tree): C3 and C5 lines, alternated on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6v}
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for side in abtest .; do
    tag=$( [ "$side" = "." ] && echo new || echo old )
    for c in c3 c5; do
      (cd $side && timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/${tag}_${c}_$r.json 2> $OUT/${tag}_${c}_$r.err) || exit $?
      python3 -c "import json;d=json.load(open('$OUT/${tag}_${c}_$r.json'));r=d.get('roofline') or {};c5=d.get('c5') or {};print('$tag $c', 'ms', round(d['ms_per_step'],4), 'kernel', r.get('kernel_avg_ms') or c5.get('scan_kernel_ms_max_over_ranks'), 'frac', r.get('frac') or c5.get('roofline_frac_of_the_shard_pass'))"
    done
  done
done
