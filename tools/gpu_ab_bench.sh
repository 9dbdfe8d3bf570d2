# usage: bash tools/gpu_ab_bench.sh TAG CONFIG [bench args...] -- the same bench line from the
# committed tree (abtest/, a git worktree built in-tree) and the working tree, alternated on
# one box: A/B of a kernel change without box-to-box spread.  Set up on the CPU side first:
#   git worktree add abtest <baseline rev> && make -C abtest/bqueryd_amd/csrc
# (abtest/ is git-ignored; remove it with `git worktree remove --force abtest` afterwards)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}; shift
CFG=$1; shift
mkdir -p $OUT
for r in 1 2; do
  for side in abtest .; do
    tag=$( [ "$side" = "." ] && echo new || echo old )
    (cd $side && timeout -k 10 300 python bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline "$@" > $OUT/${tag}_$r.json 2> $OUT/${tag}_$r.err) || exit $?
    python3 -c "import json;d=json.load(open('$OUT/${tag}_$r.json'));print('$tag', '$CFG $*', 'ms', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_avg_ms'],4), 'frac', round(d['roofline']['frac'],3))"
  done
done
