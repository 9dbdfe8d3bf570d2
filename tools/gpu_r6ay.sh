#!/bin/bash
# round 6 AY: the shared-host merge slices written by one kernel: merge / dist tests, C5 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6ay}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_merge.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -k "merge or dist or c5" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for r in 1 2; do
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-compact-record --no-cold-record > $OUT/bench_c5_$r.json 2> $OUT/bench_c5_$r.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_c5_$r.json')); c5=d.get('c5') or {}
print('c5', round(d['ms_per_step'],4), 'shard pass', c5.get('shard_pass_ms_max_over_ranks'), 'merge', c5.get('merge_ms_max_over_ranks'), 'rows ok', c5.get('merged_row_count_check'))"
done
