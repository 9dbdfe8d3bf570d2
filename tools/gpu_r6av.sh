#!/bin/bash
# round 6 AV: device-table results through one copy kernel: the whole GPU suite, smoke, C5 / C3 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6av}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
for c in c5 c3; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-compact-record --no-cold-record > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_$c.json')); r=d.get('roofline') or {}; c5=d.get('c5') or {}
print('$c', round(d['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in r.items() if 'ms' in k or k == 'frac'}, 'c5 sub', c5.get('ms_per_step'), c5.get('shard_pass_ms_max_over_ranks'), c5.get('merge_ms_max_over_ranks'))"
done
