#!/bin/bash
# round 6 Q: final check at HEAD -- the whole GPU suite, smoke, the default bench line and C3 / C4 / C5 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 500 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
for c in c3 c4; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
done
python3 - <<PY
import json
for c in ['c2','c3','c4']:
    d=json.load(open('$OUT/bench_%s.json' % c)); r=d.get('roofline') or {}
    print(c, '%.3e rows/s' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel %.4f' % r.get('kernel_avg_ms'), 'frac %.3f' % r.get('frac'), 'whole-query frac %s' % r.get('frac_whole_query_incl_result_copy'), 'cold %s' % d.get('cold_first_query_ms'))
d=json.load(open('$OUT/bench_c2.json'))
print('c5 sub', {k: d['c5'].get(k) for k in ('value','ms_per_step','merge_ms_max_over_ranks','roofline_frac_of_the_shard_pass','error')})
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
PY
