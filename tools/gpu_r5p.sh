# round-5 final A: full GPU suite, smoke, default bench line (C2 + compact + c5 + CPU baseline), C3 / C4 / C4 sorted / C5 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5z}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_c2.json')); r=d['roofline']; c=d['c5'] or {}; k=d['compact'] or {}; cpu=d['cpu_baseline'] or {}
print('c2', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['frac'], 'compact', k.get('ms_per_step'), k.get('scan_kernel_ms'), k.get('build_device_ms'), 'c5', c.get('ms_per_step'), c.get('roofline_frac_of_the_shard_pass'), 'cpu', cpu.get('value'))"
for cfg in "c3" "c4" "c4 --sorted" "c5"; do
set -- $cfg
tag=$1${2:+_sorted}
timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_$tag.json')); r=d['roofline'] or {}; c=d.get('c5') or {}
print('$tag', d['value'], round(d['ms_per_step'],4), r.get('kernel_avg_ms'), r.get('frac'), c.get('scan_kernel_ms_max_over_ranks'), c.get('roofline_frac_of_the_shard_pass'))"
done
