# round-5 refresh of the round-4-only lines: C5 full shape on one GPU (8 in-process ranks), C3 wide-span fares, message-level C3 / C1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5y}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config c5 --local-ranks 8 --steps 5 --warmup 2 > $OUT/bench_c5_8ranks.json 2> $OUT/bench_c5_8ranks.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_c5_8ranks.json')); c=d['config']; p=c['projected_node']
print('c5 8 ranks', d['value'], d['ms_per_step'], 'proj', p['ms_per_step'], p['x_over_one_gpu'], 'merge crit', c['merge_ms_critical_path'], 'frac', d['roofline']['frac'])"
timeout -k 10 200 python bench.py --config c3 --variant wide --steps 10 --warmup 3 --no-cpu-baseline --no-c5 > $OUT/bench_c3_wide.json 2> $OUT/bench_c3_wide.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_c3_wide.json')); r=d['roofline']
print('c3 wide', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['frac'])"
timeout -k 10 300 python tools/bench_e2e.py --config c3 > $OUT/e2e_c3.json 2> $OUT/e2e_c3.err || exit $?
tail -c 600 $OUT/e2e_c3.json
timeout -k 10 300 python tools/bench_e2e.py --config c1 > $OUT/e2e_c1.json 2> $OUT/e2e_c1.err || exit $?
tail -c 600 $OUT/e2e_c1.json
