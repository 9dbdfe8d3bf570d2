#!/bin/bash
# round 6 AA: the slot emit (no compaction, no host round trip before the large-result emit):
# its parity tests, the GPU parity suite, then the C3 step timeline and C3 / C5 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6aa}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "slot_emit or remaining_engine_options or std" > $OUT/pytest_slot.txt 2>&1 || { tail -30 $OUT/pytest_slot.txt; exit 1; }
tail -3 $OUT/pytest_slot.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -m gpu > $OUT/pytest_parity.txt 2>&1 || { tail -30 $OUT/pytest_parity.txt; exit 1; }
tail -3 $OUT/pytest_parity.txt
for se in 1 2 0; do
BQGPU_OPTIONS="slot_emit=$se" timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-compact-record --no-cold-record > $OUT/c3_se$se.json 2> $OUT/c3_se$se.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_se$se.json'));r=d['roofline'];c=d.get('c5') or {};print('slot_emit=$se C3 ms', round(d['ms_per_step'],4), 'kernels', round(r['kernel_avg_ms'],4), 'frac', round(r['frac'],4), 'C5 ms', c.get('ms_per_step'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $OUT/tl -o tl --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/tl_bench.json 2> $OUT/tl_bench.err || exit $?
python3 tools/step_timeline.py $OUT/tl bq_jit_part_scatter > $OUT/timeline.txt
