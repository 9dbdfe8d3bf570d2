#!/bin/bash
# round 6 AH: the epoch row map + two-slot emit: parity (slot emit tests, then the parity and
# full-size suites), C3 lines per slot_emit value, and the default's kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6ai}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "slot_emit or remaining_engine_options or row_map" > $OUT/pytest_slot.txt 2>&1 || { tail -30 $OUT/pytest_slot.txt; exit 1; }
tail -2 $OUT/pytest_slot.txt
true
true
for se in 1; do
BQGPU_OPTIONS="slot_emit=$se" timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-compact-record --no-cold-record > $OUT/c3_se$se.json 2> $OUT/c3_se$se.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_se$se.json'));r=d['roofline'];c=d.get('c5') or {};print('slot_emit=$se C3 ms', round(d['ms_per_step'],4), 'device', round(r['device_ms_per_query'],4), 'kernels', round(r['kernel_avg_ms'],4), 'frac', round(r['frac'],4), 'C5 ms', c.get('ms_per_step'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/kt.json 2> $OUT/kt.err || exit $?
python3 - $OUT/kt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print('%-60s %5s %9.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
