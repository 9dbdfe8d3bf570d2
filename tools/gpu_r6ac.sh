#!/bin/bash
# round 6 AC: what bounds the slot emit (temporary probes: no rank lookup / slot-order writes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6ac}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o kt --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/$tag.json 2> $OUT/$tag.err || return 1
  python3 - $OUT/$tag $tag <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('emit', 'aos', 'setbits', 'compact', 'scan_seg', 'word_scan', 'block_scan')):
        print('%-10s %-50s %8.1f us' % (sys.argv[2], r['Name'][:50], float(r['AverageNs']) / 1e3))
PY
}
run base BQGPU_OPTIONS=slot_emit=1 && run p1_nolookup BQG_EMIT_PROBE=1 && run p2_nostore BQG_EMIT_PROBE=2 && run p3_nobits BQG_EMIT_PROBE=3 && run k8 BQG_EMIT_PROBE=8 && run k1 BQG_EMIT_PROBE=9
