#!/bin/bash
# round 6 Y: C3 partition shape sweep with the streaming-store scatter (engine options through BQGPU_OPTIONS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6y}
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for o in "" "part_wbits=12,part_splits=1" "part_wbits=12,part_splits=2" "part_win=2048" "part_k=1"; do
tag=$(echo "x$o" | tr ',=' '__')
BQGPU_OPTIONS="$o" timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record --no-cold-record > $OUT/$tag.$r.json 2> $OUT/$tag.$r.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/$tag.$r.json'));r=d['roofline'];print('%-32s' % '$o', 'ms', round(d['ms_per_step'],4), 'kernels', round(r['kernel_avg_ms'],4), 'frac', round(r['frac'],4))"
done
done
