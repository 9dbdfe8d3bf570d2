#!/bin/bash
# C3 aggregate sensitivity: the packed aggregate without its LDS atomics (exp1) / with the add only (exp2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5aj}
mkdir -p $OUT
export TMPDIR=/tmp
cp bqueryd_amd/libbqgpu.so /tmp/lib_main.so
i=0
for v in main exp1 exp2; do
i=$((i+1))
if [ $v = main ]; then cp /tmp/lib_main.so bqueryd_amd/libbqgpu.so; else cp bqueryd_amd/libbqgpu_$v.so bqueryd_amd/libbqgpu.so; fi
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$i -o kt -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-compact-record > $OUT/kt$i.json 2> $OUT/kt$i.err || exit $?
echo "== $v"; python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kt$i/kt_kernel_stats.csv')):
    if 'aggregate' in r['Name']:
        print('  %-40s %8.1f us' % (r['Name'][:40], float(r['AverageNs'])/1000))"
done
cp /tmp/lib_main.so bqueryd_amd/libbqgpu.so
