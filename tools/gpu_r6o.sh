#!/bin/bash
# round 6 O: cold first query of C3 / C4 (where it goes: kernel trace of a fresh process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6o}
mkdir -p $OUT
export TMPDIR=/tmp
for c in c3 c4; do
timeout -k 10 200 python tools/cold_probe.py $c > $OUT/cold_$c.json 2> $OUT/cold_$c.err || { tail -20 $OUT/cold_$c.err; exit 1; }
cat $OUT/cold_$c.json; echo
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/tr_$c -o tr -- python3 tools/cold_probe.py $c > /dev/null 2> $OUT/tr_$c.err || exit $?
done
python3 - <<PY
import csv, glob
for c in ['c3', 'c4']:
    d = '$OUT/tr_%s' % c
    h = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in csv.DictReader(open(glob.glob(d + '/**/*hip_api_trace.csv', recursive=True)[0]))]
    k = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:50]) for r in csv.DictReader(open(glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0]))]
    h.sort(); k.sort()
    print('==', c, 'longest API calls:')
    for s, e, f in sorted(h, key=lambda x: x[1] - x[0], reverse=True)[:12]:
        print('   %-30s %9.1f us' % (f, (e - s) / 1e3))
    print('   longest kernels:')
    for s, e, f in sorted(k, key=lambda x: x[1] - x[0], reverse=True)[:8]:
        print('   %-50s %9.1f us' % (f, (e - s) / 1e3))
PY
