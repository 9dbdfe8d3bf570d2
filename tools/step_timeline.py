#!/usr/bin/env python3
"""The last timed steps of a rocprofv3 --kernel-trace --hip-trace [--memory-copy-trace] run, as a
timeline: every kernel and copy (start / end) and every HIP API call between the step's first
launch and the next step's first launch, in microseconds from the step start.
usage: step_timeline.py DIR [ANCHOR]  (ANCHOR: a substring of the step's first kernel's name,
default bq_jit_scan_private -- C2; bq_jit_part_scatter for C3)"""
import csv
import glob
import os
import sys

d = sys.argv[1]
kfile = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)[0]
hfile = glob.glob(os.path.join(d, '**', '*hip_api_trace.csv'), recursive=True)[0]
ks = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:40]) for r in csv.DictReader(open(kfile))]
hs = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in csv.DictReader(open(hfile))]
cfile = glob.glob(os.path.join(d, '**', '*memory_copy_trace.csv'), recursive=True)
if cfile:
    ks += [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'COPY ' + r.get('Direction', '')) for r in csv.DictReader(open(cfile[0]))]
ks.sort()
hs.sort()
anchor = sys.argv[2] if len(sys.argv) > 2 else 'bq_jit_scan_private'
scans = [k for k in ks if anchor in k[2]]
print('scan launches', len(scans))
for i in range(len(scans) - 4, len(scans) - 1):
    t0, t1 = scans[i][0], scans[i + 1][0]
    print('--- step: scan start -> next scan start %.1f us' % ((t1 - t0) / 1e3))
    ev = [(k[0], 'K+', k[2]) for k in ks if t0 <= k[0] < t1] + [(k[1], 'K-', k[2]) for k in ks if t0 <= k[1] < t1]
    ev += [(h[0], 'A+', h[2]) for h in hs if t0 - 50000 <= h[0] < t1 and (h[1] - h[0]) > 500 or (t0 <= h[0] < t1)]
    for t, kind, name in sorted(ev):
        if t < t0 - 50000:
            continue
        print('  %9.1f %s %s' % ((t - t0) / 1e3, kind, name))
    print('  api calls in the step:')
    agg = {}
    for h in hs:
        if t0 <= h[0] < t1:
            a = agg.setdefault(h[2], [0, 0.0])
            a[0] += 1
            a[1] += (h[1] - h[0]) / 1e3
    for n, (c, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print('    %-40s %3d calls %8.1f us' % (n, c, us))
