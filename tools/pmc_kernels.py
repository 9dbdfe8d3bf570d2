#!/usr/bin/env python3
"""Per-kernel average FETCH_SIZE / WRITE_SIZE from two rocprofv3 --pmc output directories.

usage: pmc_kernels.py FETCH_DIR WRITE_DIR
Prints one line per kernel: launches, FETCH_SIZE KiB, 2x FETCH bytes (gfx950 wide-stream
correction, MI355X_MICROARCH.md §HBM), WRITE bytes.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def collect(d, counter):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get('Counter_Name') == counter:
                acc[r['Kernel_Name'][:90]].append(float(r['Counter_Value']))
    return acc


f = collect(sys.argv[1], 'FETCH_SIZE')
w = collect(sys.argv[2], 'WRITE_SIZE')
print('%-90s %6s %14s %14s' % ('kernel', 'n', 'read_MB(2xF)', 'write_MB'))
for k in sorted(set(f) | set(w)):
    fv, wv = f.get(k, [0]), w.get(k, [0])
    print('%-90s %6d %14.2f %14.2f' % (k, len(fv), 2 * sum(fv) / len(fv) * 1024 / 1e6, sum(wv) / len(wv) * 1024 / 1e6))
