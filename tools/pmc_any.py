#!/usr/bin/env python3
"""Per-kernel averages of every counter in one or more rocprofv3 --pmc output directories.

usage: pmc_any.py DIR [DIR ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(path)):
            acc[r['Kernel_Name'][:60]][r['Counter_Name']].append(float(r['Counter_Value']))
for k in sorted(acc):
    cs = acc[k]
    print(k)
    for c in sorted(cs):
        v = cs[c]
        print('    %-28s n=%-4d avg=%.6g' % (c, len(v), sum(v) / len(v)))
