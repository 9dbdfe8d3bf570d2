#!/usr/bin/env python3
"""Per-kernel average of every counter in one rocprofv3 --pmc output directory.

usage: pmc_sq.py DIR [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(sys.argv[1], '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(path)):
        acc[r['Kernel_Name'][:70]][r['Counter_Name']].append(float(r['Counter_Value']))
want = sys.argv[2] if len(sys.argv) > 2 else ''
for k, cs in sorted(acc.items()):
    if want not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print('   %-28s n=%3d avg %.4g' % (c, len(v), sum(v) / len(v)))
