#!/usr/bin/env python3
"""HBM bytes per launch of a config's dominant kernel(s) from two rocprofv3 --pmc passes.

usage: pmc_to_json.py FETCH_DIR WRITE_DIR CONFIG ROWS OUT.json KERNEL_SUBSTR [KERNEL_SUBSTR ...]

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half the bytes of a
wide coalesced streaming read, so hbm_read = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for
16-byte streaming stores.  Several kernel substrings (C3: count + scatter + aggregate) are
summed: the bench times them together as one "launch".
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, counter, kernel):
    vals = []
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel in r['Kernel_Name'] and r['Counter_Name'] == counter:
                vals.append(float(r['Counter_Value']))
    if not vals:
        raise SystemExit('no %s samples for %s in %s' % (counter, kernel, d))
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, config, rows, out = sys.argv[1:6]
    kernels = sys.argv[6:]
    read = write = 0.0
    detail = {}
    for k in kernels:
        f, nf = per_launch(fdir, 'FETCH_SIZE', k)
        w, nw = per_launch(wdir, 'WRITE_SIZE', k)
        detail[k] = {'fetch_size_kib': f, 'write_size_kib': w, 'samples': [nf, nw],
                     'hbm_read_bytes': 2 * f * 1024, 'hbm_write_bytes': w * 1024}
        read += 2 * f * 1024
        write += w * 1024
    d = {'config': config, 'rows': int(rows), 'kernels': kernels, 'per_kernel': detail,
         'correction': 'hbm_read = 2 x FETCH_SIZE (gfx950 wide-stream under-count), WRITE_SIZE as is',
         'hbm_read_bytes_per_launch': int(round(read)), 'hbm_write_bytes_per_launch': int(round(write)),
         'hbm_bytes_per_launch': int(round(read + write))}
    with open(out, 'w') as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d))


if __name__ == '__main__':
    main()
