#!/usr/bin/env python3
"""Device-decode ingest of a C2 shard's three columns, for rocprofv3 kernel timing and a
host-side phase breakdown (usage: python tools/prof_blosc.py [--rows N] [--reps R])."""
import argparse
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=100_000_000)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--cname', default='lz4')
    ap.add_argument('--decode', default='device')
    args = ap.parse_args()
    from bqueryd_amd import bcolz_io, synth
    from bqueryd_amd.engine import Device, ShardTable
    cfg = synth.CONFIGS['c2']
    cols = synth.taxi_shard(args.rows, config_id=2, columns=synth.query_columns(cfg))
    scratch = tempfile.mkdtemp(prefix='bqgpu_blosc_')
    try:
        root = os.path.join(scratch, 'shard.bcolzs')
        bcolz_io.write_ctable(root, cols, cname=args.cname)
        dev = Device(0)
        for r in range(args.reps + 1):
            t = ShardTable({}, device=dev, nrows=args.rows)
            for name in cols:
                meta = bcolz_io.CArrayMeta(bcolz_io.ctable_column_dir(root, name))
                t.add_column(name, meta.dtype)
                t0 = time.perf_counter()
                rep = t.load_carray(name, meta.rootdir, meta.chunklen, nthreads=16, decode=args.decode)
                dt = time.perf_counter() - t0
                print('rep %d %s: %.2f ms, %s' % (r, name, dt * 1e3, rep), flush=True)
            t.close()
    finally:
        shutil.rmtree(scratch, ignore_errors=True)


if __name__ == '__main__':
    main()
