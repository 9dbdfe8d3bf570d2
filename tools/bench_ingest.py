#!/usr/bin/env python3
"""Cold-path measurement (SURVEY.md §8d "cold", §8f row 1): a C2 shard on disk as a bcolz
ctable -> host blosc decode threads -> pinned double buffers -> H2D -> HBM, then the query.

Legs (best of --reps, page cache warm -- the disk itself is not measured):
  ingest_host    bqg_table_load_carray of the query's three columns, host blosc decode threads
  ingest_device  the same with the frames decoded on the GPU (decoded bytes / s)
  cold_query ctable(rootdir) + where_terms + groupby with nothing resident (ingest + query)
  warm_query the same query again (columns resident in HBM)
  host_decode_1t  the reference's own cold path shape: one thread decoding every chunk
                  (bcolz.set_nthreads(1), worker.py:40) into host memory, no query
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=100_000_000)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--threads', type=int, default=16)
    ap.add_argument('--cname', default='lz4')
    ap.add_argument('--dir', default=None, help='scratch directory for the shard (default: a temp dir)')
    ap.add_argument('--decode', default='auto', help='decoder of the cold_query leg (auto / host / device)')
    args = ap.parse_args()

    from bqueryd_amd import bcolz_io, synth
    from bqueryd_amd.ctable import ctable
    from bqueryd_amd.engine import Device, ShardTable

    cfg = synth.CONFIGS['c2']
    cols = synth.taxi_shard(args.rows, config_id=2, columns=synth.query_columns(cfg))
    nbytes = sum(a.nbytes for a in cols.values())
    scratch = tempfile.mkdtemp(prefix='bqgpu_ingest_', dir=args.dir)
    try:
        root = os.path.join(scratch, 'shard.bcolzs')
        t0 = time.perf_counter()
        bcolz_io.write_ctable(root, cols, cname=args.cname)
        write_s = time.perf_counter() - t0
        on_disk = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(root) for f in fs)
        dev = Device(0)

        def ingest(decode):
            t = ShardTable({}, device=dev, nrows=args.rows)
            t0 = time.perf_counter()
            specs = []
            for name in cols:
                meta = bcolz_io.CArrayMeta(bcolz_io.ctable_column_dir(root, name))
                t.add_column(name, meta.dtype)
                specs.append((name, meta.rootdir, meta.chunklen))
            t.load_carrays(specs, nthreads=args.threads, decode=decode)
            dev.synchronize()
            dt = time.perf_counter() - t0
            t.close()
            return dt

        def query(ct):
            t0 = time.perf_counter()
            bool_arr = ct.where_terms(cfg['where'], cache=True)
            ct.groupby(cfg['groupby'], cfg['aggs'], bool_arr=bool_arr)
            return time.perf_counter() - t0

        legs = {}
        for decode in ('host', 'device'):
            ingest(decode)  # first touch: page cache, pinned staging
            s = min(ingest(decode) for _ in range(args.reps))
            legs['ingest_' + decode] = {'s': s, 'decoded_GBps': nbytes / s / 1e9, 'rows_per_s': args.rows / s,
                                        'threads': args.threads}
            print('ingest %s: %.1f ms' % (decode, s * 1e3), file=sys.stderr, flush=True)
        cold, warm = [], []
        os.environ['BQGPU_INGEST_DECODE'] = args.decode
        for _ in range(args.reps):
            ct = ctable(rootdir=root, mode='r', auto_cache=True, device=dev)
            cold.append(query(ct))
            warm.append(query(ct))
            ct.close()
        t0 = time.perf_counter()
        for name in cols:
            bcolz_io.read_carray(bcolz_io.ctable_column_dir(root, name))
        host_1t = time.perf_counter() - t0
        line = {
            'workload': 'C2 shard cold path: %d rows, columns %s, bcolz/%s on local disk (page cache warm)'
                        % (args.rows, list(cols), args.cname),
            'decoded_bytes': nbytes, 'on_disk_bytes': on_disk, 'write_s': write_s,
            **legs,
            'cold_query': {'s': min(cold), 'rows_per_s': args.rows / min(cold), 'decode': args.decode},
            'warm_query': {'s': min(warm), 'rows_per_s': args.rows / min(warm)},
            'host_decode_1t': {'s': host_1t, 'decoded_GBps': nbytes / host_1t / 1e9,
                               'note': 'one thread, host memory only (the reference worker\'s decode shape)'},
        }
        print(json.dumps(line), flush=True)
    finally:
        shutil.rmtree(scratch, ignore_errors=True)


if __name__ == '__main__':
    main()
