"""Per-query host overhead of the C2 step on the GPU box: wall time of the Python call, of
the bare C-ABI call with a prebuilt query, and the device time the library reports.

    python tools/host_overhead.py [--rows N] [--reps R]
"""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from bqueryd_amd import synth, _lib as L  # noqa: E402
from bqueryd_amd.engine import Device, ShardTable, parse_agg_list  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=100_000_000)
    ap.add_argument('--reps', type=int, default=200)
    ap.add_argument('--config', default='c2')
    a = ap.parse_args()
    cfg = synth.CONFIGS[a.config]
    cols = synth.taxi_shard(a.rows, config_id=synth.CONFIG_ID[a.config], columns=synth.query_columns(cfg))
    dev = Device(0)
    t = ShardTable(cols, device=dev)
    for _ in range(5):
        t.groupby(cfg['groupby'], cfg['aggs'], where_terms=cfg['where'])

    def timed(fn, timing):
        # timing 0 off, 1 scan + query events, 2 scan events only
        dev.enable_timing(timing != 0, scan_only=timing == 2)
        dev.synchronize()
        w = []
        dv = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            w.append(time.perf_counter() - t0)
            if timing == 1:
                dv.append(dev.last_timing()['total_ms'])
        return np.median(w) * 1e6, (np.median(dv) * 1e3 if dv else float('nan'))

    full = lambda: t.groupby(cfg['groupby'], cfg['aggs'], where_terms=cfg['where'])  # noqa: E731
    ops = parse_agg_list(t.dtypes, cfg['aggs'])
    keep = []
    q = t._query(list(cfg['groupby']), [(o[0], o[2]) for o in ops], cfg['where'], None, keep)

    def bare():
        res = ctypes.c_void_p()
        dev.check(t._lib.bqg_groupby(dev.handle, t.handle, ctypes.byref(q), ctypes.byref(res)))
        L.lib().bqg_result_free(res)

    for name, fn in (('python groupby', full), ('bare C call', bare)):
        for timing in (0, 2, 1):
            w, d = timed(fn, timing)
            print('%-16s timing=%d  wall %.1f us  device total %.1f us' % (name, timing, w, d), flush=True)


if __name__ == '__main__':
    main()
