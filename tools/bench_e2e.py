#!/usr/bin/env python3
"""End-to-end C1 measurement (BASELINE.json configs[0]): the whole bqueryd message path.

C1 = 10 shards x 1 M rows on disk as bcolz ctables, ``groupby(['payment_type'],
[['fare_amount', 'sum', 'fare_amount']], aggregate=True)``.  One query =

  worker: CalcPath.handle_work per shard (worker.py:269-348: open ctable, groupby, write the
          result ctable, tar it)  ->  controller: tar of tars (controller.py:146-221)  ->
  client: rpc.uncompress_groupby_to_df(aggregate=True) (rpc.py:134-179).

Legs (each the best of ``--reps``):
  gpu_warm   shards resident in HBM (ShardCache hit: the steady state of a worker)
  gpu_cold   fresh cache: bcolz decode on the host + H2D copy + query (PCIe-inclusive)
  cpu_port   the same path with the C port of bquery (oracle/cbquery.c) as the calc, on
             already-decoded columns, ``--cpu-workers`` processes (one shard per task) and the
             oracle's client merge -- the reference's architecture on this host's cores.

This is a latency-shaped end-to-end figure (per-message Python + file + tar overheads dominate
at 1 M rows/shard); the headline device throughput is bench.py.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import shutil
import sys
import tempfile
import time
from collections import OrderedDict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GROUPBY = ['payment_type']
AGGS = [['fare_amount', 'sum', 'fare_amount']]
COLS = ('payment_type', 'fare_amount')


def _cpu_task(args):
    """One reference-shaped worker message on the CPU: decode the shard (one thread,
    worker.py:40), the C port of bquery's groupby, then the result ctable + tar reply exactly
    as the GPU worker writes it (worker.py:335-346)."""
    path, = args
    from bqueryd_amd import bcolz_io
    from bqueryd_amd.worker import rm_file_or_dir, tar_directory
    from oracle import cbquery
    t0 = time.perf_counter()
    cols = bcolz_io.read_ctable(path, columns=list(COLS), nthreads=1)
    out = cbquery.handle_work(cols, GROUPBY, AGGS, [])
    tmp_dir = tempfile.mkdtemp(prefix='result_')
    try:
        rm_file_or_dir(tmp_dir)
        bcolz_io.write_ctable(tmp_dir, out)
        data = tar_directory(tmp_dir)
    finally:
        rm_file_or_dir(tmp_dir)
    return data, time.perf_counter() - t0


def _large_message(args):
    """C3 / C5 message-level cost on one GPU: the bcolz shard(s) on disk, resident in HBM after
    a first message (the worker's steady state), then per message: shard-cache lookup, the
    query (device passes + the result's copy to host memory) and the result ctable + tar
    (worker.py:335-346), timed per stage (CalcPath.last_stages); and the unchanged client's
    untar + merge of that one reply (rpc.py:134-179).
      c3: one 100 M-row shard, groupby (pickup_location, vendor_id), sum / count (~1 M groups);
      c5: one node-level message over one GPU's 10 x 12.5 M-row shards (one pass over the
          union + the world-1 merge, ~1 M groups) -- a rank's share of C5."""
    from bqueryd_amd import bcolz_io, messages, rpc, synth
    from bqueryd_amd.engine import get_device
    from bqueryd_amd.worker import CalcPath
    cfg = synth.CONFIGS[args.config]
    cols_needed = synth.query_columns(cfg)
    if args.config == 'c3':
        n_shards, rows = 1, args.rows or cfg['rows']
    else:
        n_shards, rows = args.shards or 10, args.rows or cfg['rows'] // cfg['shards']
    data_dir = tempfile.mkdtemp(prefix='bqgpu_%s_' % args.config)
    try:
        files = []
        for i in range(n_shards):
            cols = synth.taxi_shard(rows, config_id=synth.CONFIG_ID[args.config], n_shards=max(n_shards, cfg.get('shards', 1)),
                                    shard=i, columns=cols_needed)
            fn = 'tripdata-%d.bcolzs' % i
            bcolz_io.write_ctable(os.path.join(data_dir, fn), cols)
            files.append(fn)
            del cols
        dev = get_device()
        calc = CalcPath(data_dir, device=dev)
        m = messages.CalcMessage({'payload': 'groupby', 'token': 'ab' * 8, 'filename': files[0]})
        m.set_args_kwargs([files[0] if args.config == 'c3' else list(files), cfg['groupby'], cfg['aggs'], cfg['where']],
                          {'aggregate': True})
        calc.handle_work(m)  # load + warm
        best = None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            data = calc.handle_work(m)['data']
            t1 = time.perf_counter()
            df = rpc.uncompress_groupby_to_df(rpc.tar_of_tars({files[0]: data}), cfg['groupby'], cfg['aggs'],
                                              cfg['where'], aggregate=True, device=dev)
            t2 = time.perf_counter()
            if best is None or t1 - t0 < best['message_s']:
                best = dict(calc.last_stages, message_s=t1 - t0, client_merge_s=t2 - t1, reply_bytes=len(data),
                            groups=int(len(df)))
        total = n_shards * rows
        line = {'workload': '%s message level: %d bcolz shard(s) x %d rows resident in HBM, groupby %s, aggs %s, '
                            'aggregate=True%s' % (args.config.upper(), n_shards, rows, cfg['groupby'],
                                                 [a[1] for a in cfg['aggs']],
                                                 ', one node-level message (world 1)' if args.config == 'c5' else ''),
                'rows': total, 'gpu_warm': dict(best, rows_per_s=total / best['message_s']),
                'host_threads_for_result_compression': bcolz_io._pool()._max_workers}
        print(json.dumps(line), flush=True)
    finally:
        shutil.rmtree(data_dir, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c1', choices=['c1', 'c3', 'c5'])
    ap.add_argument('--shards', type=int, default=None)
    ap.add_argument('--rows', type=int, default=None)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--cpu-workers', type=int, default=None,
                    help='C1 CPU port: worker processes (default: 2, as BASELINE configs[0] states, and all cores)')
    ap.add_argument('--no-gpu', action='store_true')
    ap.add_argument('--profile', default=None,
                    help='write a cProfile summary of 50 warm per-file messages (handle_work) to this file')
    args = ap.parse_args()
    if args.config != 'c1':
        return _large_message(args)
    args.shards = args.shards or 10
    args.rows = args.rows or 1_000_000

    from bqueryd_amd import bcolz_io, messages, rpc, synth
    from oracle import bquery_oracle as bo
    from oracle import cbquery
    cbquery.build()

    data_dir = tempfile.mkdtemp(prefix='bqgpu_c1_')
    try:
        files, shards = [], []
        for i in range(args.shards):
            cols = synth.taxi_shard(args.rows, config_id=1, n_shards=args.shards, shard=i, columns=COLS)
            fn = 'tripdata-%d.bcolzs' % i
            bcolz_io.write_ctable(os.path.join(data_dir, fn), cols)
            files.append(fn)
            shards.append(cols)
        ref = bo.client_merge([bo.handle_work(s, GROUPBY, AGGS, []) for s in shards], GROUPBY, AGGS,
                              aggregate=True)
        ref = dict(zip(ref['payment_type'].tolist(), ref['fare_amount'].tolist()))
        total_rows = args.shards * args.rows
        line = {'workload': 'C1 end-to-end: %d bcolz shards x %d rows, groupby %s sum fare_amount, '
                            'aggregate=True' % (args.shards, args.rows, GROUPBY),
                'rows': total_rows}

        def check(df):
            got = dict(zip(df['payment_type'].tolist(), df['fare_amount'].tolist()))
            assert set(got) == set(ref), (sorted(got), sorted(ref))
            for k in ref:
                assert abs(got[k] - ref[k]) <= 1e-12 * max(1.0, abs(ref[k])), (k, got[k], ref[k])

        def msg_for(fn):
            m = messages.CalcMessage({'payload': 'groupby', 'token': 'ab' * 8, 'filename': fn})
            m.set_args_kwargs([fn, GROUPBY, AGGS, []], {'aggregate': True})
            return m

        if not args.no_gpu:
            from bqueryd_amd.engine import get_device
            from bqueryd_amd.worker import CalcPath, ShardCache
            dev = get_device()

            def gpu_query(calc):
                t0 = time.perf_counter()
                replies = OrderedDict((fn, calc.handle_work(msg_for(fn))['data']) for fn in files)
                t1 = time.perf_counter()
                df = rpc.uncompress_groupby_to_df(rpc.tar_of_tars(replies), GROUPBY, AGGS, [], aggregate=True,
                                                  device=dev)
                t2 = time.perf_counter()
                check(df)
                return t2 - t0, t1 - t0, t2 - t1

            calc = CalcPath(data_dir, device=dev)
            gpu_query(calc)  # warm the cache
            if args.profile:
                import cProfile
                import io
                import pstats
                msgs = [msg_for(fn) for fn in files] * 5
                pr = cProfile.Profile()
                t0 = time.perf_counter()
                pr.enable()
                for m in msgs:
                    calc.handle_work(m)
                pr.disable()
                per_msg = (time.perf_counter() - t0) / len(msgs)
                sio = io.StringIO()
                pstats.Stats(pr, stream=sio).sort_stats('cumulative').print_stats(45)
                t0 = time.perf_counter()
                for m in msgs:
                    calc.handle_work(m)
                plain = (time.perf_counter() - t0) / len(msgs)
                with open(args.profile, 'w') as f:
                    f.write('warm per-file message: %.1f us (unprofiled), %.1f us under cProfile\n' % (
                        plain * 1e6, per_msg * 1e6))
                    f.write(sio.getvalue())
            warm = min((gpu_query(calc) for _ in range(args.reps)), key=lambda x: x[0])
            cold = min((gpu_query(CalcPath(data_dir, device=dev, cache=ShardCache(device=dev)))
                        for _ in range(args.reps)), key=lambda x: x[0])
            line['gpu_warm'] = {'s_per_query': warm[0], 'worker_s': warm[1], 'client_merge_s': warm[2],
                                'rows_per_s': total_rows / warm[0]}
            line['gpu_cold'] = {'s_per_query': cold[0], 'worker_s': cold[1], 'client_merge_s': cold[2],
                                'rows_per_s': total_rows / cold[0],
                                'note': 'includes bcolz decode on the host and the H2D copy'}

            # node-level message: the node's files in one message, one merged reply
            def node_query(calc):
                m = messages.CalcMessage({'payload': 'groupby', 'token': 'ab' * 8, 'filename': files[0]})
                m.set_args_kwargs([list(files), GROUPBY, AGGS, []], {'aggregate': True})
                t0 = time.perf_counter()
                data = calc.handle_work(m)['data']
                t1 = time.perf_counter()
                df = rpc.uncompress_groupby_to_df(rpc.tar_of_tars({files[0]: data}), GROUPBY, AGGS, [],
                                                  aggregate=True, device=dev)
                t2 = time.perf_counter()
                check(df)
                return t2 - t0, t1 - t0, t2 - t1

            node_query(calc)
            node = min((node_query(calc) for _ in range(args.reps)), key=lambda x: x[0])
            line['gpu_node_warm'] = {'s_per_query': node[0], 'worker_s': node[1], 'client_merge_s': node[2],
                                     'rows_per_s': total_rows / node[0],
                                     'note': 'one node-level message (args[0] = the files, aggregate=True): one '
                                             'pass over the resident shard union + RCCL merge, one reply'}

        # CPU: the reference's architecture (one calc per shard on a pool of worker processes):
        # 2 workers as BASELINE configs[0] states ("CPU controller + 2 workers"), and all cores
        from oracle import cpu_cluster
        ctx = mp.get_context('spawn')  # no fork of a process that initialised the GPU
        counts = [args.cpu_workers] if args.cpu_workers else sorted({2, cpu_cluster.host_cores()})
        for nw in counts:
            with ctx.Pool(nw) as pool:
                pool.map(_cpu_task, [(os.path.join(data_dir, files[0]),)])
                best = None
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    res = pool.map(_cpu_task, [(os.path.join(data_dir, fn),) for fn in files])
                    reply = rpc.tar_of_tars(OrderedDict((fn, r[0]) for fn, r in zip(files, res)))
                    merged = bo.client_merge(rpc.read_shard_results(reply), GROUPBY, AGGS, aggregate=True)
                    dt = time.perf_counter() - t0
                    calc_s = sum(r[1] for r in res)
                    if best is None or dt < best[0]:
                        best = (dt, calc_s)
                check(merged)
            key = 'cpu_port' if nw == 2 or len(counts) == 1 else 'cpu_port_all_cores'
            line[key] = {'s_per_query': best[0], 'rows_per_s': total_rows / best[0],
                         'calc_core_s': best[1], 'workers': nw, 'kind': 'port', 'cpu_model': cpu_cluster.cpu_model(),
                         'note': 'per shard in worker processes: bcolz decode (1 thread) + oracle/cbquery.c '
                                 'calc + result ctable + tar; tar of tars; client untar + oracle merge'}
        print(json.dumps(line), flush=True)
    finally:
        shutil.rmtree(data_dir, ignore_errors=True)


if __name__ == '__main__':
    main()
