#!/usr/bin/env python3
"""Benchmark of the shard-groupby hot path (BASELINE.json metric) on MI355X.

A "step" is one bqueryd per-shard calc (``bqueryd/worker.py:313``: where-terms + groupby +
emit back to host memory) over one synthetic taxi-shaped shard already resident in HBM.
Default workload = BASELINE.json configs[1] (C2): 100 M rows, groupby ``payment_type``,
sum/mean/count of ``fare_amount`` where ``passenger_count >= 2``.

The headline scans the columns as stored (engine option ``compact=0``), so
``roofline.algorithmic_bytes_per_launch`` is SURVEY.md §8(d)'s figure (columns x itemsize x
rows) and ``frac`` is a bandwidth; the compact resident copies are reported in the
line's ``compact`` sub-record with their build cost and the query count that repays it.

Multi-GPU: one process per GPU, launched by ``python -m torch.distributed.run
--nproc-per-node N bench.py --gpus N`` or, with ``--gpus N`` and no ``WORLD_SIZE`` in the
environment, by this script itself (N rank processes started before anything touches a GPU;
``--dry-launch`` prints them).  Each rank owns its own 100 M-row shard (weak scaling: shards are
independent in bqueryd, no data-path collective without ``aggregate=True``); barrier + max over
ranks around the timed region, gloo only for that bookkeeping.  The line's ``c5`` sub-record is
north_star's scaling config at the same N: 10 shards x 12.5 M rows per rank, aggregated in one
pass per rank, then the ``aggregate=True`` merge across the N ranks over RCCL (rpc.py:164-173).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
MODES = ['private-lds', 'shared-lds', 'global-dense', 'global-hash', 'partitioned', 'fused-distinct']
KERNELS = ['k_scan_private', 'k_scan_shared', 'k_scan_global', 'k_scan_global<hash>',
           'bq_jit_part_scatter+k_part_aggregate+k_part_combine+bq_jit_part_first_rows (tile scatter, aggregate, split combine and first-row pass, timed together)',
           'k_scd_fused (rows + count_distinct + sorted_count_distinct in one pass)']


def _dist_env():
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    return ws, rank, local


class _stdout_to_stderr:
    """Route file descriptor 1 to stderr for a block (native libraries printing to stdout)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


class _Comm:
    """Barrier / max-reduce across ranks (gloo, CPU only).  Single process: no-ops."""

    def __init__(self, ws):
        self.ws = ws
        self.dist = None
        if ws > 1:
            import torch.distributed as dist
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            with _stdout_to_stderr():  # gloo announces its peers on stdout: the JSON line is the only stdout
                dist.init_process_group('gloo')
            self.dist = dist

    def broadcast_bytes(self, b):
        """Rank 0's bytes on every rank (the RCCL unique id of the C5 merge)."""
        if not self.dist:
            return b
        box = [b]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def _cpu_baseline(cols, cfg, reps=2):
    """The C port of bquery's per-shard algorithm (oracle/cbquery.c), one thread."""
    from oracle import cbquery
    cbquery.build()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        cbquery.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where'])
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    n = len(next(iter(cols.values())))
    return n / best, best


def _cpu_cluster_baseline(cfg, args, rows, single):
    """The reference's deployment shape on this host's cores (oracle/cpu_cluster.py): one
    controller + N single-threaded workers running the C port of bquery's per-shard groupby
    over the workload split into max(8, 2 x cores) shards (every worker gets messages, as in
    the reference's deployment: one message per shard file to any free worker,
    misc/supervisor.conf:21, controller.py:113-144), client sum-merge (rpc.py:164-173);
    N = 2 and N = all cores.  ``value`` is the all-cores cluster."""
    import shutil
    import tempfile
    from oracle import cpu_cluster
    cores = cpu_cluster.host_cores()
    n_shards = max(8, 2 * cores)
    per = max(1, rows // n_shards)
    counts = sorted(set([2, cores]))
    tmp = tempfile.mkdtemp(prefix='bqgpu-cpu-cluster-')
    try:
        res, _ = cpu_cluster.run(cfg, n_shards, per, counts, config_id=synth_config_id(args.config),
                                 variant=args.variant, bcolz_dir=tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    rate, secs = res[cores]['bcolz']
    return {'value': rate, 'unit': 'rows/s', 'cores': cores, 'kind': 'port',
            'sample': ('%s as %d bcolz shards x %d rows (lz4): 1 controller + %d single-threaded worker processes, '
                       'each reading + blosc-decoding its shard on one thread and running oracle/cbquery.c (the C '
                       'port of bquery\'s multi-pass per-shard groupby: where mask, khash factorize, filter '
                       're-factorize, one pass per aggregation; misc/supervisor.conf:21, worker.py:40) + the client '
                       'sum-merge (rpc.py:164-173); best of 2: %.3f s' % (args.config.upper(), n_shards, per, cores,
                                                                           secs)),
            'cpu_model': cpu_cluster.cpu_model(),
            'n_shards': n_shards,
            'decoded_columns': {'value': res[cores]['decoded'][0], 'unit': 'rows/s', 'cores': cores,
                                'seconds': res[cores]['decoded'][1],
                                'sample': 'the same, columns handed over decoded (shared memory): compute only'},
            'workers_2': {'value': res[2]['bcolz'][0], 'unit': 'rows/s', 'cores': 2, 'seconds': res[2]['bcolz'][1],
                          'decoded_value': res[2]['decoded'][0]},
            'single_worker_one_shard': single}


def synth_config_id(config):
    from bqueryd_amd import synth
    return synth.CONFIG_ID[config]


def _load_traffic(config, rows):
    """(HBM bytes per scan launch, source) from the committed rocprofv3 PMC summary of this
    config (profiles/pmc_<cfg>.json: separate FETCH_SIZE / WRITE_SIZE passes), if present and
    taken at this row count.  It is NOT measured by this run: counter passes need their own
    profiler runs (MI355X_MICROARCH.md), so the line names the file it quotes."""
    path = os.path.join(HERE, 'profiles', 'pmc_%s.json' % config)
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get('rows') == rows:
            src = 'profiles/pmc_%s.json (committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes%s; not this run)' % (
                config, ', ' + d['taken'] if d.get('taken') else '')
            return d.get('hbm_bytes_per_launch'), src
    except (OSError, ValueError):
        pass
    return None, None


def _c5_local_ranks(args):
    """C5 at its full shape on ONE GPU: 80 shards x 12.5 M rows = 1 B rows over
    ``--local-ranks`` ranks (10 shards each, one libbqgpu context per rank, all on this GPU),
    each rank's shards aggregated in one pass over their union, then the W-rank
    ``aggregate=True`` merge (bqg_merge_group over the in-process transport: the code RCCL
    runs, device copies as the wire).  ``value`` is the measured rate of the whole 1 B-row job
    on this one GPU (ranks run one after another); the line also projects the 8-GPU node from
    the measured parts: each rank's shard pass (as it runs alone on a GPU) + the W-rank merge's
    critical path (every phase as long as its slowest rank, each rank's device work measured
    on its own; the exchange is measured as one on-die copy of all ranks' messages, faster than
    xGMI links, so the line also gives the exchange modelled from the bytes per link), and
    measures the one-GPU C5 step (one rank's 10 shards + the world-1 merge) for the
    x-over-one-GPU ratio of north_star."""
    from concurrent.futures import ThreadPoolExecutor

    from bqueryd_amd import dist as bdist
    from bqueryd_amd import synth
    from bqueryd_amd.engine import Device, ShardTable

    cfg = synth.CONFIGS['c5']
    W = args.local_ranks
    per_rank = max(1, cfg['shards'] // 8)  # the 8-GPU layout: 10 shards per rank
    shard_rows = args.rows or cfg['rows'] // cfg['shards']
    n_shards = W * per_rank
    devs = [Device(int(os.environ.get('BQGPU_BENCH_DEVICE', 0))) for _ in range(W)]
    tables = [[] for _ in range(W)]

    def make(i):
        return synth.taxi_shard(shard_rows, config_id=5, n_shards=max(cfg['shards'], n_shards), shard=i,
                                variant=args.variant, columns=synth.query_columns(cfg))
    with ThreadPoolExecutor(16) as ex:  # numpy's generators release the GIL
        for i, s in enumerate(ex.map(make, range(n_shards))):
            tables[i // per_rank].append(ShardTable(s, device=devs[i // per_rank]))
            del s
    colos = [bdist.ColocatedShards(t) for t in tables]
    for c in colos:
        c.union(synth.query_columns(cfg))  # each rank's shard set, resident once (untimed, like the load)
    probe, _ = colos[0].groupby_tables(cfg['groupby'], cfg['aggs'])
    dtypes = {n: np.dtype(probe[0].dtypes[n]) for n in probe[0].names}
    for p_ in probe:
        p_.close()
    group = bdist.CommGroup(devs, transport='local')
    shard_s = [[] for _ in range(W)]
    merge_s, timings, phases = [], [], []

    def step():
        per = []
        for r, c in enumerate(colos):
            t0 = time.perf_counter()
            p, reduced = c.groupby_tables(cfg['groupby'], cfg['aggs'])
            shard_s[r].append(time.perf_counter() - t0)
            timings.append(devs[r].last_timing())
            per.append(p)
        t1 = time.perf_counter()
        merged = bdist.merge_group_device(per, cfg['groupby'], cfg['aggs'], dtypes, group, reduced=True)
        merge_s.append(time.perf_counter() - t1)
        phases.append([list(bdist.merge_phases(d).values()) for d in devs])
        for tabs in per:
            for p in tabs:
                p.close()
        return merged

    for i in range(args.warmup):
        out = step()
        if i == 0:
            devs[0].jit_wait(180)
    if int(out['n'].sum()) != n_shards * shard_rows:
        raise SystemExit('sanity check failed: %d merged rows' % int(out['n'].sum()))
    for d in devs:
        d.enable_timing(True)
    for lst in shard_s + [merge_s, timings, phases]:
        del lst[:]
    for d in devs:
        d.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    for d in devs:
        d.synchronize()
    elapsed = time.perf_counter() - t0
    group.close()

    # the one-GPU C5 step: rank 0's shards + the world-1 RCCL merge
    with _stdout_to_stderr():
        rccl = bdist.RcclComm(devs[0])
    one_s, one_merge_s = [], []
    for k in range(args.warmup + args.steps):
        t0 = time.perf_counter()
        per, reduced = colos[0].groupby_tables(cfg['groupby'], cfg['aggs'])
        t1 = time.perf_counter()
        bdist.merge_partials_device(per, cfg['groupby'], cfg['aggs'], dtypes, rccl, reduced=reduced)
        for p in per:
            p.close()
        if k >= args.warmup:
            one_s.append(time.perf_counter() - t0)
            one_merge_s.append(time.perf_counter() - t1)
    rccl.close()
    for c in colos:
        c.close()

    rank_ms = [1e3 * float(np.mean(s)) for s in shard_s]
    merge_ms = 1e3 * float(np.mean(merge_s))
    ph = np.mean(np.array(phases), axis=0)  # [rank][phase] ms
    phase_max = {n: float(ph[:, i].max()) for i, n in enumerate(bdist.MERGE_PHASES)}
    host_copy_ms = phase_max['gather']  # each rank's slice copied to host memory, measured alone
    # the merge as 8 GPUs would run it: each phase as long as its slowest rank (the collective
    # steps measured as one in-process transfer of all ranks), the host copies included
    # the exchange over xGMI instead of one on-die copy: a rank's reduced table holds at most
    # every merged key; it sends 1/W of it to each of W-1 peers, one point-to-point link each
    # at ~50 GB/s achieved (MI355X_MICROARCH.md: 7 links x ~153 GB/s peak), plus ~20 us of
    # RCCL group latency; the projection takes the larger of the measured and modelled exchange
    res_bytes = float(sum(np.dtype(dtypes[n]).itemsize for n in dtypes))
    per_link = float(len(out[next(iter(out))])) / W * res_bytes
    xgmi_ms = per_link / 50e9 * 1e3 + 0.02 if W > 1 else 0.0
    merge_crit_ms = sum(phase_max.values()) - phase_max['exchange'] + max(phase_max['exchange'], xgmi_ms)
    one_ms = 1e3 * float(np.mean(one_s))
    proj_ms = max(rank_ms) + merge_crit_ms
    total_rows = n_shards * shard_rows
    one_rate = per_rank * shard_rows / (one_ms * 1e-3)
    proj_rate = total_rows / (proj_ms * 1e-3)
    scan_avg = float(np.mean([t['scan_ms'] for t in timings]))
    bytes_per_launch = timings[-1]['bytes']
    achieved = bytes_per_launch / (scan_avg * 1e-3) / 1e9
    line = {
        'metric': 'groupby rows/sec (whole node) + achieved HBM GB/s vs peak, 1/2/4/8 GPUs',
        'value': total_rows * args.steps / elapsed,
        'unit': 'rows/s',
        'n_gpus': 1,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic taxi-shaped shards (SURVEY.md §8d generator, %s variant), resident in HBM' % args.variant,
        'config': {
            'workload': ('C5 full shape: %d shards x %d rows = %d rows, %d ranks as %d libbqgpu contexts on ONE GPU '
                         '(in-process transport), groupby %s, aggs %s, aggregate=True merge across the ranks; value = '
                         'the whole job on this one GPU, ranks one after another' % (
                             n_shards, shard_rows, total_rows, W, W, cfg['groupby'], [a[1] for a in cfg['aggs']])),
            'rows_per_rank': per_rank * shard_rows,
            'parallelism': '%d in-process ranks on one GPU' % W,
            'shard_pass_ms_per_rank': rank_ms,
            'merge_ms_all_ranks': merge_ms,
            'merge_phase_ms_max_over_ranks': phase_max,
            'merge_result_to_host_ms': host_copy_ms,
            'merge_ms_critical_path': merge_crit_ms,
            'merge_exchange_modelled_xgmi_ms': xgmi_ms,
            'merge': 'bqg_merge_group_host at world %d: pack kernel, count all-gather, per-column exchange, hash '
                     'reduce (partials in source order), each rank\'s partition copied straight into its slice '
                     'of one pinned host result; every rank\'s work on this one GPU' % W,
            'one_gpu': {'ms_per_step': one_ms, 'rows_per_s': one_rate, 'merge_ms_world1': 1e3 * float(np.mean(one_merge_s)),
                        'what': 'one rank\'s %d shards in one pass + the world-1 RCCL merge (bench.py --config c5 at N=1)'
                                % per_rank},
            'projected_node': {'gpus': W, 'ms_per_step': proj_ms, 'rows_per_s': proj_rate,
                               'x_over_one_gpu': proj_rate / one_rate,
                               'basis': 'max over ranks of the measured shard pass (each as alone on its GPU) + the '
                                        'merge\'s critical path: every merge phase as long as its slowest rank '
                                        '(host wall time per rank, each rank\'s device work waited for on its own, '
                                        'its slice of the result copied to host memory alone; the payload exchange '
                                        'the larger of one in-process transfer of all %d ranks on this GPU and the '
                                        'xGMI model); not an 8-GPU measurement' % W},
        },
        'roofline': {
            'bound': 'hbm',
            'achieved': achieved,
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS,
            'traffic': None,
            'traffic_source': None,
            'kernel': KERNELS[timings[-1]['mode'] or 0],
            'kernel_avg_ms': scan_avg,
            'algorithmic_bytes_per_launch': bytes_per_launch,
        },
        'cpu_baseline': None,
    }
    print(json.dumps(line), flush=True)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(('127.0.0.1', 0))
        return sk.getsockname()[1]


def launch_plan(n, argv):
    """(command, environment additions) of each of the ``n`` rank processes ``--gpus n``
    starts when no launcher did (rank r on GPU r, rendezvous on 127.0.0.1)."""
    port = _free_port()
    cmd = [sys.executable, os.path.abspath(__file__)] + [a for a in argv if a != '--dry-launch']
    return [(cmd, {'WORLD_SIZE': str(n), 'RANK': str(r), 'LOCAL_RANK': str(r), 'LOCAL_WORLD_SIZE': str(n),
                   'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)}) for r in range(n)]


def _launch_ranks(n, argv, dry, plan=None, grace_s=15.0, poll_s=0.2):
    """Start the N rank processes (before this process touches a GPU) and wait for them; rank
    0's stdout is this process's, the others' is discarded.  When a rank fails (non-zero exit,
    e.g. a watchdog that found a collective hung), the others get ``grace_s`` seconds to end
    on their own -- rank 0 prints the line it has -- and are then terminated, so a hung peer
    never keeps the job alive.  Exit status: the first failing rank's, else 0."""
    import subprocess
    plan = plan if plan is not None else launch_plan(n, argv)
    if dry:
        print(json.dumps({'launch': 'self', 'ranks': n, 'commands': [c for c, _ in plan], 'env': [e for _, e in plan]}),
              flush=True)
        return 0
    procs = []
    for r, (cmd, extra) in enumerate(plan):
        procs.append(subprocess.Popen(cmd, env=dict(os.environ, **extra),
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    first_bad, t_bad = None, None
    while True:
        rcs = [p.poll() for p in procs]
        for r, rc in enumerate(rcs):
            if rc not in (None, 0) and first_bad is None:
                first_bad, t_bad = rc, time.monotonic()
                sys.stderr.write('bench.py: rank %d exited with status %d\n' % (r, rc))
        if all(rc is not None for rc in rcs):
            break
        if first_bad is not None and time.monotonic() - t_bad > grace_s:
            for r, p in enumerate(procs):
                if p.poll() is None:
                    sys.stderr.write('bench.py: terminating rank %d (a peer failed)\n' % r)
                    p.terminate()
            for p in procs:
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(poll_s)
    return first_bad if first_bad is not None else 0


# Where each rank is (a watchdog reports it when a sub-benchmark hangs): the stage the bench is
# in, and the libbqgpu context whose merge progress (bqg_comm_progress) names the collective.
_PROGRESS = {'stage': 'start', 'device': None}


def _stage(text):
    _PROGRESS['stage'] = text


def _status_dir():
    """Per-job directory the ranks' watchdogs leave their status in (one node: MASTER_PORT
    names the job)."""
    import tempfile
    return os.path.join(tempfile.gettempdir(), 'bqgpu-bench-%s' % os.environ.get('MASTER_PORT', 'solo'))


def _rank_status(rank):
    st = {'rank': rank, 'stage': _PROGRESS['stage']}
    dev = _PROGRESS.get('device')
    if dev is not None:
        try:
            from bqueryd_amd import dist as bdist
            st['merge'] = bdist.merge_progress(dev)
        except Exception as e:  # no communicator yet, or the library is gone
            st['merge'] = 'n/a (%s)' % e
    return st


class _Watchdog:
    """Ends this rank if a sub-benchmark hangs (an RCCL collective that never completes):
    after ``seconds`` every rank records where it is (stage + merge phase) in the job's status
    directory; rank 0 waits briefly for its peers' records, calls ``on_timeout(statuses)`` (it
    prints the line it has, the hung part marked with them) and every rank exits with status
    ``EXIT_HUNG`` -- a hang is a failed run, never rc 0."""

    EXIT_HUNG = 3

    def __init__(self, seconds, on_timeout, rank=0, ws=1, peer_wait_s=8.0):
        import threading
        self.done = threading.Event()
        self.t = threading.Thread(target=self._run, args=(seconds, on_timeout, rank, ws, peer_wait_s), daemon=True)
        self.t.start()

    def _run(self, seconds, on_timeout, rank, ws, peer_wait_s):
        if self.done.wait(seconds):
            return
        try:
            mine = _rank_status(rank)
            sys.stderr.write('bench.py: rank %d hung: %s\n' % (rank, json.dumps(mine)))
            d = _status_dir()
            statuses = {rank: mine}
            try:
                os.makedirs(d, exist_ok=True)
                with open(os.path.join(d, 'rank%d.json' % rank), 'w') as f:
                    json.dump(mine, f)
            except OSError:
                pass
            if rank == 0:
                t_end = time.monotonic() + (peer_wait_s if ws > 1 else 0.0)
                while True:
                    for r in range(1, ws):
                        if r not in statuses:
                            try:
                                with open(os.path.join(d, 'rank%d.json' % r)) as f:
                                    statuses[r] = json.load(f)
                            except (OSError, ValueError):
                                pass
                    if len(statuses) == ws or time.monotonic() > t_end:
                        break
                    time.sleep(0.1)
                on_timeout([statuses.get(r, {'rank': r, 'stage': 'no status (exited or hung before its watchdog)'})
                            for r in range(ws)])
            else:
                time.sleep(peer_wait_s + 2.0)  # rank 0 reads the status and prints before the launcher reaps
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(self.EXIT_HUNG)

    def cancel(self):
        self.done.set()


def _c5_ranks(args, comm, dev, ws, rank, steps, warmup, shard_rows=None):
    """C5 on this node's ranks (north_star's scaling config): 10 shards x 12.5 M rows per rank
    (80 shards at 8 ranks), each rank's shards aggregated in one pass over their union, then
    the aggregate=True merge (hash partition, RCCL exchange over xGMI, reduce, gather to rank 0)
    at world ``ws``.  A step is the rank's shard pass + the merge; ``ms_per_step`` is the max
    over ranks.  Returns the record on rank 0 (None elsewhere)."""
    from bqueryd_amd import dist as bdist
    from bqueryd_amd import synth
    from bqueryd_amd.engine import ShardTable

    cfg = synth.CONFIGS['c5']
    per_rank = max(1, cfg['shards'] // 8)
    shard_rows = shard_rows or cfg['rows'] // cfg['shards']
    rows = per_rank * shard_rows
    _stage('c5: generating shards')
    t_gen = time.perf_counter()
    from concurrent.futures import ThreadPoolExecutor

    def make(i):
        return synth.taxi_shard(shard_rows, config_id=5, n_shards=max(cfg['shards'], ws * per_rank),
                                shard=rank * per_rank + i, variant=args.variant, columns=synth.query_columns(cfg))
    tables = []
    with ThreadPoolExecutor(8) as ex:  # numpy's generators release the GIL
        for sc in ex.map(make, range(per_rank)):
            tables.append(ShardTable(sc, device=dev))
            del sc
    gen_s = time.perf_counter() - t_gen
    _stage('c5: RCCL communicator init (world %d)' % ws)
    if os.environ.get('BQGPU_BENCH_ONE_GPU_RCCL') == '1':
        # rehearsal of the multi-GPU run on a one-GPU box (with BQGPU_BENCH_DEVICE=0): RCCL
        # refuses two ranks on one device of one host, so each rank claims a host of its own
        # and the ranks talk over RCCL's socket transport (tools/dist_check.py does the same)
        os.environ['NCCL_HOSTID'] = 'bqgpu-rank%d' % rank
        os.environ.setdefault('NCCL_SOCKET_IFNAME', 'lo')
        os.environ.setdefault('NCCL_IB_DISABLE', '1')
    with _stdout_to_stderr():  # librccl prints a banner on stdout at init
        uid = comm.broadcast_bytes(bdist.new_unique_id() if rank == 0 else None)
        rccl = bdist.RcclComm(dev, rank, ws, uid)
    _PROGRESS['device'] = dev
    _stage('c5: shard union + probe groupby')
    colo = bdist.ColocatedShards(tables)
    colo.union(synth.query_columns(cfg))  # the rank's shard set, resident once (like the load)
    probe, _ = colo.groupby_tables(cfg['groupby'], cfg['aggs'])
    dtypes = {n: np.dtype(probe[0].dtypes[n]) for n in probe[0].names}
    names = list(probe[0].names)
    local_rows = sum(p_.nrows for p_ in probe)
    for p_ in probe:
        p_.close()
    # the merged rows land in node-shared host memory (bqg_merge_shared_host): every rank copies
    # its partition over its own link, as a one-process-per-GPU worker node would serve the
    # reply -- no gather to rank 0 and no single large copy behind rank 0's link.  Sized from
    # the largest rank's reduced table (ranks mostly share keys), grown if the merge has more.
    _stage('c5: shared result block')
    shm = {'cap': int(comm.max(local_rows) * 1.25) + 1024, 'block': None, 'n': 0}
    shm_tag = comm.broadcast_bytes(('bqgpu-c5-%d-%d' % (os.getpid(), int(time.time()))).encode() if rank == 0 else None)

    def open_block():
        shm['n'] += 1
        shm['block'] = bdist.SharedResult('%s-%d' % (shm_tag.decode(), shm['n']), shm['cap'], names, dtypes,
                                          create=rank == 0)
    if rank == 0:
        open_block()
    comm.barrier()
    if rank != 0:
        open_block()
    phase, timings, merged_rows = [], [], []
    where = ['']

    def merge(per, reduced):
        while True:
            try:
                return bdist.merge_partials_shared(per, cfg['groupby'], cfg['aggs'], dtypes, rccl, shm['block'],
                                                   reduced=reduced)
            except ValueError as e:  # every rank alike: grow the block and merge again
                comm.barrier()
                shm['block'].close()
                shm['cap'] = int(e.args[1])
                if rank == 0:
                    open_block()
                comm.barrier()
                if rank != 0:
                    open_block()

    def step():
        _PROGRESS['stage'] = where[0] + ' shard pass'
        t0 = time.perf_counter()
        per, reduced = colo.groupby_tables(cfg['groupby'], cfg['aggs'])
        timings.append(dev.last_timing())
        _PROGRESS['stage'] = where[0] + ' merge'
        t1 = time.perf_counter()
        n = merge(per, reduced)
        for p_ in per:
            p_.close()
        phase.append((t1 - t0, time.perf_counter() - t1))
        merged_rows.append(n)
        return n

    for i in range(warmup):
        where[0] = 'c5: warmup step %d/%d:' % (i + 1, warmup)
        out = step()
        if i == 0:
            _stage('c5: waiting for background kernel compiles')
            dev.jit_wait(180)
    ok = None
    if rank == 0:  # every scanned row counted once, across the ranks (rank 0 reads the shared block)
        ok = int(shm['block'].columns(out)['n'].sum()) == ws * rows
    # timed steps without device timing (with it, the merge waits for each phase's device work)
    dev.enable_timing(False)
    del phase[:], timings[:]
    _stage('c5: barrier before the timed steps')
    comm.barrier()
    dev.synchronize()
    where[0] = 'c5: timed steps:'
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dev.synchronize()
    t1 = time.perf_counter()
    _stage('c5: barrier after the timed steps')
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    shard_ms = comm.max(1e3 * float(np.mean([p[0] for p in phase])))
    merge_ms = comm.max(1e3 * float(np.mean([p[1] for p in phase])))
    # the shard pass's scan kernels: HIP events over a few more (untimed) steps
    dev.enable_timing(True, scan_only=True)
    del timings[:]
    where[0] = 'c5: device-timed steps:'
    for _ in range(3):
        step()
    dev.synchronize()
    _stage('c5: closing')
    scan_ms = comm.max(float(np.mean([t['scan_ms'] for t in timings])))
    dev.enable_timing(False)
    _PROGRESS['device'] = None
    comm.barrier()  # every rank done with the shared block before rank 0 unlinks it
    shm['block'].close()
    rccl.close()
    colo.close()
    for t in tables:
        t.close()
    _stage('c5: done')
    if rank != 0:
        return None
    alg = timings[-1]['bytes']
    return {
        'workload': ('C5: %d ranks x %d shards x %d rows = %d rows, groupby %s, aggs %s, one pass over each rank\'s '
                     'shards + the aggregate=True merge across the ranks over RCCL (bqg_merge_shared_host at world '
                     '%d: the merged rows into node-shared host memory, each rank\'s partition over its own link)'
                     % (ws, per_rank, shard_rows, ws * rows, cfg['groupby'], [a[1] for a in cfg['aggs']], ws)),
        'merged_rows': merged_rows[-1] if merged_rows else None,
        'value': ws * rows * steps / elapsed,
        'unit': 'rows/s',
        'n_gpus': ws,
        'rows_per_gpu': rows,
        'ms_per_step': elapsed / steps * 1e3,
        'shard_pass_ms_max_over_ranks': shard_ms,
        'merge_ms_max_over_ranks': merge_ms,
        'scan_kernel_ms_max_over_ranks': scan_ms,
        'roofline_frac_of_the_shard_pass': alg / (scan_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        'merged_row_count_check': ok,
        'scaling': 'weak',
        'data_gen_s': gen_s,
        'note': 'the driver\'s N = 1, 2, 4, 8 runs give the curve: north_star asks value(8) >= 6 x value(1)',
    }


def _run_c5_guarded(line, run_c5, comm, rank, ws, timeout_s):
    """The c5 sub-record under a watchdog.  Every rank starts it together (a barrier first),
    so a collective that hangs on a new node ends every rank within ``timeout_s``: rank 0
    prints the line with ``c5.error`` naming each rank's stage and merge phase, and the
    process exits non-zero (``_Watchdog.EXIT_HUNG``).  An exception inside c5 only marks
    the sub-record (the headline stands)."""
    def on_timeout(statuses):
        if rank == 0:
            line['c5'] = {'error': 'did not finish within %.0f s: the run fails with status %d; each rank\'s stage '
                                   'and merge phase when it was abandoned are in `ranks`' % (timeout_s,
                                                                                            _Watchdog.EXIT_HUNG),
                          'ranks': statuses}
            print(json.dumps(line), flush=True)
    try:  # a previous job's record under the same port is not this rank's
        os.remove(os.path.join(_status_dir(), 'rank%d.json' % rank))
    except OSError:
        pass
    _stage('c5: barrier before the sub-record')
    comm.barrier()
    wd = _Watchdog(timeout_s, on_timeout, rank=rank, ws=ws)
    try:
        line['c5'] = run_c5()
    except Exception as e:  # the headline stands; the sub-record says what failed
        line['c5'] = {'error': '%s: %s' % (type(e).__name__, e), 'stage': _PROGRESS['stage']}
    wd.cancel()


def _cold_first_query(dev, step):
    """The first query of the bench's shape on a fresh worker, as on a new box: the run-time
    specialiser's disk cache pointed at an empty directory (BQGPU_JIT_CACHE), so the query finds
    no compiled kernel for its shape.  With option jit_async (the default) it runs the
    precompiled generic kernel while a host thread compiles the specialised one; the bench then
    waits for that compile (bqg_jit_wait) so every timed step runs the specialised kernel."""
    import shutil
    import tempfile
    tmp = tempfile.mkdtemp(prefix='bqgpu-jit-cold-')
    old = os.environ.get('BQGPU_JIT_CACHE')
    os.environ['BQGPU_JIT_CACHE'] = tmp
    try:
        dev.synchronize()
        t0 = time.perf_counter()
        step()
        dev.synchronize()
        first_ms = 1e3 * (time.perf_counter() - t0)
        first_spec = dev.last_timing()['specialized']
        t1 = time.perf_counter()
        w = dev.jit_wait(180)
        wait_s = time.perf_counter() - t1
    finally:
        if old is None:
            os.environ.pop('BQGPU_JIT_CACHE', None)
        else:
            os.environ['BQGPU_JIT_CACHE'] = old
        shutil.rmtree(tmp, ignore_errors=True)
    return {'first_query_ms': first_ms,
            'first_query_kernel': 'specialised' if first_spec else 'generic (precompiled; the specialised one compiling '
                                                                   'on a host thread)',
            'jit_async': bool(dev.get_option('jit_async')),
            'background_compile_wait_s': wait_s, 'background_compiles': w,
            'what': 'wall time of the first query on the freshly loaded shard with an empty run-time-compile cache '
                    '(a new box): plan, statistics, slot arrays, scan, emit, result to host'}


def _compact_record(dev, table, step, steps, warmup, full_ms, full_scan_ms):
    """The compact resident copies on the same shard and query: their build on
    the first query that reads them (device time), the steady step and scan over them, the HBM
    they add, and how many queries repay the build."""
    table.drop_compact()
    base_bytes = table.device_bytes()
    dev.set_option('compact', 1)
    try:
        dev.enable_timing(True)
        dev.synchronize()
        t0 = time.perf_counter()
        step()
        dev.synchronize()
        first_ms = 1e3 * (time.perf_counter() - t0)
        first = dev.last_timing()
        copy_bytes = table.device_bytes() - base_bytes
        if copy_bytes <= 0:
            return {'built': False, 'note': 'no column of this query has a narrower resident form'}
        dev.jit_wait(180)  # the copies' query shape, compiled in the background: timed specialised
        for _ in range(warmup):
            step()
        dev.enable_timing(True, scan_only=True)
        dev.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        dev.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        last = dev.last_timing()
        scan = last['scan_ms_sum'] / max(1, last['timed_queries'])
    finally:
        dev.set_option('compact', 0)
        table.drop_compact()
    gain = full_ms - ms
    return {
        'built': True,
        'what': 'integer columns as offsets from their minimum in the fewest bytes holding their range, float64 '
                'columns that are only summed as their exact integer codes (1-2 byte offsets when they span < 2^16)',
        'ms_per_step': ms,
        'rows_per_s': last['rows'] / (ms * 1e-3),
        'scan_kernel_ms': scan,
        'bytes_read_per_launch': last['bytes_read'],
        'read_gbs': last['bytes_read'] / (scan * 1e-3) / 1e9,
        'read_frac_of_peak': last['bytes_read'] / (scan * 1e-3) / 1e9 / HBM_PEAK_GBS,
        'build_device_ms': first['compact_ms'],
        'first_query_ms': first_ms,
        'first_query_device_ms': first['total_ms'],
        'hbm_bytes_added': copy_bytes,
        'break_even_queries': (first['compact_ms'] / gain) if gain > 0 else None,
        'vs_full_width_step': full_ms / ms if ms > 0 else None,
        'vs_full_width_scan': full_scan_ms / scan if scan > 0 else None,
        'note': 'not the headline: the copies are a derived cache built by the first query that reads them '
                '(its device time is build_device_ms); the headline scans the columns as stored',
    }


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None, help='ranks (default: WORLD_SIZE, else 1)')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', default='c2', choices=['c2', 'c3', 'c4', 'c5'])
    ap.add_argument('--sorted', action='store_true', help='C4: rows sorted by (pu_location_id, passenger_count)')
    ap.add_argument('--c5-per-shard', action='store_true',
                    help='C5: one groupby per shard + local re-group instead of one pass over the rank\'s shards')
    ap.add_argument('--rows', type=int, default=None, help='override rows per shard')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-c5', action='store_true', help='leave out the c5 sub-record')
    ap.add_argument('--no-cold-record', action='store_true',
                    help='leave out the cold_start record (profiler runs: its generic-kernel steps share the trace)')
    ap.add_argument('--no-compact-record', action='store_true',
                    help='leave out the compact sub-record (profiler runs: its scans share the kernel name)')
    ap.add_argument('--compact', action='store_true',
                    help='time the compact resident copies as the headline (not §8(d)-consistent; profiling)')
    ap.add_argument('--variant', default='exact', choices=['exact', 'raw', 'wide'])
    ap.add_argument('--local-ranks', type=int, default=1,
                    help='C5: the full 80-shard workload over this many ranks as contexts on one GPU')
    ap.add_argument('--dry-launch', action='store_true', help='print the rank processes --gpus N would start')
    ap.add_argument('--c5-timeout', type=float, default=300.0, help='seconds before a hung c5 sub-record is abandoned')
    args = ap.parse_args(argv)
    if args.config == 'c5' and args.local_ranks > 1:
        return _c5_local_ranks(args)
    if 'WORLD_SIZE' not in os.environ and (args.gpus or 1) > 1:
        return _launch_ranks(args.gpus, argv, args.dry_launch)
    if args.dry_launch:
        print(json.dumps({'launch': 'none', 'ranks': int(os.environ.get('WORLD_SIZE', '1'))}), flush=True)
        return 0

    ws, rank, local = _dist_env()
    comm = _Comm(ws)
    seen = int(round(comm.sum(1)))
    if seen != ws or (args.gpus is not None and args.gpus != ws):
        comm.close()
        raise SystemExit('bench.py --gpus %s: %d ranks joined, WORLD_SIZE %d' % (args.gpus, seen, ws))

    from bqueryd_amd import synth
    from bqueryd_amd.engine import Device, ShardTable

    cfg = synth.CONFIGS[args.config]
    # BQGPU_BENCH_DEVICE pins every rank to one GPU (rehearsing the multi-rank path on a one-GPU box)
    dev = Device(int(os.environ.get('BQGPU_BENCH_DEVICE', local)))
    if not args.compact:
        dev.set_option('compact', 0)  # the headline scans the columns as stored (SURVEY §8d bytes)
    if args.config == 'c5':
        rec = _c5_ranks(args, comm, dev, ws, rank, args.steps, args.warmup,
                        shard_rows=args.rows)
        comm.close()
        if rank == 0:
            line = {'metric': 'groupby rows/sec (whole node) + achieved HBM GB/s vs peak, 1/2/4/8 GPUs',
                    'value': rec['value'], 'unit': 'rows/s', 'n_gpus': ws, 'steps': args.steps,
                    'warmup': args.warmup, 'ms_per_step': rec['ms_per_step'], 'higher_is_better': True,
                    'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64',
                    'data': 'synthetic taxi-shaped shards (SURVEY.md §8d generator, %s variant), resident in HBM'
                            % args.variant,
                    'config': {'workload': rec['workload'], 'rows_per_gpu': rec['rows_per_gpu'],
                               'parallelism': 'shard-per-rank x%d + RCCL merge' % ws},
                    'roofline': None, 'cpu_baseline': None, 'c5': rec}
            print(json.dumps(line), flush=True)
        return 0

    npass_expected = None
    rows = args.rows or cfg['rows']
    # --sorted: C4's second variant, rows ordered by (pu_location_id, passenger_count)
    # (SURVEY.md §8d), the row order sorted_count_distinct is meant for
    sort_by = ['pu_location_id', 'passenger_count'] if (args.sorted and args.config == 'c4') else None
    cols = synth.taxi_shard(rows, config_id=synth.CONFIG_ID[args.config], n_shards=max(ws, 1),
                            shard=rank, variant=args.variant, columns=synth.query_columns(cfg),
                            sort_by=sort_by)
    table = ShardTable(cols, device=dev)
    if cfg['where']:
        npass_expected = int(np.count_nonzero(cols['passenger_count'] >= 2))
    timings = []
    g_cols, g_aggs, g_where = cfg['groupby'], cfg['aggs'], cfg['where']

    def step():
        # (timed steps: the library sums each query's scan events, read once after the loop)
        return table.groupby(g_cols, g_aggs, where_terms=g_where)[0]

    def step_t():
        out = step()
        timings.append(dev.last_timing())
        return out

    # the first query on a fresh worker: an empty JIT cache (a new box), the query shape's
    # specialised kernel compiled in the background while this query runs the generic one
    cold = None if args.no_cold_record else _cold_first_query(dev, step)
    if cold is None:
        step()
        dev.jit_wait(180)  # the timed steps run the specialised kernel
    for _ in range(args.warmup):
        out = step()
    cnt_col = [a[2] for a in cfg['aggs'] if a[1] == 'count']
    if npass_expected is not None and cnt_col and out is not None:
        got = int(out[cnt_col[0]].sum())
        if got != npass_expected:
            raise SystemExit('sanity check failed: %d != %d passing rows' % (got, npass_expected))

    # device timing of the dominant (scan) kernel: HIP events on the library's stream around
    # the scan launches (scan_only: the whole-query events are recorded after the timed steps)
    dev.enable_timing(True, scan_only=True)  # (resets the library's running scan-time sum)
    comm.barrier()
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dev.synchronize()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    total_rows = comm.sum(rows * args.steps)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_rows / elapsed
    last = dev.last_timing()
    if last['timed_queries'] != args.steps:
        raise SystemExit('timing: %d scan windows for %d steps' % (last['timed_queries'], args.steps))
    scan_avg = last['scan_ms_sum'] / last['timed_queries']
    bytes_per_launch = last['bytes']
    read_per_launch = last['bytes_read']
    mode = last['mode']

    # whole-query device time (first launch to result), from extra untimed steps
    dev.enable_timing(True)
    del timings[:]
    for _ in range(min(args.steps, 10)):
        step_t()
    dev.synchronize()
    device_avg = float(np.mean([t['total_ms'] for t in timings])) if timings else float('nan')
    copy_avg = float(np.mean([t['copy_ms'] for t in timings])) if timings else float('nan')
    achieved = bytes_per_launch / (scan_avg * 1e-3) / 1e9 if scan_avg > 0 else 0.0

    # the generic (precompiled) kernel's steady step: what a cold shape's first query is held to
    if cold is not None:
        with dev.options(jit=0):
            for _ in range(2):
                step()
            dev.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            dev.synchronize()
            gen_ms = (time.perf_counter() - t0) / args.steps * 1e3
        cold['generic_steady_ms_per_step'] = gen_ms
        cold['first_over_generic_steady'] = cold['first_query_ms'] / gen_ms if gen_ms > 0 else None
    compact = None
    if rank == 0 and not args.compact and not args.no_compact_record and mode in (0, 1, 2, 5):
        compact = _compact_record(dev, table, step, args.steps, args.warmup, ms_per_step, scan_avg)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        rate, secs = _cpu_baseline(cols, cfg)
        single = {'value': rate, 'unit': 'rows/s', 'cores': 1,
                  'sample': 'one %d-row %s shard, one worker (best of 2: %.2f s)' % (rows, args.config.upper(), secs)}
        cpu = _cpu_cluster_baseline(cfg, args, rows, single)
    del cols
    table.close()
    traffic, traffic_source = _load_traffic(args.config if not args.compact else args.config + '_compact', rows)
    dev.enable_timing(False)

    line = {
        'metric': 'groupby rows/sec (whole node) + achieved HBM GB/s vs peak, 1/2/4/8 GPUs',
        'value': value,
        'unit': 'rows/s',
        'n_gpus': ws,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': ms_per_step,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic taxi-shaped shards (SURVEY.md §8d generator, %s variant), resident in HBM' % args.variant,
        'config': {
            'workload': '%s: %d rows per GPU (1 shard), groupby %s, aggs %s, where %s%s' % (
                args.config.upper(), rows, cfg['groupby'], [a[1] for a in cfg['aggs']], cfg['where'],
                ', rows sorted by (pu_location_id, passenger_count)' if (args.sorted and args.config == 'c4') else ''),
            'rows_per_gpu': rows,
            'parallelism': 'shard-per-rank x%d' % ws,
            'engine_mode': MODES[mode or 0],
            'resident_columns': ('compact copies (--compact; not the §8(d) headline)' if args.compact else
                                 'as stored (engine option compact=0): the scan reads every query column at its '
                                 'stored width'),
            **({'narrow_entries': bool(last.get('narrow'))} if mode == 4 else {}),
        },
        'roofline': {
            'bound': 'hbm',
            'achieved': achieved,
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS,
            'traffic': traffic,
            'traffic_source': traffic_source,
            'kernel': KERNELS[mode or 0],
            'kernel_avg_ms': scan_avg,
            'algorithmic_bytes_per_launch': bytes_per_launch,
            'algorithmic_bytes_definition': 'SURVEY.md §8(d): the distinct columns the query reads x their stored '
                                            'itemsize x rows + the output table (G x columns x 8 B)',
            'bytes_read_per_launch': read_per_launch,
            'device_ms_per_query': device_avg,
            # the same algorithmic bytes over the WHOLE query's device time (every kernel of the
            # query, the fills, and the result's copy to host memory): what the kernels beside
            # the scan cost -- for C2 the one-workgroup finish, for C3 the large-result emit
            # (compaction, first-row bitmap, rank pass) and the 24 MB PCIe copy
            'frac_whole_query_incl_result_copy': (bytes_per_launch / (device_avg * 1e-3) / 1e9 / HBM_PEAK_GBS
                                                  if device_avg == device_avg and device_avg > 0 else None),
            # ... and over every kernel of the query (its device time less the result's copy to
            # host memory, which runs at the PCIe rate): what the kernels beside the counted ones
            # cost (for C3 the large-result emit: first-row marks, rank scan, emit)
            'result_copy_ms': copy_avg if copy_avg == copy_avg else None,
            'device_ms_per_query_excl_result_copy': (device_avg - copy_avg if copy_avg == copy_avg else None),
            'frac_all_kernels': (bytes_per_launch / ((device_avg - copy_avg) * 1e-3) / 1e9 / HBM_PEAK_GBS
                                 if copy_avg == copy_avg and device_avg - copy_avg > 0 else None),
        },
        'cpu_baseline': cpu,
        'cold_first_query_ms': cold['first_query_ms'] if cold else None,
        'cold_start': cold,
        'compact': compact,
        'c5': None,
    }
    if not args.no_c5:
        _run_c5_guarded(line, lambda: _c5_ranks(args, comm, dev, ws, rank, min(args.steps, 10), min(args.warmup, 3)),
                        comm, rank, ws, args.c5_timeout)
    comm.close()
    if rank != 0:
        return 0
    print(json.dumps(line), flush=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
