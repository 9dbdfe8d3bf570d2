"""CPU cluster baseline: the reference's deployment shape timed on the host cores --
TEST / BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

bqueryd runs one controller and N single-threaded calc workers per node
(``misc/supervisor.conf:21``: 10 workers; ``bcolz.set_nthreads(1)``, ``worker.py:40``).  The
controller sends one calc message per shard file to a free worker (``controller.py:471-508``,
``controller.py:113-144``), every worker answers with its shard's finalized table
(``worker.py:269-348``), and the client sums them by key (``rpc.py:164-173``).  Here:

* N worker processes (``multiprocessing`` spawn context), each running the C port of bquery's
  per-shard groupby (``oracle/cbquery.c``: materialised where mask, khash factorize, filter
  re-factorize, one pass per aggregation; single-threaded);
* the parent is the controller (a shared queue hands out one shard index per message, so a
  free worker takes the next shard) and the client (``bquery_oracle.client_merge`` with
  ``aggregate=True`` over the replies);
* shards are the bench's synthetic taxi shards, written before the timed region as bcolz
  ctables (a node's data dir: any free worker can take any shard); the worker that takes a
  message reads and blosc-decodes the shard's columns on its one thread, as the reference's
  worker does, then runs the C port.  A second timing hands the workers the decoded columns
  through shared memory: the compute of the calc path alone.

Timed: from the first dispatched message to the merged table on the client.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import platform
import time


def _worker(wid, layout, files, cfg, tasks, results, ready):
    import numpy as np
    from multiprocessing import shared_memory
    from oracle import cbquery
    cbquery.lib()
    blocks, data = [], {}
    if files is None:
        # decoded shards, shared read-only by every worker
        for i, cols in layout.items():
            data[i] = {}
            for name, (shm_name, dtype, n) in cols.items():
                shm = shared_memory.SharedMemory(name=shm_name)
                blocks.append(shm)
                data[i][name] = np.ndarray((n,), dtype=np.dtype(dtype), buffer=shm.buf)
    else:
        from bqueryd_amd import bcolz_io
        bcolz_io.blosc()
    ready.put(wid)
    while True:
        i = tasks.get()
        if i is None:
            break
        if files is None:
            cols = data[i]
        else:
            # the shard's bcolz columns, blosc-decoded on this worker's one thread
            # (bcolz.set_nthreads(1), worker.py:40) -- what bquery iterates over
            cols = bcolz_io.read_ctable(files[i], columns=list(layout[i]), nthreads=1)
        out = cbquery.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where'])
        results.put((i, {k: np.array(v) for k, v in out.items()}))
    data.clear()
    for shm in blocks:
        shm.close()


def host_cores():
    """CPU cores this process may use: the affinity set, capped by OMP_NUM_THREADS when set
    (the GPU box exports the box's CPU share there)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get('OMP_NUM_THREADS')
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def run(cfg, n_shards, rows_per_shard, worker_counts, config_id=2, variant='exact', reps=2, bcolz_dir=None):
    """Time one aggregate=True query over ``n_shards`` shards with each worker count in
    ``worker_counts``; returns {n_workers: {'decoded': (rows/s, s), 'bcolz': (rows/s, s)}} and
    the last merged table.  'decoded': the shards' columns already in (shared) memory -- the
    compute of the calc path alone; 'bcolz' (when ``bcolz_dir`` is given): the shards are
    bcolz ctables (lz4, the writer of bqueryd_amd.bcolz_io) under ``bcolz_dir``, read and
    blosc-decoded by the worker that takes the message, as the reference's worker does."""
    from multiprocessing import shared_memory

    import numpy as np

    from bqueryd_amd import synth
    from oracle import bquery_oracle as bo
    columns = synth.query_columns(cfg)
    shms, layout, out, merged, files = [], {}, {}, None, None
    if bcolz_dir is not None:
        import os as _os
        from bqueryd_amd import bcolz_io
        files = {i: _os.path.join(bcolz_dir, 'shard-%d.bcolzs' % i) for i in range(n_shards)}
    try:
        for i in range(n_shards):
            cols = synth.taxi_shard(rows_per_shard, config_id=config_id, n_shards=n_shards, shard=i,
                                    variant=variant, columns=columns)
            if files is not None:
                bcolz_io.write_ctable(files[i], cols)
            layout[i] = {}
            for name, arr in cols.items():
                shm = shared_memory.SharedMemory(create=True, size=max(1, arr.nbytes))
                shms.append(shm)
                np.ndarray(arr.shape, dtype=arr.dtype, buffer=shm.buf)[:] = arr
                layout[i][name] = (shm.name, arr.dtype.str, len(arr))
            del cols
        ctx = mp.get_context('spawn')
        for n_workers, source in [(n, src) for n in worker_counts for src in
                                  (['decoded'] + (['bcolz'] if files is not None else []))]:
            tasks, results, ready = ctx.Queue(), ctx.Queue(), ctx.Queue()
            procs = [ctx.Process(target=_worker, args=(w, layout, files if source == 'bcolz' else None, cfg,
                                                       tasks, results, ready), daemon=True)
                     for w in range(n_workers)]
            for p in procs:
                p.start()
            try:
                for _ in procs:
                    ready.get(timeout=600)
                best = None
                for _ in range(reps):
                    t0 = time.perf_counter()
                    for i in range(n_shards):  # the controller: one calc message per shard file
                        tasks.put(i)
                    replies = dict(results.get(timeout=600) for _ in range(n_shards))
                    # the client (rpc.py:151-173): glob order is file-system order; index order here
                    merged = bo.client_merge([replies[i] for i in range(n_shards)], cfg['groupby'], cfg['aggs'],
                                             aggregate=True)
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                for _ in procs:
                    tasks.put(None)
                for p in procs:
                    p.join(timeout=60)
            finally:
                for p in procs:
                    if p.is_alive():
                        p.terminate()
            out.setdefault(n_workers, {})[source] = (n_shards * rows_per_shard / best, best)
    finally:
        for shm in shms:
            shm.close()
            shm.unlink()
    return out, merged
