"""The bqueryd worker calc path on the GPU (replaces bqueryd/worker.py:269-348).

``CalcPath.handle_work(msg)`` has the contract of ``WorkerNode.handle_work``: it reads
``[filename, groupby_col_list, aggregation_list, where_terms_list]`` and the kwargs
``expand_filter_column`` / ``aggregate`` (default True) from the message
(worker.py:277-284), runs the shard's calc on the GPU, and returns the message with
``msg['data']`` = the bytes of a tar holding one bcolz ctable directory named ``result_*``
(worker.py:335-346) -- or ``''`` when the factorization check proves no row can pass
(worker.py:298-301).  Errors propagate as exceptions, so the unchanged
``WorkerBase.handle_in`` turns them into an ``ErrorMessage`` (worker.py:171-176).

Shards stay resident in HBM between messages (LRU by bytes, keyed by path and mtime): the
GPU analogue of bquery's ``auto_cache`` factor caches (worker.py:291), which are written too.
The result tar is built in memory (same members as ``tarfile.add(tmp_dir)``; no temporary
directory or tar file on disk).

Node-level calc (co-located shards): a message whose ``args[0]`` is a LIST of
the node's shard files, sent with an explicit ``aggregate=True``, is answered with ONE result
tar holding the merged table -- every shard's groupby on the node's GPUs (one pass over the
union of a GPU's shards for sum / count), summed by key across the GPUs over RCCL
(``dist.merge_group_device``).  The client's ``aggregate=True`` merge is a sum of the shard
tables it receives (rpc.py:164-173), so a pre-summed table merges to the same answer.  The
per-file message stays the default; INTEGRATION.md §4 shows the controller side.
"""
from __future__ import annotations

import os
import random
import shutil
import string
import time
from collections import OrderedDict

import numpy as np

from . import bcolz_io
from .ctable import ctable
from .engine import get_device, is_string


def rm_file_or_dir(path, ignore_errors=True):
    """bqueryd/tool.py:16-27."""
    if path is None or not os.path.exists(path):
        return
    if os.path.isdir(path) and not os.path.islink(path):
        shutil.rmtree(path, ignore_errors=ignore_errors)
    else:
        try:
            os.remove(path)
        except OSError:
            if not ignore_errors:
                raise


def result_name():
    """The archive name of a result ctable: like ``tempfile.mkdtemp(prefix='result_')``."""
    return 'result_' + ''.join(random.choice(string.ascii_lowercase + string.digits + '_') for _ in range(8))


class ShardCache:
    """Device-resident shards, least-recently-used eviction by resident bytes.  ``extra`` (set
    by the node-level state) holds the other HBM this cache's budget covers -- the co-located
    unions of the cached shards: ``extra.bytes()`` is what they hold, ``extra.drop_oldest()``
    frees one (False when none is left), ``extra.forget(ct)`` drops the ones built over an
    evicted shard."""

    def __init__(self, budget_bytes=None, device=None):
        self.budget = budget_bytes if budget_bytes is not None else int(
            float(os.environ.get('BQGPU_CACHE_GB', '64')) * (1 << 30))
        self.device = device
        self._items = OrderedDict()
        self._real = {}  # rootdir -> realpath (resolved once: a warm message's largest file-system cost)
        self.extra = None

    def _key(self, rootdir):
        real = self._real.get(rootdir)
        if real is None:
            real = self._real[rootdir] = os.path.realpath(rootdir)
        try:
            return (real, os.stat(os.path.join(rootdir, '__rootdirs__')).st_mtime_ns)
        except OSError:
            return (real, None)

    def open(self, rootdir):
        key = self._key(rootdir)
        ct = self._items.pop(key, None)
        if ct is None:
            ct = ctable(rootdir=rootdir, mode='r', auto_cache=True, device=self.device)
        self._items[key] = ct
        self._evict()
        return ct

    def _resident(self, ct):
        # what the table holds in HBM, its compact resident copies included (a copy is built by
        # the first query that reads it)
        t = ct._table
        return 0 if t is None or not getattr(t, 'handle', None) else t.device_bytes()

    def resident_bytes(self):
        return sum(self._resident(c) for c in self._items.values()) + (self.extra.bytes() if self.extra else 0)

    def _evict(self):
        # unions go first (they are rebuilt from resident shards), then the least recently
        # used shards, always keeping the one just opened
        while self.resident_bytes() > self.budget:
            if self.extra and self.extra.drop_oldest():
                continue
            if len(self._items) <= 1:
                break
            _, ct = self._items.popitem(last=False)
            if self.extra:
                self.extra.forget(ct)
            ct.close()


def _gpu_ordinals():
    """GPUs of a node-level calc: ``BQGPU_DEVICES`` (comma-separated ordinals), else all."""
    env = os.environ.get('BQGPU_DEVICES')
    if env:
        return [int(x) for x in env.split(',') if x.strip()]
    from .engine import device_count
    return list(range(device_count()))


class CalcPath:
    """Drop-in for the calc part of ``WorkerNode`` (worker.py:269-348)."""

    def __init__(self, data_dir, device=None, cache=None):
        self.data_dir = data_dir
        self.device = device or get_device()
        self.cache = cache if cache is not None else ShardCache(device=self.device)
        self._node = None  # node-level state, created by the first multi-file message
        self.last_stages = {}  # host wall time per stage of the last message

    def handle_work(self, msg):
        if msg.isa('execute_code'):
            raise NotImplementedError('execute_code stays on the reference WorkerNode')
        args, kwargs = msg.get_args_kwargs()
        filename, groupby_col_list, aggregation_list, where_terms_list = args[0], args[1], args[2], args[3]
        expand_filter_column = kwargs.get('expand_filter_column')
        aggregate = kwargs.get('aggregate', True)
        if isinstance(filename, (list, tuple)):
            return self._handle_node(msg, list(filename), groupby_col_list, aggregation_list, where_terms_list,
                                     kwargs)

        rootdir = os.path.join(self.data_dir, filename)
        if not os.path.exists(rootdir):
            raise Exception('Path %s does not exist' % rootdir)
        t0 = time.perf_counter()
        ct = self.cache.open(rootdir)
        t1 = time.perf_counter()
        result = _shard_calc(ct, groupby_col_list, aggregation_list, where_terms_list, expand_filter_column,
                             aggregate)
        t2 = time.perf_counter()
        msg['data'] = '' if result is None else bcolz_io.ctable_tar(result, result_name())
        # per-message stage timings (the reference only logs the RPC's wall time)
        self.last_stages = {'open_s': t1 - t0, 'calc_s': t2 - t1, 'result_tar_s': time.perf_counter() - t2,
                            'groups': 0 if result is None else len(next(iter(result.values()), ()))}
        return msg

    # ---- node-level calc (co-located shards)
    def _handle_node(self, msg, filenames, groupby_col_list, aggregation_list, where_terms_list, kwargs):
        from . import dist
        if kwargs.get('aggregate') is not True:
            raise ValueError('a node-level calc (a list of files) needs an explicit aggregate=True: '
                             'only the client\'s aggregate=True merge sums shard results (rpc.py:164-173)')
        if not filenames:
            raise ValueError('a node-level calc needs at least one file')
        for x in aggregation_list:
            if not (isinstance(x, (list, tuple)) and len(x) == 3):
                raise ValueError('aggregate=True needs [in_col, op, out_col] aggregations (rpc.py:171)')
        expand_filter_column = kwargs.get('expand_filter_column')
        node = self._node_state()
        for fn in filenames:
            if not os.path.exists(os.path.join(self.data_dir, fn)):
                raise Exception('Path %s does not exist' % os.path.join(self.data_dir, fn))
        per_rank = [[] for _ in node.devices]
        shards = [[] for _ in node.devices]
        for fn in sorted(filenames):
            rootdir = os.path.join(self.data_dir, fn)
            r = node.place(rootdir)
            ct = node.caches[r].open(rootdir)
            if where_terms_list and not ct.where_terms_factorization_check(where_terms_list):
                continue  # this shard's reply would be '' (worker.py:298-301): nothing to merge
            shards[r].append(ct)
        t_open = time.perf_counter()
        names = list(groupby_col_list) + [x[2] for x in aggregation_list]
        if any(is_string(ct.cols[c]) for cts in shards for ct in cts for c in groupby_col_list):
            # string keys: every shard's dictionary codes are its own, so the shard results
            # merge on the host values (the client's re-group, rpc.py:164-173, on the GPU)
            from .rpc import merge_tables
            per = []
            for cts in shards:
                for ct in cts:
                    res = _shard_calc(ct, groupby_col_list, aggregation_list, where_terms_list, expand_filter_column,
                                      True)
                    if res is not None:
                        per.append(res)
            t_calc = time.perf_counter()
            merged = merge_tables(per, groupby_col_list, aggregation_list, aggregate=True, device=self.device)
            t_merge = time.perf_counter()
            msg['data'] = '' if merged is None else bcolz_io.ctable_tar(
                OrderedDict((n, np.asarray(merged[n])) for n in names), result_name())
            msg['filenames'] = list(filenames)
            self.last_stages = {'calc_s': t_calc - t_open, 'merge_s': t_merge - t_calc,
                                'result_tar_s': time.perf_counter() - t_merge}
            return msg
        dtypes = None
        # one pass over a GPU's shard union for decomposable aggregations -- not over string
        # columns, whose dictionary codes differ per shard (the union concatenates codes)
        used = list(groupby_col_list) + [x[0] for x in aggregation_list] + [t[0] for t in (where_terms_list or [])]
        fused = dist.decomposable(aggregation_list) and not expand_filter_column and not any(
            is_string(ct.cols[c]) for cts in shards for ct in cts for c in used if c in ct.cols)
        reduced = fused
        for r, cts in enumerate(shards):
            if not cts:
                continue
            if fused:
                cols = list(dict.fromkeys(list(groupby_col_list) + [x[0] for x in aggregation_list] +
                                          [t[0] for t in (where_terms_list or [])]))
                tables = [ct._ensure_device(cols) for ct in cts]
                for ct in cts:
                    ct._auto_cache(groupby_col_list)
                colo = node.colocated(r, cts, tables)
                union = colo.union(cols)
                per_rank[r].append(union.groupby_table(groupby_col_list, aggregation_list,
                                                       where_terms=where_terms_list or None))
                node.union_built(r)
            else:
                for ct in cts:
                    t = _shard_calc_device(ct, groupby_col_list, aggregation_list, where_terms_list,
                                           expand_filter_column)
                    if t is not None:
                        per_rank[r].append(t)
            if dtypes is None and per_rank[r]:
                t0 = per_rank[r][0]
                dtypes = OrderedDict((n, t0.dtypes[n]) for n in t0.names)
        t_calc = time.perf_counter()
        try:
            if dtypes is None:
                msg['data'] = ''  # no shard can contribute a row
                return msg
            merged = dist.merge_group_device(per_rank, groupby_col_list, aggregation_list, dtypes, node.group,
                                             reduced=reduced)
        finally:
            for tabs in per_rank:
                for t in tabs:
                    t.close()
        t_merge = time.perf_counter()
        merged = OrderedDict((n, np.asarray(merged[n])) for n in names)
        msg['data'] = bcolz_io.ctable_tar(merged, result_name())
        msg['filenames'] = list(filenames)
        self.last_stages = {'calc_s': t_calc - t_open, 'merge_s': t_merge - t_calc,
                            'result_tar_s': time.perf_counter() - t_merge, 'groups': len(merged[names[0]])}
        return msg

    def _node_state(self):
        if self._node is None:
            self._node = _NodeState(_gpu_ordinals(), self.device)
        return self._node


class _NodeState:
    """The GPUs of a node-level calc: one context, shard cache and RCCL rank per GPU (one
    process driving all of them: ``bqg_comm_init_all``), stable shard placement (a file
    stays on the GPU that first loaded it; new files go to the GPU holding the fewest rows),
    and the co-located unions of each GPU's shard sets."""

    def __init__(self, ordinals, default_device):
        from . import dist
        from .engine import Device
        if not ordinals:
            raise RuntimeError('no GPU for a node-level calc')
        self.devices = [default_device if o == default_device.ordinal else Device(o) for o in ordinals]
        self.caches = [ShardCache(device=d) for d in self.devices]
        self.group = dist.CommGroup(self.devices, transport='rccl')
        self._place = {}
        self._rows = [0] * len(self.devices)
        self._unions = OrderedDict()
        for r, c in enumerate(self.caches):
            c.extra = _RankUnions(self, r)

    def place(self, rootdir):
        r = self._place.get(rootdir)
        if r is None:
            r = min(range(len(self.devices)), key=lambda i: self._rows[i])
            self._place[rootdir] = r
            try:
                self._rows[r] += bcolz_io.ctable_len(rootdir) + 1
            except (OSError, ValueError, KeyError):
                self._rows[r] += 1
        return r

    def colocated(self, rank, cts, tables):
        from . import dist
        key = (rank, tuple(id(c) for c in cts))
        colo = self._unions.pop(key, None)
        if colo is None or [id(t) for t in colo.tables] != [id(t) for t in tables]:
            if colo is not None:
                colo.close()
            colo = dist.ColocatedShards(tables)
            colo.members = list(cts)
        self._unions[key] = colo
        while len(self._unions) > 4:
            _, old = self._unions.popitem(last=False)
            old.close()
        return colo

    def union_built(self, rank):
        """A union of ``rank`` was (re)built: its bytes now count against that GPU's cache."""
        self.caches[rank]._evict()


class _RankUnions:
    """The co-located unions of one GPU, as the ``extra`` HBM of its shard cache."""

    def __init__(self, node, rank):
        self.node, self.rank = node, rank

    def _mine(self):
        return [(k, c) for k, c in self.node._unions.items() if k[0] == self.rank]

    def bytes(self):
        return sum(c.resident_bytes() for _, c in self._mine())

    def drop_oldest(self):
        mine = [(k, c) for k, c in self._mine() if c.resident_bytes()]
        if not mine:
            return False
        k, c = mine[0]
        del self.node._unions[k]
        c.close()
        return True

    def forget(self, ct):
        for k, c in self._mine():
            if any(m is ct for m in getattr(c, 'members', ())):
                del self.node._unions[k]
                c.close()


def _shard_mask(ct, where_terms_list, expand_filter_column):
    """(proceed, bool_arr): the worker's filter preparation (worker.py:293-307)."""
    if not where_terms_list:
        bool_arr = None
    else:
        if not ct.where_terms_factorization_check(where_terms_list):
            return False, None
        bool_arr = ct.where_terms(where_terms_list, cache=True)
    if expand_filter_column:
        bool_arr = ct.is_in_ordered_subgroups(basket_col=expand_filter_column, bool_arr=bool_arr)
    return True, bool_arr


def _shard_calc(ct, groupby_col_list, aggregation_list, where_terms_list, expand_filter_column, aggregate):
    """One shard's result columns (worker.py:291-323), or None for the '' early-out."""
    ok, bool_arr = _shard_mask(ct, where_terms_list, expand_filter_column)
    if not ok:
        return None
    if aggregate:
        return ct.groupby(groupby_col_list, aggregation_list, bool_arr=bool_arr).columns
    column_list = list(groupby_col_list) + [x[0] for x in aggregation_list]
    return ct.select(column_list, bool_arr=bool_arr).columns


def _shard_calc_device(ct, groupby_col_list, aggregation_list, where_terms_list, expand_filter_column):
    """One shard's aggregate=True result kept in HBM (a ShardTable)."""
    ok, bool_arr = _shard_mask(ct, where_terms_list, expand_filter_column)
    if not ok:
        return None
    return ct.groupby_device(groupby_col_list, aggregation_list, bool_arr=bool_arr)


def tar_directory(path):
    """``tarfile.open(mode='w').add(path, arcname=basename(path))`` -> bytes (worker.py:337-345)."""
    import io
    import tarfile
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode='w') as archive:
        archive.add(path, arcname=os.path.basename(path))
    return buf.getvalue()
