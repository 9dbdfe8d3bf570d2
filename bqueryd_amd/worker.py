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
GPU analogue of bquery's ``auto_cache`` factor caches (worker.py:291).
"""
from __future__ import annotations

import io
import os
import shutil
import tarfile
import tempfile
from collections import OrderedDict

from .ctable import ctable
from .engine import get_device


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


class ShardCache:
    """Device-resident shards, least-recently-used eviction by resident bytes."""

    def __init__(self, budget_bytes=None, device=None):
        self.budget = budget_bytes if budget_bytes is not None else int(
            float(os.environ.get('BQGPU_CACHE_GB', '64')) * (1 << 30))
        self.device = device
        self._items = OrderedDict()

    def _key(self, rootdir):
        try:
            st = os.stat(os.path.join(rootdir, '__rootdirs__'))
            return (os.path.realpath(rootdir), st.st_mtime_ns)
        except OSError:
            return (os.path.realpath(rootdir), None)

    def open(self, rootdir):
        key = self._key(rootdir)
        ct = self._items.pop(key, None)
        if ct is None:
            ct = ctable(rootdir=rootdir, mode='r', auto_cache=True, device=self.device)
        self._items[key] = ct
        self._evict()
        return ct

    def _resident(self, ct):
        t = ct._table
        return 0 if t is None else sum(t.nrows * dt.itemsize for dt in t.dtypes.values())

    def _evict(self):
        while len(self._items) > 1 and sum(self._resident(c) for c in self._items.values()) > self.budget:
            _, ct = self._items.popitem(last=False)
            ct.close()


class CalcPath:
    """Drop-in for the calc part of ``WorkerNode`` (worker.py:269-348)."""

    def __init__(self, data_dir, device=None, cache=None):
        self.data_dir = data_dir
        self.device = device or get_device()
        self.cache = cache if cache is not None else ShardCache(device=self.device)

    def handle_work(self, msg):
        if msg.isa('execute_code'):
            raise NotImplementedError('execute_code stays on the reference WorkerNode')
        tmp_dir = tempfile.mkdtemp(prefix='result_')
        args, kwargs = msg.get_args_kwargs()
        filename, groupby_col_list, aggregation_list, where_terms_list = args[0], args[1], args[2], args[3]
        expand_filter_column = kwargs.get('expand_filter_column')
        aggregate = kwargs.get('aggregate', True)

        rootdir = os.path.join(self.data_dir, filename)
        if not os.path.exists(rootdir):
            rm_file_or_dir(tmp_dir)
            raise Exception('Path %s does not exist' % rootdir)
        try:
            ct = self.cache.open(rootdir)
            if not where_terms_list:
                bool_arr = None
            else:
                if not ct.where_terms_factorization_check(where_terms_list):
                    msg['data'] = ''
                    return msg
                bool_arr = ct.where_terms(where_terms_list, cache=True)
            if expand_filter_column:
                bool_arr = ct.is_in_ordered_subgroups(basket_col=expand_filter_column, bool_arr=bool_arr)
            rm_file_or_dir(tmp_dir)
            if aggregate:
                result = ct.groupby(groupby_col_list, aggregation_list, bool_arr=bool_arr, rootdir=tmp_dir)
            else:
                column_list = list(groupby_col_list) + [x[0] for x in aggregation_list]
                result = ct.select(column_list, bool_arr=bool_arr, rootdir=tmp_dir)
            result.flush()
            msg['data'] = tar_directory(tmp_dir)
            return msg
        finally:
            rm_file_or_dir(tmp_dir)


def tar_directory(path):
    """``tarfile.open(mode='w').add(path, arcname=basename(path))`` -> bytes (worker.py:337-345)."""
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode='w') as archive:
        archive.add(path, arcname=os.path.basename(path))
    return buf.getvalue()
