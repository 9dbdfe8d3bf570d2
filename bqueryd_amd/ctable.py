"""GPU ``ctable``: the bquery.ctable interface the bqueryd calc path uses, on libbqgpu.

The worker (``bqueryd/worker.py:291-323``) and the client (``bqueryd/rpc.py:158-175``) call
exactly these members of ``bquery.ctable`` [ext-bquery, unverified -- bquery is not vendored,
SURVEY.md §8c]:

  ctable(rootdir=..., mode='r', auto_cache=True)                  worker.py:291
  ct.where_terms_factorization_check(where_terms_list)            worker.py:298
  ct.where_terms(where_terms_list, cache=True)                    worker.py:303
  ct.is_in_ordered_subgroups(basket_col=..., bool_arr=...)        worker.py:307
  ct.groupby(groupby_cols, agg_list, bool_arr=..., rootdir=...)   worker.py:313, rpc.py:172
  ct[column_list].where(bool_arr) / ct[column_list]               worker.py:319-323
  ct.free_cachemem(), ct.clean_tmp_rootdir()                      worker.py:330-331
  result.flush(), result.free_cachemem(), result.todataframe()    worker.py:335-336, rpc.py:173

Columns are decoded from the bcolz rootdir on host threads only when a query first touches
them, then stay resident in HBM (``ShardTable``).  ``where_terms`` returns a lazy mask: when it
is passed straight to ``groupby`` the predicate is fused into the groupby scan (one pass over
HBM); it is only materialised when something needs the rows (basket expansion, raw rows,
``numpy.asarray``).
"""
from __future__ import annotations

import os
from collections import OrderedDict

import numpy as np

from . import bcolz_io
from .engine import ShardTable, get_device, is_string
from .terms import any_value_satisfies, parse_terms


class WhereMask:
    """Result of ``ctable.where_terms``: lazy, device-resident boolean row mask."""

    def __init__(self, ct, terms=None, device_col=None, npass=None):
        self.ct = ct
        self.terms = list(terms) if terms is not None else None
        self.device_col = device_col  # a scratch mask column this object owns
        self._table = ct._table if device_col is not None else None
        self._npass = npass

    def materialize(self):
        if self.device_col is None:
            self._table = self.ct._table_for_terms(self.terms)
            self.device_col, self._npass = self._table.where(self.terms)
        return self.device_col

    def __del__(self):
        # the mask column goes back to the shard's free list (the shard stays resident in
        # HBM between queries: worker.ShardCache)
        try:
            if self.device_col is not None and self._table is not None:
                self._table.release_mask(self.device_col)
        except Exception:
            pass

    def sum(self):
        self.materialize()
        return self._npass

    def all(self):
        return self.sum() == len(self)

    def __len__(self):
        return len(self.ct)

    def __array__(self, dtype=None, copy=None):
        col = self.materialize()
        arr = self.ct._table.read(col)
        return arr if dtype is None else arr.astype(dtype)


class ResultTable:
    """A host-side result table (what ``ct.groupby(..., rootdir=...)`` returns)."""

    def __init__(self, columns, rootdir=None):
        self.columns = OrderedDict(columns)
        self.rootdir = rootdir
        self._written = False

    @property
    def names(self):
        return list(self.columns.keys())

    def __len__(self):
        return len(next(iter(self.columns.values()))) if self.columns else 0

    def __getitem__(self, name):
        return self.columns[name]

    def flush(self):
        if self.rootdir and not self._written:
            bcolz_io.write_ctable(self.rootdir, self.columns)
            self._written = True

    def free_cachemem(self):
        pass

    def todataframe(self):
        import pandas as pd
        return pd.DataFrame(OrderedDict((k, v) for k, v in self.columns.items()))


class ctable:  # noqa: N801  (mirrors bquery's class name)
    """bquery.ctable replacement backed by HBM-resident columns."""

    def __init__(self, columns=None, rootdir=None, mode='r', auto_cache=False, device=None):
        self.rootdir = rootdir
        self.mode = mode
        self.auto_cache = auto_cache
        self.device = device or get_device()
        self._host = OrderedDict()
        if columns is not None:
            for k, v in columns.items():
                self._host[k] = np.ascontiguousarray(v)
            self._dtypes = OrderedDict((k, v.dtype) for k, v in self._host.items())
            self._len = len(next(iter(self._host.values()))) if self._host else 0
        elif rootdir is not None:
            if not os.path.isdir(rootdir):
                raise Exception('Path %s does not exist' % rootdir)
            self._dtypes = bcolz_io.ctable_dtypes(rootdir)
            self._len = bcolz_io.ctable_len(rootdir)
        else:
            raise ValueError('ctable needs columns or a rootdir')
        self._table = None

    # ---- columns
    @property
    def names(self):
        return list(self._dtypes.keys())

    @property
    def cols(self):
        return self._dtypes

    def __len__(self):
        return self._len

    @property
    def len(self):
        return self._len

    def _host_column(self, name):
        if name not in self._dtypes:
            raise KeyError(str(name))
        if name not in self._host:
            self._host[name] = bcolz_io.read_carray(bcolz_io.ctable_column_dir(self.rootdir, name))
        return self._host[name]

    def __getitem__(self, name):
        return self._host_column(name)

    def _ensure_device(self, names):
        """Make sure the named columns are resident in HBM; returns the ShardTable."""
        names = [n for n in OrderedDict.fromkeys(names)]
        for n in names:
            if n not in self._dtypes:
                raise KeyError(str(n))
        if self._table is None:
            self._table = ShardTable(OrderedDict(), device=self.device, nrows=self._len)
        missing = [n for n in names if n not in self._table.dtypes]
        cold = []
        for n in missing:
            self._table.add_column(n, self._dtypes[n])
            self._table.names.append(n)
            if n in self._host or is_string(self._dtypes[n]):
                # string columns: decoded on the host, dictionary-encoded on the GPU
                self._table.push(n, self._host_column(n))
                if is_string(self._dtypes[n]) and self.rootdir:
                    self._host.pop(n, None)
            else:
                meta = bcolz_io.CArrayMeta(bcolz_io.ctable_column_dir(self.rootdir, n))
                if meta.length != self._len:
                    raise ValueError('column %s has %d rows, table has %d' % (n, meta.length, self._len))
                cold.append((n, meta.rootdir, meta.chunklen))
        if cold:
            # cold path: the bcolz chunks of every missing column, straight into HBM in one call
            self._table.load_carrays(cold)
        if missing:
            self._table.sync()
        return self._table

    def _table_for_terms(self, terms):
        return self._ensure_device([t[0] for t in parse_terms(self._dtypes, terms)])

    # ---- where terms
    def where_terms(self, term_list, cache=False):
        parse_terms(self._dtypes, term_list)  # validate eagerly (KeyError / ValueError)
        return WhereMask(self, terms=term_list)

    def where_terms_factorization_check(self, term_list):
        """False iff a term's column has a factor cache (``<col>.values``) in the rootdir and
        none of the cached values can satisfy the term; the first term without a cache ends
        the check [ext-bquery, unverified].  The cached values (a few per column) are read
        once per cache directory and tested on the host."""
        terms = parse_terms(self._dtypes, term_list)
        for col, code, value in terms:
            vals = self._cached_values(col)
            if vals is None:
                break
            if not any_value_satisfies(np.asarray(vals).astype(self._dtypes[col]), code, value):
                return False
        return True

    # ---- factor caches (bquery auto_cache: <col>.factor / <col>.values next to the columns)
    def cache_valid(self, col):
        """bquery's test: the column and its ``.values`` cache both exist."""
        if not self.rootdir:
            return False
        coldir = bcolz_io.ctable_column_dir(self.rootdir, col)
        return os.path.exists(os.path.join(coldir, '__attrs__')) and os.path.exists(
            os.path.join(coldir + '.values', '__attrs__'))

    def _cached_values(self, col):
        if not self.rootdir:
            return None
        values_dir = bcolz_io.ctable_column_dir(self.rootdir, col) + '.values'
        try:
            key = os.stat(os.path.join(values_dir, '__attrs__')).st_mtime_ns
        except OSError:
            return None
        memo = self.__dict__.setdefault('_values_memo', {})
        hit = memo.get(col)
        if hit is None or hit[0] != key:
            hit = memo[col] = (key, bcolz_io.read_carray(values_dir))
        return hit[1]

    def _auto_cache(self, cols):
        """bquery's ``auto_cache=True`` side effect of a groupby (worker.py:291): the factor
        caches of every groupby column that has none -- labels and values from the GPU
        (``bqg_factorize``), compressed and written by a background thread into temporary
        directories next to the columns and renamed into place (.factor before .values, so a
        valid cache always has both).  Every key dtype is cached: integer columns spanning at
        most 2^27 values through a lookup table, floats (khash identity), bools and wider
        spans through a hash of the canonical key bits."""
        if not (self.auto_cache and self.rootdir and os.access(self.rootdir, os.W_OK)):
            return
        pending = self.__dict__.setdefault('_caching', set())
        for col in cols:
            if col in pending or self.cache_valid(col):
                continue
            try:
                labels, values = self._ensure_device([col]).factorize(col)
            except NotImplementedError:
                continue
            pending.add(col)
            _cache_writer().submit(_write_factor_cache, self.rootdir, col, labels, values)

    def flush_caches(self):
        """Wait until the factor caches this process scheduled are on disk."""
        _cache_writer().submit(lambda: None).result()

    def is_in_ordered_subgroups(self, basket_col=None, bool_arr=None, _max_len_subgroup=1000):
        if basket_col is None:
            raise AssertionError('basket_col is required')
        if bool_arr is None:
            return None
        table = self._ensure_device([basket_col])
        mcol, temp = self._mask_column(bool_arr)
        try:
            out = table.expand_subgroups(basket_col, mcol)
        finally:
            if temp:
                table.release_mask(mcol)
        return WhereMask(self, device_col=out)

    def _mask_column(self, bool_arr):
        """(device BOOL column holding ``bool_arr``, temporary): lazy masks are materialised
        and stay owned by their WhereMask; a host array goes to a scratch column the caller
        releases after the query."""
        if isinstance(bool_arr, WhereMask):
            return bool_arr.materialize(), False
        arr = np.ascontiguousarray(np.asarray(bool_arr, dtype=bool))
        if len(arr) != self._len:
            raise ValueError('bool_arr length %d != table length %d' % (len(arr), self._len))
        table = self._ensure_device([])
        name = table.scratch_mask()
        table.push(name, arr)
        return name, True

    # ---- calc
    def groupby(self, groupby_cols, agg_list, bool_arr=None, rootdir=None):
        from .terms import parse_agg_list
        groupby_cols = list(groupby_cols)
        ops = parse_agg_list(self._dtypes, agg_list)
        needed = groupby_cols + [o[0] for o in ops]
        terms, mask = None, None
        if isinstance(bool_arr, WhereMask) and bool_arr.device_col is None:
            terms = bool_arr.terms  # fuse the predicate into the groupby scan
            needed += [t[0] for t in parse_terms(self._dtypes, terms)]
        table = self._ensure_device(needed)
        self._auto_cache(groupby_cols)
        temp = False
        if bool_arr is not None and terms is None:
            mask, temp = self._mask_column(bool_arr)
        try:
            out, _ = table.groupby(groupby_cols, agg_list, where_terms=terms, mask=mask)
        finally:
            if temp:
                table.release_mask(mask)
        res = ResultTable(out, rootdir=rootdir)
        if rootdir:
            res.flush()
        return res

    def groupby_device(self, groupby_cols, agg_list, bool_arr=None):
        """``groupby`` whose result stays in HBM (a ShardTable: keys, then aggregations) -- the
        input of the node-level merge (worker.CalcPath, dist.merge_group_device)."""
        from .terms import parse_agg_list
        groupby_cols = list(groupby_cols)
        ops = parse_agg_list(self._dtypes, agg_list)
        needed = groupby_cols + [o[0] for o in ops]
        terms, mask = None, None
        if isinstance(bool_arr, WhereMask) and bool_arr.device_col is None:
            terms = bool_arr.terms
            needed += [t[0] for t in parse_terms(self._dtypes, terms)]
        table = self._ensure_device(needed)
        self._auto_cache(groupby_cols)
        temp = False
        if bool_arr is not None and terms is None:
            mask, temp = self._mask_column(bool_arr)
        try:
            return table.groupby_table(groupby_cols, agg_list, where_terms=terms, mask=mask)
        finally:
            if temp:
                table.release_mask(mask)

    def select(self, column_list, bool_arr=None, rootdir=None):
        """``bcolz.fromiter(ct[column_list].where(bool_arr), ...)`` (worker.py:316-323)."""
        column_list = list(column_list)
        terms, mask = None, None
        needed = list(column_list)
        if isinstance(bool_arr, WhereMask) and bool_arr.device_col is None:
            terms = bool_arr.terms
            needed += [t[0] for t in parse_terms(self._dtypes, terms)]
        table = self._ensure_device(needed)
        temp = False
        if bool_arr is not None and terms is None:
            mask, temp = self._mask_column(bool_arr)
        try:
            out = table.select_rows(column_list, where_terms=terms, mask=mask)
        finally:
            if temp:
                table.release_mask(mask)
        res = ResultTable(out, rootdir=rootdir)
        if rootdir:
            res.flush()
        return res

    # ---- bookkeeping (worker.py:330-331)
    def free_cachemem(self):
        self._host.clear() if self.rootdir else None

    def clean_tmp_rootdir(self):
        pass

    def close(self):
        if self._table is not None:
            self._table.close()
            self._table = None

    def todataframe(self):
        import pandas as pd
        return pd.DataFrame(OrderedDict((n, self._host_column(n)) for n in self.names))


_writer = None


def _cache_writer():
    """One background thread writes factor caches (the worker stays single-threaded)."""
    global _writer
    if _writer is None:
        from concurrent.futures import ThreadPoolExecutor
        _writer = ThreadPoolExecutor(max_workers=1, thread_name_prefix='bqgpu-cache')
    return _writer


def _write_factor_cache(rootdir, col, labels, values):
    import shutil
    import tempfile
    coldir = bcolz_io.ctable_column_dir(rootdir, col)
    for suffix, arr in (('.factor', labels), ('.values', values)):
        tmp = tempfile.mkdtemp(prefix='.bqgpu-cache-', dir=rootdir)
        try:
            bcolz_io.write_carray(tmp, arr)
            final = coldir + suffix
            if os.path.exists(final):
                shutil.rmtree(final, ignore_errors=True)
            os.rename(tmp, final)
        except OSError:
            shutil.rmtree(tmp, ignore_errors=True)
            return
