"""Device contexts and device-resident shard tables over libbqgpu.

``ShardTable`` is the GPU analogue of the ``bquery.ctable`` a bqueryd worker opens per shard
(``bqueryd/worker.py:291``): its columns live in HBM, and ``groupby`` / ``where`` /
``select_rows`` / ``expand_subgroups`` run the gfx950 kernels of libbqgpu.  All results come
back as numpy arrays in bquery's group order (first appearance among the passing rows).
"""
from __future__ import annotations

import ctypes
import os
from collections import OrderedDict

import numpy as np

from . import _lib as L
from .terms import normalize, parse_agg_list, parse_terms, string_term, time_value


class Device:
    """One libbqgpu context (one per GPU per host thread)."""

    def __init__(self, ordinal=0):
        self._lib = L.lib()
        h = ctypes.c_void_p()
        L.check(self._lib.bqg_create(int(ordinal), ctypes.byref(h)), None)
        self.handle = h
        self.ordinal = int(ordinal)

    def close(self):
        if self.handle:
            self._lib.bqg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc):
        L.check(rc, self.handle)

    def set_stream(self, stream_ptr):
        self.check(self._lib.bqg_set_stream(self.handle, ctypes.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        self.check(self._lib.bqg_synchronize(self.handle))

    def enable_timing(self, on=True, scan_only=False):
        """HIP-event timing of each query (``last_timing``): the scan kernels and the whole
        query, or with ``scan_only`` the scan kernels alone (``total_ms`` NaN)."""
        self.check(self._lib.bqg_enable_timing(self.handle, (2 if scan_only else 1) if on else 0))

    def last_timing(self):
        t = L.Timing()
        self.check(self._lib.bqg_last_timing(self.handle, ctypes.byref(t)))
        return {'scan_ms': t.scan_ms, 'scan_launches': t.scan_launches, 'total_ms': t.total_ms,
                'rows': t.rows, 'bytes': t.bytes, 'bytes_read': t.bytes_read, 'compact_ms': t.compact_ms,
                'scan_ms_sum': t.scan_ms_sum, 'timed_queries': t.timed_queries, 'copy_ms': t.copy_ms,
                'mode': t.mode, 'specialized': bool(t.specialized),
                'narrow': bool(t.narrow), 'pack16': t.narrow == 2, 'regrows': t.regrows}

    def set_option(self, name, value):
        """One engine option of this context (include/bqgpu.h: launch shapes and path choices,
        for tests and profiling; every value gives the same results)."""
        self.check(self._lib.bqg_set_option(self.handle, name.encode('ascii'), int(value)))

    def get_option(self, name):
        v = ctypes.c_int64()
        self.check(self._lib.bqg_get_option(self.handle, name.encode('ascii'), ctypes.byref(v)))
        return v.value

    def reset_options(self):
        self.check(self._lib.bqg_reset_options(self.handle))

    def jit_wait(self, timeout_s=None):
        """Wait for the background compiles of query-specialised kernels (option jit_async):
        ``{'idle': bool, 'compiled': n, 'failed': n}`` (``idle`` False after a timeout)."""
        idle, comp, fail = ctypes.c_int32(0), ctypes.c_int64(0), ctypes.c_int64(0)
        self.check(self._lib.bqg_jit_wait(self.handle, -1.0 if timeout_s is None else 1e3 * float(timeout_s),
                                          ctypes.byref(idle), ctypes.byref(comp), ctypes.byref(fail)))
        return {'idle': bool(idle.value), 'compiled': comp.value, 'failed': fail.value}

    def options(self, **values):
        """Context manager: the given options set for the block, the previous values restored
        after it."""
        import contextlib

        @contextlib.contextmanager
        def _cm():
            old = {k: self.get_option(k) for k in values}
            try:
                for k, v in values.items():
                    self.set_option(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_option(k, v)
        return _cm()


_devices = {}


class _Unfreezable(Exception):
    pass


_FREEZE_SCALARS = (bytes, bool, int, float, type(None))


def _freeze(x):
    """Hashable, type-exact image of a query argument (plan-cache key).  Exact-type checks
    first (this runs on every query): a plain str stands for itself, a list / tuple is a tuple
    tagged with which of the two it was; subclasses other than str / numpy scalars are not
    cached."""
    t = type(x)
    if t is str:
        return x
    if t is list or t is tuple:
        return (t is list,) + tuple([_freeze(v) for v in x])
    if t in _FREEZE_SCALARS or isinstance(x, np.generic):
        return (t, x)
    if t is set or t is frozenset:
        return ('set', frozenset([_freeze(v) for v in x]))
    if isinstance(x, str):
        return (t, x)
    raise _Unfreezable()


def device_count():
    n = ctypes.c_int()
    L.check(L.lib().bqg_device_count(ctypes.byref(n)), None)
    return n.value


def get_device(ordinal=None):
    """Process-wide cached context; ``BQGPU_DEVICE`` selects the default GPU."""
    if ordinal is None:
        ordinal = int(os.environ.get('BQGPU_DEVICE', '0'))
    dev = _devices.get(ordinal)
    if dev is None:
        dev = _devices[ordinal] = Device(ordinal)
    return dev


class _ResultHolder:
    """Owns one bqg_result; freed (its pinned block returned to the pool) when the last numpy
    view of its columns is garbage-collected."""

    def __init__(self, handle):
        self.handle = handle
        self._free = L.lib().bqg_result_free

    def __del__(self):
        if self.handle:
            self._free(self.handle)
            self.handle = None


_CHAR_ARRAYS = {}


def _char_array(n):
    """ctypes.c_char * n, created once per size (a new array type per result column costs more
    than the rest of wrapping it)."""
    t = _CHAR_ARRAYS.get(n)
    if t is None:
        if len(_CHAR_ARRAYS) > 4096:
            _CHAR_ARRAYS.clear()
        t = _CHAR_ARRAYS[n] = ctypes.c_char * n
    return t


def _result_to_columns(dev, res_handle, names):
    """Zero-copy numpy views of a result's columns (pinned host memory of the library)."""
    view = L.ResultView()
    rc = L.lib().bqg_result_view_get(res_handle, ctypes.byref(view))
    holder = _ResultHolder(res_handle)
    dev.check(rc)
    n = view.n_rows
    out = OrderedDict()
    for j, name in enumerate(names):
        dt = L.DTYPES[view.dtypes[j]]
        nbytes = n * dt.itemsize
        if nbytes == 0:
            out[name] = np.zeros(0, dtype=dt)
            continue
        buf = _char_array(nbytes).from_address(view.cols[j])
        buf._bqg_holder = holder
        out[name] = np.frombuffer(buf, dtype=dt)
    return out, bool(view.filtered)


def is_string(dt):
    """numpy fixed-width bytes ('S<n>') / unicode ('U<n>'): dictionary codes on the device."""
    return np.dtype(dt).kind in 'SU'


def is_time(dt):
    """numpy datetime64 / timedelta64: their int64 ticks on the device."""
    return np.dtype(dt).kind in 'Mm'


def device_dtype(dt):
    """The dtype a logical column has in HBM: int32 dictionary codes for strings, int64 ticks
    for datetime64 / timedelta64, the dtype itself otherwise."""
    dt = np.dtype(dt)
    if is_string(dt):
        return np.dtype(np.int32)
    if is_time(dt):
        return np.dtype(np.int64)
    return dt


class StringDict:
    """The dictionary of a string column (``bqg_encode_bytes``): ``values[code]`` -- code 0 is the
    empty string, code r + 1 the value of first-appearance rank r (so a zero-initialised code
    compares like bquery's zero-initialised string)."""

    def __init__(self, dtype, ranked):
        self.dtype = np.dtype(dtype)
        empty = np.zeros(1, self.dtype)
        self.values = np.concatenate([empty, np.asarray(ranked, self.dtype)])
        self._index = None

    def decode(self, codes):
        return self.values[np.asarray(codes)]

    def code_of(self, value):
        if self._index is None:
            self._index = {}
            for c, v in enumerate(self.values.tolist()):
                self._index.setdefault(v, c)
        return self._index.get(value)


class ShardTable:
    """Device-resident columns of one shard.  String columns ('S<n>' / 'U<n>') live in HBM as
    INT32 dictionary codes (``bqg_encode_bytes``, on the GPU) with their dictionary on the host;
    datetime64 / timedelta64 columns as their int64 ticks.  Keys, terms and results translate
    at the boundary, so every kernel sees integer columns."""

    def __init__(self, columns, device=None, nrows=None):
        """``columns``: mapping name -> 1-D numpy array (all the same length); ``nrows`` is
        required only when ``columns`` is empty (columns added later)."""
        self.dev = device or get_device()
        self._lib = L.lib()
        names = list(columns.keys())
        arrays = [np.ascontiguousarray(columns[n]) for n in names]
        n = len(arrays[0]) if arrays else int(nrows or 0)
        for a in arrays:
            if a.ndim != 1 or len(a) != n:
                raise ValueError('all columns must be 1-D arrays of the same length')
            if device_dtype(a.dtype) not in L.DTYPE_CODE:
                raise NotImplementedError('column dtype %s is not supported on the GPU' % a.dtype)
        codes = (ctypes.c_int32 * max(1, len(arrays)))(*[L.DTYPE_CODE[device_dtype(a.dtype)] for a in arrays])
        h = ctypes.c_void_p()
        self.dev.check(self._lib.bqg_table_create(self.dev.handle, n, len(arrays), codes,
                                                  ctypes.byref(h)))
        self.handle = h
        self.nrows = n
        self.names = names
        self.dtypes = OrderedDict((nm, a.dtype) for nm, a in zip(names, arrays))
        self._slot = {nm: i for i, nm in enumerate(names)}
        self._scratch = []
        self._strings = {}
        for i, a in enumerate(arrays):
            self.push(names[i], a)
        self.sync()

    @classmethod
    def _wrap(cls, handle, names, dtypes, device, strings=None):
        """A ShardTable around a table the library created (a device-resident result);
        ``strings``: the dictionaries of its string columns (codes of the table they came from)."""
        t = cls.__new__(cls)
        t.dev = device
        t._lib = L.lib()
        t.handle = handle
        n = ctypes.c_int64()
        device.check(t._lib.bqg_table_nrows(handle, ctypes.byref(n)))
        t.nrows = n.value
        t.names = list(names)
        t.dtypes = OrderedDict((nm, np.dtype(dt)) for nm, dt in zip(names, dtypes))
        t._slot = {nm: i for i, nm in enumerate(names)}
        t._scratch = []
        t._strings = dict(strings or {})
        return t

    @classmethod
    def from_parts(cls, parts, names=None, device=None):
        """One table holding the row-concatenation of ``parts`` -- mappings name -> array, or
        device-resident ShardTables -- each part copied straight to its row offset in HBM (no
        host-side concatenation; page-locked parts go by DMA without staging, device parts
        by device-to-device copies)."""
        parts = [p for p in parts if p is not None]
        names = list(names or (parts[0].names if isinstance(parts[0], ShardTable) else parts[0].keys()))

        def rows(p):
            return p.nrows if isinstance(p, ShardTable) else len(p[names[0]])

        def dtype(p, n):
            return p.dtypes[n] if isinstance(p, ShardTable) else np.asarray(p[n]).dtype

        if any(isinstance(p, ShardTable) and any(n in p._strings for n in names) for p in parts):
            raise NotImplementedError('from_parts of device string columns: their dictionaries differ per table')
        total = sum(rows(p) for p in parts)
        t = cls(OrderedDict(), device=device, nrows=total)
        for n in names:
            t.add_column(n, dtype(parts[0], n))
            t.names.append(n)
        off = 0
        for p in parts:
            m = rows(p)
            if m:
                for n in names:
                    if isinstance(p, ShardTable):
                        t.push_device(n, p.column_ptr(n), m, off)
                    else:
                        t.push(n, p[n], off)
            off += m
        t.sync()
        return t

    # ---- lifecycle
    def close(self):
        if getattr(self, 'handle', None):
            self._lib.bqg_table_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.nrows

    # ---- data movement
    def slot(self, name):
        if isinstance(name, int):
            return name
        if name not in self._slot:
            raise KeyError(str(name))
        return self._slot[name]

    @property
    def version(self):
        """Bumped by every write into the table's columns (caches over its data key on it)."""
        return self.__dict__.get('_version', 0)

    def _touch(self):
        self.__dict__['_version'] = self.version + 1
        # cached plans hold where-terms on string columns as dictionary codes: new data means a
        # new dictionary, so every plan is rebuilt
        self.__dict__.pop('_plans', None)

    def _logical(self, col):
        s = self.slot(col)
        for k, v in self._slot.items():
            if v == s:
                return k, self.dtypes[k]
        raise KeyError(str(col))

    def push(self, col, array, row_offset=0):
        self._touch()
        name, dt = self._logical(col)
        a = np.ascontiguousarray(array)
        if is_string(dt):
            return self._encode_strings(name, a.astype(dt, copy=False), row_offset)
        if is_time(dt):
            a = a.astype(dt, copy=False).view(np.int64)
        self.dev.check(self._lib.bqg_push_chunk(self.handle, self.slot(col), a.ctypes.data,
                                                len(a), int(row_offset)))

    def _encode_strings(self, name, a, row_offset):
        """A whole string column -> INT32 codes in HBM + its dictionary (bqg_encode_bytes)."""
        if row_offset != 0 or len(a) != self.nrows:
            raise NotImplementedError('string columns are pushed whole')
        a = np.ascontiguousarray(a)
        width = a.dtype.itemsize
        n_values = ctypes.c_int64()
        cap = min(len(a), 1 << 16)
        for _ in range(2):
            values = np.empty(max(cap, 1), dtype=a.dtype)
            rc = self._lib.bqg_encode_bytes(self.dev.handle, self.handle, self.slot(name), a.ctypes.data, width,
                                            values.ctypes.data, len(values), ctypes.byref(n_values))
            if rc == 0 or n_values.value <= len(values):
                break
            cap = n_values.value  # more distinct values than the first guess: once more, sized
        self.dev.check(rc)
        self._strings[name] = StringDict(a.dtype, values[:n_values.value])

    def push_device(self, col, dev_ptr, nrows, row_offset=0):
        """Device-to-device copy of ``nrows`` elements at ``dev_ptr`` into column ``col``."""
        self._touch()
        self.dev.check(self._lib.bqg_push_chunk(self.handle, self.slot(col), ctypes.c_void_p(int(dev_ptr)),
                                                int(nrows), int(row_offset)))

    def read_device(self, col, dev_ptr, nrows=None, row_offset=0):
        """Device-to-device copy of column ``col`` into the device buffer at ``dev_ptr``."""
        n = self.nrows - row_offset if nrows is None else nrows
        self.dev.check(self._lib.bqg_table_read(self.handle, self.slot(col), ctypes.c_void_p(int(dev_ptr)),
                                                int(n), int(row_offset)))

    def column_ptr(self, col):
        p = ctypes.c_void_p()
        self.dev.check(self._lib.bqg_table_column_ptr(self.handle, self.slot(col), ctypes.byref(p)))
        return p.value or 0

    def load_carray(self, col, carray_dir, chunklen, nthreads=None, decode=None):
        """Decode a bcolz carray directory straight into device column ``col``; statistics
        follow at the next ``sync``.  ``decode``: 'device' (host threads read the chunk files,
        the GPU decodes the blosc frames), 'host' (host threads decode, pinned double-buffered
        DMA) or 'auto' (default; env BQGPU_INGEST_DECODE).  Returns the ingest report as a
        dict."""
        return self.load_carrays([(col, carray_dir, chunklen)], nthreads=nthreads, decode=decode)[0]

    def load_carrays(self, specs, nthreads=None, decode=None):
        """``load_carray`` for several columns in one call: [(col, carray_dir, chunklen)].  With
        the device decoder the columns' chunks are batched together (file reads of one column
        overlap the kernels of the previous one).  Returns one report per column."""
        self._touch()
        if not nthreads:
            nthreads = int(os.environ.get('BQGPU_INGEST_THREADS', '0')) or min(16, len(os.sched_getaffinity(0)))
        decode = decode or os.environ.get('BQGPU_INGEST_DECODE', 'auto')
        if decode not in L.DECODE_CODE:
            raise ValueError('decode must be one of %s' % sorted(L.DECODE_CODE))
        n = len(specs)
        cols = (ctypes.c_int32 * max(n, 1))(*[self.slot(c) for c, _, _ in specs])
        dirs = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(d) for _, d, _ in specs])
        lens = (ctypes.c_int64 * max(n, 1))(*[int(k) for _, _, k in specs])
        st = (L.IngestStats * max(n, 1))()
        self.dev.check(self._lib.bqg_table_load_carrays(self.handle, n, cols, dirs, lens, int(nthreads),
                                                        L.DECODE_CODE[decode], st))
        return [{f: getattr(st[i], f) for f, _ in L.IngestStats._fields_} for i in range(n)]

    def sync(self):
        self.dev.check(self._lib.bqg_table_sync(self.handle))

    def device_bytes(self):
        """HBM this table holds: its column allocations plus their compact resident copies."""
        b = ctypes.c_int64()
        self.dev.check(self._lib.bqg_table_device_bytes(self.handle, ctypes.byref(b)))
        return b.value

    def build_compact(self, cols=None):
        """Build the compact resident copies of ``cols`` (default: every column)
        now rather than on the first query that reads them; returns how many were built."""
        cols = list(self.names if cols is None else cols)
        arr = (ctypes.c_int32 * max(1, len(cols)))(*[self.slot(c) for c in cols])
        built = ctypes.c_int32()
        self.dev.check(self._lib.bqg_table_build_compact(self.handle, len(cols), arr, ctypes.byref(built)))
        return built.value

    def drop_compact(self):
        """Release the table's compact resident copies (rebuilt on demand)."""
        self.dev.check(self._lib.bqg_table_drop_compact(self.handle))

    def add_column(self, name, dtype):
        s = ctypes.c_int32()
        self.dev.check(self._lib.bqg_table_add_column(self.handle, L.DTYPE_CODE[device_dtype(dtype)],
                                                      ctypes.byref(s)))
        self._slot[name] = s.value
        self.dtypes[name] = np.dtype(dtype)
        self.__dict__.pop('_plans', None)  # a re-added name maps to a new slot / dtype
        return s.value

    def scratch_mask(self):
        """A device BOOL column for a mask, taken from the table's free list when one was
        released (``release_mask``), else added: a resident shard queried in a loop keeps a
        constant number of mask columns."""
        free = self.__dict__.setdefault('_free_masks', [])
        if free:
            return free.pop()
        name = '__mask_%d__' % len(self._scratch)
        self.add_column(name, np.bool_)
        self._scratch.append(name)
        return name

    def release_mask(self, name):
        """Return a ``scratch_mask`` column to the free list (its contents are dead)."""
        if name in self._scratch and getattr(self, 'handle', None):
            free = self.__dict__.setdefault('_free_masks', [])
            if name not in free:
                free.append(name)

    def read(self, col):
        s = self.slot(col)
        name, dt = self._logical(col)
        out = np.empty(self.nrows, dtype=device_dtype(dt))
        self.dev.check(self._lib.bqg_table_read(self.handle, s, out.ctypes.data, self.nrows, 0))
        return self._to_logical(name, out)

    def _to_logical(self, name, arr):
        """Device values of column ``name`` (codes, ticks) as the column's own dtype."""
        dt = self.dtypes.get(name)
        if dt is not None and is_string(dt):
            return self._strings[name].decode(arr)
        if dt is not None and is_time(dt):
            return np.ascontiguousarray(arr).view(dt)
        return arr

    def stats(self, col):
        imin, imax = ctypes.c_int64(), ctypes.c_int64()
        fmin, fmax = ctypes.c_double(), ctypes.c_double()
        nan = ctypes.c_int32()
        self.dev.check(self._lib.bqg_table_stats(self.handle, self.slot(col), ctypes.byref(imin),
                                                 ctypes.byref(imax), ctypes.byref(fmin),
                                                 ctypes.byref(fmax), ctypes.byref(nan)))
        dt = self.dtypes[col] if not isinstance(col, int) else None
        empty = nan.value < 0
        if dt is not None and dt.kind == 'f':
            return {'min': fmin.value, 'max': fmax.value, 'has_nan': nan.value > 0, 'empty': empty}
        if dt is not None and dt == np.uint64:
            return {'min': imin.value & 0xFFFFFFFFFFFFFFFF, 'max': imax.value & 0xFFFFFFFFFFFFFFFF,
                    'has_nan': False, 'empty': empty}
        return {'min': imin.value, 'max': imax.value, 'has_nan': False, 'empty': empty}

    # ---- query construction
    def _terms(self, term_list, keep):
        parsed = parse_terms(self.dtypes, term_list)
        arr = (L.Term * max(1, len(parsed)))()
        for i, (col, code, value) in enumerate(parsed):
            dt = self.dtypes[col]
            if is_string(dt):
                op, ivals, fvals = string_term(self._strings[col].values, code, value)
                dt = np.dtype(np.int32)
            elif is_time(dt):
                op, ivals, fvals = normalize(np.int64, code, time_value(dt, code, value))
                dt = np.dtype(np.int64)
            else:
                op, ivals, fvals = normalize(dt, code, value)
            if dt == np.uint64:
                iv = np.array([v & 0xFFFFFFFFFFFFFFFF for v in ivals] or [0], np.uint64).view(np.int64)
            else:
                iv = np.array(ivals or [0], np.int64)
            fv = np.array(fvals or [0.0], np.float64)
            keep += [iv, fv]
            arr[i] = L.Term(self.slot(col), op, max(len(ivals), len(fvals)), iv.ctypes.data,
                            fv.ctypes.data)
        return arr, len(parsed)

    def _query(self, groupby_cols, aggs, term_list, mask, keep):
        keys = np.array([self.slot(c) for c in groupby_cols] or [0], np.int32)
        keep.append(keys)
        terms, nt = self._terms(term_list or [], keep)
        keep.append(terms)
        agg_arr = (L.Agg * max(1, len(aggs)))(*[L.Agg(self.slot(c), L.AGG_CODE[op])
                                                for c, op in aggs])
        keep.append(agg_arr)
        q = L.Query(len(groupby_cols), keys.ctypes.data, nt, ctypes.addressof(terms),
                    -1 if mask is None else self.slot(mask), len(aggs), ctypes.addressof(agg_arr))
        return q

    # ---- calc path
    def where(self, term_list, out_mask=None):
        """Evaluate where-terms into a device BOOL column; returns (mask name, passing rows)."""
        keep = []
        terms, nt = self._terms(term_list, keep)
        if out_mask is None:
            out_mask = self.scratch_mask()
        npass = ctypes.c_int64()
        self.dev.check(self._lib.bqg_where(self.dev.handle, self.handle, nt,
                                           ctypes.addressof(terms), self.slot(out_mask),
                                           ctypes.byref(npass)))
        return out_mask, npass.value

    def expand_subgroups(self, basket_col, mask, out_mask=None):
        if out_mask is None:
            out_mask = self.scratch_mask()
        self.dev.check(self._lib.bqg_expand_subgroups(self.dev.handle, self.handle,
                                                      self.slot(basket_col), self.slot(mask),
                                                      self.slot(out_mask)))
        return out_mask

    def _plan(self, groupby_cols, agg_list, where_terms, mask):
        """(output names, parsed aggregations, C query struct) of a groupby, built once per
        distinct query text and table (the struct points into arrays the plan keeps alive):
        repeated queries on a resident shard skip the Python-side parsing."""
        # the key is the query's values with their types (np.float32(0.1) and 0.1 normalise to
        # different bounds); anything but plain lists / tuples / sets of scalars and strings
        # (arrays, generators, other iterables) is not cached
        try:
            key = (_freeze(groupby_cols), _freeze(agg_list), _freeze(where_terms or []), mask)
            cacheable = True
        except _Unfreezable:
            key, cacheable = None, False
        plans = self.__dict__.setdefault('_plans', OrderedDict())
        hit = plans.get(key) if cacheable else None
        if hit is not None:
            return hit[:3] + hit[4:]
        groupby_cols = list(groupby_cols)
        for c in groupby_cols:
            self.slot(c)
        ops = self._parse_aggs(agg_list)
        names = groupby_cols + [o[1] for o in ops]
        if len(set(names)) != len(names):
            raise ValueError('duplicate output column names: %s' % names)
        keep = []
        q = self._query(groupby_cols, [(o[0], o[2]) for o in ops], where_terms, mask, keep)
        # key columns whose device values (codes, ticks) map back to another dtype
        logical = [c for c in groupby_cols
                   if self.dtypes.get(c) is not None and (is_string(self.dtypes[c]) or is_time(self.dtypes[c]))]
        if cacheable:
            if len(plans) >= 64:
                plans.popitem(last=False)
            plans[key] = (names, ops, q, keep, logical)
        else:
            self.__dict__['_last_plan_keep'] = keep  # the struct's arrays live until the next query
        return names, ops, q, logical

    def _parse_aggs(self, agg_list):
        ops = parse_agg_list(self.dtypes, agg_list)
        for in_col, out_col, op, dt in ops:
            if op in ('sum', 'mean', 'std') and (is_string(self.dtypes[in_col]) or is_time(self.dtypes[in_col])):
                raise NotImplementedError('%s of a %s column' % (op, self.dtypes[in_col]))
        return ops

    def groupby(self, groupby_cols, agg_list, where_terms=None, mask=None):
        """bquery ``ctable.groupby`` semantics; returns (OrderedDict of columns, filtered)."""
        names, ops, q, logical = self._plan(groupby_cols, agg_list, where_terms, mask)
        res = ctypes.c_void_p()
        self.dev.check(self._lib.bqg_groupby(self.dev.handle, self.handle, ctypes.byref(q),
                                             ctypes.byref(res)))
        out, filtered = _result_to_columns(self.dev, res, names)
        for k in logical:
            out[k] = self._to_logical(k, out[k])
        for (in_col, out_col, op, dt) in ops:
            if out[out_col].dtype != dt:
                out[out_col] = out[out_col].astype(dt)
        return out, filtered

    def groupby_table(self, groupby_cols, agg_list, where_terms=None, mask=None):
        """``groupby`` whose result stays in HBM: a new ShardTable (keys, then aggregations)."""
        groupby_cols = list(groupby_cols)
        for c in groupby_cols:
            self.slot(c)
        ops = self._parse_aggs(agg_list)
        names = groupby_cols + [o[1] for o in ops]
        if len(set(names)) != len(names):
            raise ValueError('duplicate output column names: %s' % names)
        keep = []
        q = self._query(groupby_cols, [(o[0], o[2]) for o in ops], where_terms, mask, keep)
        h = ctypes.c_void_p()
        self.dev.check(self._lib.bqg_groupby_table(self.dev.handle, self.handle, ctypes.byref(q), ctypes.byref(h)))
        dts = [self.dtypes[c] for c in groupby_cols] + [o[3] for o in ops]
        return ShardTable._wrap(h, names, dts, self.dev, {c: self._strings[c] for c in groupby_cols if c in self._strings})

    def select_rows_table(self, cols, where_terms=None, mask=None):
        """``select_rows`` whose result stays in HBM: a new ShardTable."""
        cols = list(cols)
        keep = []
        q = self._query([], [], where_terms, mask, keep)
        sel = np.array([self.slot(c) for c in cols] or [0], np.int32)
        h = ctypes.c_void_p()
        self.dev.check(self._lib.bqg_select_rows_table(self.dev.handle, self.handle, ctypes.byref(q), len(cols),
                                                       sel.ctypes.data, ctypes.byref(h)))
        return ShardTable._wrap(h, cols, [self.dtypes[c] for c in cols], self.dev,
                                {c: self._strings[c] for c in cols if c in self._strings})

    def to_host(self, cols=None):
        """The table's columns as numpy arrays."""
        return OrderedDict((c, self.read(c)) for c in (cols or self.names))

    def factorize(self, col, labels=True):
        """bquery's factor cache of column ``col`` (``bqg_factorize``): (int64 first-appearance
        label of every row, or None; distinct values in label order).  Any key dtype: integer
        columns spanning at most 2^27 values through a lookup table, floats (khash identity),
        bools and wider spans through a hash of the canonical key bits."""
        s = self.slot(col)
        logical = np.dtype(self.dtypes[col])
        dt = device_dtype(logical)
        cap = min(self.nrows, 1 << 22)
        if dt.kind in 'iu':
            st = self.stats(col)
            cap = min(self.nrows, 1 if st['empty'] else int(st['max']) - int(st['min']) + 1)
        elif dt.kind == 'b':
            cap = min(self.nrows, 2)
        lab = np.empty(self.nrows, np.int64) if labels else None
        n_values = ctypes.c_int64()
        for _ in range(2):
            values = np.empty(max(cap, 1), dtype=dt)
            rc = self._lib.bqg_factorize(self.dev.handle, self.handle, s, lab.ctypes.data if labels else None,
                                         values.ctypes.data, len(values), ctypes.byref(n_values))
            if rc == 0 or n_values.value <= len(values):
                break
            cap = n_values.value  # more distinct values than the first guess: once more, sized
        self.dev.check(rc)
        return lab, self._to_logical(col, values[:n_values.value])

    def select_rows(self, cols, where_terms=None, mask=None):
        """aggregate=False: the passing rows of ``cols`` in row order."""
        cols = list(cols)
        keep = []
        q = self._query([], [], where_terms, mask, keep)
        sel = np.array([self.slot(c) for c in cols] or [0], np.int32)
        res = ctypes.c_void_p()
        self.dev.check(self._lib.bqg_select_rows(self.dev.handle, self.handle, ctypes.byref(q),
                                                 len(cols), sel.ctypes.data, ctypes.byref(res)))
        out, _ = _result_to_columns(self.dev, res, cols)
        for c in cols:
            out[c] = self._to_logical(c, out[c])
        return out
