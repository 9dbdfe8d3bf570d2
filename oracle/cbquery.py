"""ctypes front-end of the C restatement (oracle/cbquery.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
It normalises where-terms with the same exact int/float rules as bquery_oracle._exact_cmp
and calls the single-threaded C port of bquery's multi-pass groupby.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from collections import OrderedDict
from fractions import Fraction

import numpy as np

from . import bquery_oracle as bo

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, '_build', 'libcbquery.so')

DT_CODES = {
    np.dtype(np.bool_): 0, np.dtype(np.int8): 1, np.dtype(np.int16): 2, np.dtype(np.int32): 3,
    np.dtype(np.int64): 4, np.dtype(np.uint8): 5, np.dtype(np.uint16): 6,
    np.dtype(np.uint32): 7, np.dtype(np.uint64): 8, np.dtype(np.float32): 9,
    np.dtype(np.float64): 10,
}
AGG_CODES = {'sum': 0, 'count': 1, 'count_distinct': 2, 'sorted_count_distinct': 3,
             'mean': 4, 'std': 5}
T_FALSE, T_TRUE = -1, 0


class _Term(ctypes.Structure):
    _fields_ = [('col', ctypes.c_int32), ('op', ctypes.c_int32), ('nvals', ctypes.c_int32),
                ('is_float', ctypes.c_int32), ('ivals', ctypes.c_void_p),
                ('fvals', ctypes.c_void_p)]


class _Result(ctypes.Structure):
    _fields_ = [('n_groups', ctypes.c_int64), ('group_rows', ctypes.POINTER(ctypes.c_int64)),
                ('agg_out', ctypes.POINTER(ctypes.c_void_p))]


_lib = None


def build():
    subprocess.check_call(['make', '-s', '-C', _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.cbq_where.restype = ctypes.c_int64
        _lib.cbq_groupby.restype = ctypes.c_int
    return _lib


def normalize_term(dtype, code, value):
    """(op, int64 values, float values) with constant folding; exact Python semantics."""
    kind = np.dtype(dtype).kind
    if kind in 'biu':
        if kind == 'b':
            lo, hi = 0, 1
        else:
            info = np.iinfo(dtype)
            lo, hi = int(info.min), int(info.max)
        if code in (bo.OP_IN, bo.OP_NIN):
            members = []
            for m in value:
                m = int(m) if isinstance(m, bool) else m
                if isinstance(m, float):
                    if math.isnan(m) or math.isinf(m) or Fraction(m).denominator != 1:
                        continue
                    m = int(m)
                if lo <= m <= hi:
                    members.append(m)
            members = sorted(set(members))
            if not members:
                return (T_FALSE if code == bo.OP_IN else T_TRUE), [], []
            return code, members, []
        v = int(value) if isinstance(value, bool) else value
        if isinstance(v, float):
            if math.isnan(v):
                return (T_TRUE if code == bo.OP_NE else T_FALSE), [], []
            if math.isinf(v):
                big = v > 0
                res = {bo.OP_EQ: False, bo.OP_NE: True, bo.OP_GT: not big, bo.OP_GE: not big,
                       bo.OP_LT: big, bo.OP_LE: big}[code]
                return (T_TRUE if res else T_FALSE), [], []
            fr = Fraction(v)
            if code in (bo.OP_EQ, bo.OP_NE):
                if fr.denominator != 1:
                    return (T_TRUE if code == bo.OP_NE else T_FALSE), [], []
                v = int(fr)
            elif code in (bo.OP_GT, bo.OP_LE):
                v = math.floor(fr)
            else:
                v = math.ceil(fr)
        if v > hi or v < lo:
            above = v > hi
            res = {bo.OP_EQ: False, bo.OP_NE: True, bo.OP_GT: not above, bo.OP_GE: not above,
                   bo.OP_LT: above, bo.OP_LE: above}[code]
            return (T_TRUE if res else T_FALSE), [], []
        return code, [int(v)], []
    if kind == 'f':
        if code in (bo.OP_IN, bo.OP_NIN):
            return code, [], sorted(float(m) for m in value)
        return code, [], [float(value)]
    raise NotImplementedError('where_terms on dtype %s' % dtype)


def _mk_terms(columns, names, term_list):
    terms = bo.parse_terms(columns, term_list)
    keep = []
    structs = (_Term * max(1, len(terms)))()
    for i, (col, code, value) in enumerate(terms):
        dt = columns[col].dtype
        op, ivals, fvals = normalize_term(dt, code, value)
        if dt == np.uint64:
            iv = np.array([v & 0xFFFFFFFFFFFFFFFF for v in ivals] or [0], dtype=np.uint64).view(np.int64)
        else:
            iv = np.array(ivals or [0], dtype=np.int64)
        fv = np.array(fvals or [0.0], dtype=np.float64)
        keep += [iv, fv]
        structs[i] = _Term(names.index(col), op, max(len(ivals), len(fvals)),
                           1 if dt.kind == 'f' else 0, iv.ctypes.data, fv.ctypes.data)
    return structs, len(terms), keep


def _prep(columns):
    names = list(columns.keys())
    arrs = [np.ascontiguousarray(columns[n]) for n in names]
    ptrs = (ctypes.c_void_p * max(1, len(arrs)))(*[a.ctypes.data for a in arrs])
    dts = (ctypes.c_int * max(1, len(arrs)))(*[DT_CODES[a.dtype] for a in arrs])
    n = len(arrs[0]) if arrs else 0
    return names, arrs, ptrs, dts, n


def where_terms(columns, term_list):
    names, arrs, ptrs, dts, n = _prep(columns)
    structs, nt, keep = _mk_terms(columns, names, term_list)
    mask = np.empty(n, np.uint8)
    lib().cbq_where(ctypes.c_int64(n), ptrs, dts, nt, structs,
                    mask.ctypes.data_as(ctypes.c_void_p))
    return mask.view(bool)


def groupby(columns, groupby_cols, agg_list, bool_arr=None):
    """Same contract as bquery_oracle.groupby, computed by the C port."""
    names, arrs, ptrs, dts, n = _prep(columns)
    ops = bo.parse_agg_list(columns, agg_list)
    keys = (ctypes.c_int * max(1, len(groupby_cols)))(*[names.index(c) for c in groupby_cols])
    acols = (ctypes.c_int * max(1, len(ops)))(*[names.index(o[0]) for o in ops])
    aops = (ctypes.c_int * max(1, len(ops)))(*[AGG_CODES[o[2]] for o in ops])
    mask = None
    if bool_arr is not None:
        mask = np.ascontiguousarray(np.asarray(bool_arr, dtype=bool)).view(np.uint8)
    res = _Result()
    rc = lib().cbq_groupby(ctypes.c_int64(n), ptrs, dts, len(groupby_cols), keys,
                           None if mask is None else mask.ctypes.data_as(ctypes.c_void_p),
                           len(ops), acols, aops, ctypes.byref(res))
    if rc != 0:
        raise RuntimeError('cbq_groupby failed')
    try:
        g = res.n_groups
        rows = np.ctypeslib.as_array(res.group_rows, shape=(max(g, 1),))[:g].copy()
        out = OrderedDict()
        for c in groupby_cols:
            out[c] = columns[c][rows] if g else columns[c][:0]
        for a, (in_col, out_col, op, dt) in enumerate(ops):
            buf = ctypes.cast(res.agg_out[a], ctypes.POINTER(ctypes.c_char))
            raw = ctypes.string_at(buf, g * dt.itemsize) if g else b''
            out[out_col] = np.frombuffer(raw, dtype=dt).copy()
        return out
    finally:
        lib().cbq_free_result(ctypes.byref(res), len(ops))


def handle_work(columns, groupby_cols, agg_list, where_terms_list):
    bool_arr = where_terms(columns, where_terms_list) if where_terms_list else None
    return groupby(columns, groupby_cols, agg_list, bool_arr=bool_arr)
