"""CPU restatement of bqueryd's per-shard groupby path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker; the product
package ``bqueryd_amd`` never imports anything under ``oracle/``.

What it restates (reference = visualfabriq/bqueryd v0.3.10, read-only at /root/reference):

* the worker calc path ``WorkerNode.handle_work`` (``bqueryd/worker.py:269-348``):
  where-terms filter -> optional basket expansion -> ``groupby`` or raw filtered rows;
* the controller gather (``bqueryd/controller.py:146-221``): shard results keyed by filename,
  empty ``''`` results skipped;
* the client merge ``RPC.uncompress_groupby_to_df`` (``bqueryd/rpc.py:134-179``): per-shard
  tables appended, ``aggregate=True`` re-groups with ``sum`` of the finalized values.

The arithmetic itself lives in the external ``bquery`` package (pinned only as
``bquery>=0.2.10``, ``setup.py:70``), which is NOT in /root/reference nor installed here.
Its algorithm is restated from the public bquery 0.2.x design as summarised in SURVEY.md
§3.2 / §8a rows A6-A10; every such rule is tagged ``[ext-bquery, unverified]``.

Parity status (also in DESIGN.md §4; the pins are ``tests/test_oracle.py``):
* PINNED against the reference's own test oracle, pandas (``tests/test_simple_rpc.py:139-190``):
  the reference's cases (single-key ``sum`` / ``mean`` / ``count`` without a filter, and
  full-vs-sharded counts), and every rule pandas can express: multi-key first-appearance
  group order (``groupby(sort=False)``), where-term filters and the skip slot (``df[mask]``),
  count_distinct (``nunique``), std (``std(ddof=0)``), raw rows (``aggregate=False``),
  basket expansion (``transform('any')`` over runs), the ``aggregate=True`` client merge
  (concat + ``groupby(sort=False).sum()``), and sorted_count_distinct up to its zero-init rule.
* PARITY UNPINNED (bquery-only rules; bquery / bcolz are absent and no reference-held golden
  vectors exist): sorted_count_distinct's zero-initialised ``last`` rule, the
  bit pattern of Knuth's incremental mean, float32 row-order sums, and the factorization
  check's exact operator semantics.

All row-order-dependent reductions (float sums, Knuth mean, Welford std,
sorted_count_distinct) are evaluated strictly in row order, as bquery's Cython loops do.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from fractions import Fraction

import numpy as np

# op codes of bquery's where_terms [ext-bquery, unverified]
OP_EQ, OP_NE, OP_IN, OP_NIN, OP_GT, OP_GE, OP_LT, OP_LE = range(1, 9)
_OP_NAMES = {
    '==': OP_EQ, 'eq': OP_EQ,
    '!=': OP_NE, 'neq': OP_NE,
    'in': OP_IN,
    'nin': OP_NIN, 'not in': OP_NIN,
    '>': OP_GT, '>=': OP_GE, '<': OP_LT, '<=': OP_LE,
}

AGG_OPS = ('sum', 'count', 'count_distinct', 'sorted_count_distinct', 'mean', 'std')


# ----------------------------------------------------------------------------------------
# where_terms (worker.py:303 -> bquery ctable.where_terms)   [ext-bquery, unverified]
# ----------------------------------------------------------------------------------------
def parse_terms(columns, term_list):
    """Validate and normalise a where-terms list exactly like bquery's ``where_terms``.

    Returns a list of (col, op_code, value) with single-element in/nin collapsed to ==/!=.
    Raises KeyError for an unknown column or operator, ValueError for malformed in-lists.
    """
    if type(term_list) not in (list, set, tuple):
        raise ValueError("Only term lists are supported")
    out = []
    for term in term_list:
        col, op, value = term[0], term[1], term[2]
        op = op.lower().strip(' ')
        if col not in columns:
            raise KeyError(str(col) + ' not in table')
        if op not in _OP_NAMES:
            raise KeyError(str(op) + ' is not an accepted operator for filtering')
        code = _OP_NAMES[op]
        if code in (OP_IN, OP_NIN):
            if type(value) not in (list, set, tuple):
                raise ValueError("In selections need lists, sets or tuples")
            if len(value) < 1:
                raise ValueError("A value list needs to have values")
            if len(value) == 1:
                code = OP_EQ if code == OP_IN else OP_NE
                value = list(value)[0]
            else:
                value = set(value)
        out.append((col, code, value))
    return out


def _exact_cmp(arr, code, value):
    """Row-wise ``arr[i] <op> value`` with Python's exact mixed int/float semantics.

    bquery's apply_where_terms compares numpy scalars from the row tuple against the Python
    filter value one row at a time; Python compares ints and floats exactly, numpy-scalar
    float32 is promoted to float64.  This helper reproduces that without a per-row loop.
    """
    if isinstance(value, bool):
        value = int(value)
    kind = arr.dtype.kind
    if kind in 'SU':
        # string columns: bytes / str compared as numpy stores them (trailing NULs are padding;
        # a py2 str value -- latin-1 after the worker's unpickling -- matches 'S' bytes)
        if kind == 'S' and isinstance(value, str):
            value = value.encode('latin-1')
        if kind == 'U' and isinstance(value, bytes):
            value = value.decode('latin-1')
        if not isinstance(value, (bytes, str)):
            return np.full(arr.shape, code == OP_NE)
        v = value
    elif kind in 'Mm':
        # datetime64 / timedelta64: compared as the column's ticks (ints pass as ticks)
        if isinstance(value, (int, np.integer)):
            v = np.asarray(value, np.int64).view(arr.dtype)
        else:
            v = np.asarray(value).astype(arr.dtype)
    elif kind == 'b':
        arr = arr.astype(np.int64)
        kind = 'i'
    if kind in 'iu':
        if isinstance(value, float):
            if math.isnan(value):
                return np.full(arr.shape, code == OP_NE)
            if math.isinf(value):
                big = value > 0
                res = {OP_EQ: False, OP_NE: True, OP_GT: not big, OP_GE: not big,
                       OP_LT: big, OP_LE: big}[code]
                return np.full(arr.shape, res)
            fr = Fraction(value)
            if code in (OP_EQ, OP_NE):
                if fr.denominator != 1:
                    return np.full(arr.shape, code == OP_NE)
                value = int(fr)
            elif code == OP_GT:
                value = math.floor(fr)
            elif code == OP_GE:
                value = math.ceil(fr)
            elif code == OP_LT:
                value = math.ceil(fr)
            elif code == OP_LE:
                value = math.floor(fr)
        value = int(value)
        info = np.iinfo(arr.dtype)
        if value > info.max or value < info.min:
            above = value > info.max
            res = {OP_EQ: False, OP_NE: True, OP_GT: not above, OP_GE: not above,
                   OP_LT: above, OP_LE: above}[code]
            return np.full(arr.shape, res)
        v = arr.dtype.type(value)
    elif kind == 'f':
        arr = arr.astype(np.float64)
        v = float(value)
    elif kind not in 'SUMm':
        raise NotImplementedError('where_terms on dtype %s' % arr.dtype)
    if code == OP_EQ:
        return arr == v
    if code == OP_NE:
        return arr != v
    if code == OP_GT:
        return arr > v
    if code == OP_GE:
        return arr >= v
    if code == OP_LT:
        return arr < v
    if code == OP_LE:
        return arr <= v
    raise ValueError(code)


def where_terms(columns, term_list):
    """bool mask = AND over terms (bquery ``ctable.where_terms``, called at worker.py:303)."""
    terms = parse_terms(columns, term_list)
    n = len(next(iter(columns.values()))) if columns else 0
    mask = np.ones(n, dtype=bool)
    for col, code, value in terms:
        arr = columns[col]
        if code in (OP_IN, OP_NIN):
            hit = np.zeros(n, dtype=bool)
            for member in value:
                hit |= _exact_cmp(arr, OP_EQ, member)
            mask &= hit if code == OP_IN else ~hit
        else:
            mask &= _exact_cmp(arr, code, value)
    return mask


def factorization_check(values_cache, columns, term_list):
    """``ctable.where_terms_factorization_check`` (worker.py:298) [ext-bquery, unverified].

    ``values_cache`` maps column -> iterable of the distinct values stored in its
    ``<col>.values`` factor cache.  A term whose column has no cache is not checked.
    Returns False iff some cached term can be proven unsatisfiable.
    """
    terms = parse_terms(columns, term_list)
    for col, code, value in terms:
        if col not in values_cache:
            break
        vals = np.asarray(list(values_cache[col]), dtype=columns[col].dtype)
        if code in (OP_IN, OP_NIN):
            hit = np.zeros(len(vals), dtype=bool)
            for member in value:
                hit |= _exact_cmp(vals, OP_EQ, member)
            ok = bool(np.any(hit if code == OP_IN else ~hit))
        else:
            ok = bool(np.any(_exact_cmp(vals, code, value)))
        if not ok:
            return False
    return True


# ----------------------------------------------------------------------------------------
# factorisation (bquery make_group_index)   [ext-bquery, unverified]
# ----------------------------------------------------------------------------------------
def factorize(arr):
    """Dense int64 labels in first-appearance order, plus the uniques in label order.

    Float keys follow pandas/khash equality: NaN == NaN, -0.0 == +0.0.
    """
    arr = np.asarray(arr)
    if len(arr) == 0:
        return np.zeros(0, np.int64), arr[:0]
    key = arr
    if arr.dtype.kind == 'f':
        key = arr.astype(np.float64) + 0.0  # -0.0 -> +0.0
        key = np.where(np.isnan(key), np.nan, key)
    uniq, first_idx, inv = np.unique(key, return_index=True, return_inverse=True)
    order = np.argsort(first_idx, kind='stable')
    rank = np.empty(len(order), np.int64)
    rank[order] = np.arange(len(order), dtype=np.int64)
    labels = rank[inv.reshape(-1)]
    return labels, arr[first_idx[order]]


def make_group_index(columns, groupby_cols, bool_arr):
    """Returns (factor, nr_groups, skip_key) as bquery's ``make_group_index``."""
    n = len(next(iter(columns.values())))
    if len(groupby_cols) == 0:
        factor = np.zeros(n, np.int64)
        nr_groups = 1
    elif len(groupby_cols) == 1:
        factor, uniq = factorize(columns[groupby_cols[0]])
        nr_groups = len(uniq)
    else:
        labels = [factorize(columns[c])[0] for c in groupby_cols]
        combo = np.stack(labels, axis=1) if n else np.zeros((0, len(labels)), np.int64)
        if n:
            _, first_idx, inv = np.unique(combo, axis=0, return_index=True, return_inverse=True)
            order = np.argsort(first_idx, kind='stable')
            rank = np.empty(len(order), np.int64)
            rank[order] = np.arange(len(order), dtype=np.int64)
            factor = rank[inv.reshape(-1)]
            nr_groups = len(order)
        else:
            factor = np.zeros(0, np.int64)
            nr_groups = 0
    skip_key = None
    if bool_arr is not None:
        # bcolz.eval('(factor + 1) * bool - 1') then re-factorize
        f2 = (factor + 1) * bool_arr.astype(np.int64) - 1
        factor, uniq = factorize(f2)
        hits = np.nonzero(uniq == -1)[0]
        if len(hits):
            skip_key = int(hits[0])
        nr_groups = len(uniq)
    if skip_key is None:
        skip_key = nr_groups
    return factor, nr_groups, skip_key


# ----------------------------------------------------------------------------------------
# aggregation (create_agg_ctable / aggregate_groups)   [ext-bquery, unverified]
# ----------------------------------------------------------------------------------------
def parse_agg_list(columns, agg_list):
    """create_agg_ctable: returns [(in_col, out_col, op, out_dtype)]."""
    ops = []
    for info in agg_list:
        if not isinstance(info, list):
            in_col, op, out_col = info, 'sum', info
        else:
            in_col, op = info[0], info[1]
            out_col = in_col if len(info) == 2 else info[2]
        if op not in AGG_OPS:
            raise NotImplementedError('Unknown Aggregation Type: ' + str(op))
        if in_col not in columns:
            raise KeyError(str(in_col))
        if op in ('count', 'count_distinct', 'sorted_count_distinct'):
            dt = np.dtype(np.int64)
        elif op in ('mean', 'std'):
            dt = np.dtype(np.float64)
        else:
            dt = columns[in_col].dtype
        ops.append((in_col, out_col, op, dt))
    return ops


def _canon(v):
    """khash float equality: NaN == NaN, -0.0 == 0.0."""
    if isinstance(v, float):
        if v != v:
            return ('nan',)
        return v + 0.0
    return v


def aggregate_one(values, factor, nr_groups, skip_key, op, out_dtype):
    """One aggregation pass over the rows, in row order, skipping ``skip_key``."""
    keep = factor != skip_key
    f = factor[keep]
    v = values[keep]
    if op == 'sum':
        if out_dtype.kind in 'iu':
            acc = np.zeros(nr_groups, np.int64 if out_dtype.kind == 'i' else np.uint64)
            np.add.at(acc, f, v.astype(acc.dtype))
            return acc.astype(out_dtype)  # C wrap-around to the input width
        if out_dtype.kind == 'f':
            out = np.zeros(nr_groups, out_dtype)
            np.add.at(out, f, v.astype(out_dtype))  # unbuffered, in row order
            return out
        raise NotImplementedError('sum of dtype %s' % out_dtype)
    if op == 'count':
        return np.bincount(f, minlength=nr_groups).astype(np.int64)
    if op == 'mean':  # Knuth incremental mean, float64, row order
        if v.dtype.kind not in 'iuf':
            raise NotImplementedError('mean of dtype %s' % v.dtype)
        mean = np.zeros(nr_groups, np.float64)
        cnt = np.zeros(nr_groups, np.int64)
        vf = v.astype(np.float64)
        for g, x in zip(f.tolist(), vf.tolist()):
            cnt[g] += 1
            mean[g] += (x - mean[g]) / cnt[g]
        return mean
    if op == 'std':  # Welford, population (ddof=0)  [ext-bquery, unverified]
        if v.dtype.kind not in 'iuf':
            raise NotImplementedError('std of dtype %s' % v.dtype)
        mean = [0.0] * nr_groups
        m2 = [0.0] * nr_groups
        cnt = [0] * nr_groups
        for g, x in zip(f.tolist(), v.astype(np.float64).tolist()):
            cnt[g] += 1
            d = x - mean[g]
            mean[g] += d / cnt[g]
            m2[g] += d * (x - mean[g])
        return np.array([math.sqrt(m2[g] / cnt[g]) if cnt[g] else float('nan')
                         for g in range(nr_groups)], np.float64)
    if op == 'count_distinct':
        sets = [set() for _ in range(nr_groups)]
        for g, x in zip(f.tolist(), v.tolist()):
            sets[g].add(_canon(x))
        return np.array([len(s) for s in sets], np.int64)
    if op == 'sorted_count_distinct':
        # last[] zero-initialised; the first processed row sets last[0]=v, out[0]=1;
        # every later row adds (v != last[g]); every row then sets last[g]=v.
        last = np.zeros(nr_groups, values.dtype).tolist()
        out = [0] * nr_groups
        first = True
        for g, x in zip(f.tolist(), v.tolist()):
            if first:
                last[0] = x
                out[0] = 1
                first = False
            elif x != last[g]:
                out[g] += 1
            last[g] = x
        return np.array(out, np.int64)
    raise NotImplementedError(op)


def groupby_value(keycol, factor, nr_groups, skip_key):
    """Key value of each group slot (last row written wins; skip slot left at zero)."""
    out = np.zeros(nr_groups, keycol.dtype)
    keep = factor != skip_key
    out[factor[keep]] = keycol[keep]
    return out


def groupby(columns, groupby_cols, agg_list, bool_arr=None):
    """bquery ``ctable.groupby`` (worker.py:313-314) -> OrderedDict[name -> ndarray]."""
    groupby_cols = list(groupby_cols)
    for c in groupby_cols:
        if c not in columns:
            raise KeyError(str(c))
    ops = parse_agg_list(columns, agg_list)
    if bool_arr is not None:
        bool_arr = np.asarray(bool_arr, dtype=bool)
    factor, nr_groups, skip_key = make_group_index(columns, groupby_cols, bool_arr)
    if bool_arr is not None and np.all(bool_arr):
        bool_arr = None
    out = OrderedDict()
    for c in groupby_cols:
        arr = groupby_value(columns[c], factor, nr_groups, skip_key)
        if bool_arr is not None:
            arr = np.delete(arr, skip_key)
        out[c] = arr
    for in_col, out_col, op, dt in ops:
        arr = aggregate_one(columns[in_col], factor, nr_groups, skip_key, op, dt)
        if bool_arr is not None:
            arr = np.delete(arr, skip_key)
        out[out_col] = arr
    return out


def is_in_ordered_subgroups(basket, bool_arr):
    """Expand the mask to whole runs of equal consecutive ``basket`` values that contain a
    passing row (worker.py:306-307) [ext-bquery, unverified]."""
    if bool_arr is None:
        return None
    basket = np.asarray(basket)
    n = len(basket)
    if n == 0:
        return np.zeros(0, bool)
    starts = np.ones(n, bool)
    starts[1:] = basket[1:] != basket[:-1]
    run_id = np.cumsum(starts) - 1
    run_any = np.zeros(run_id[-1] + 1, bool)
    np.logical_or.at(run_any, run_id, np.asarray(bool_arr, bool))
    return run_any[run_id]


# ----------------------------------------------------------------------------------------
# worker calc path and client merge
# ----------------------------------------------------------------------------------------
def handle_work(columns, groupby_cols, agg_list, where_terms_list, aggregate=True,
                expand_filter_column=None, values_cache=None):
    """The per-shard calc of ``WorkerNode.handle_work`` (worker.py:291-323).

    Returns ``''`` for the factorization-check early-out (worker.py:298-301), else an
    OrderedDict of result columns.
    """
    if not where_terms_list:
        bool_arr = None
    else:
        if values_cache is not None and not factorization_check(values_cache, columns,
                                                                 where_terms_list):
            return ''
        bool_arr = where_terms(columns, where_terms_list)
    if expand_filter_column:
        bool_arr = is_in_ordered_subgroups(columns[expand_filter_column], bool_arr)
    if aggregate:
        return groupby(columns, groupby_cols, agg_list, bool_arr=bool_arr)
    cols = list(groupby_cols) + [x[0] for x in agg_list]
    out = OrderedDict()
    for c in cols:
        out[c] = columns[c] if bool_arr is None else columns[c][bool_arr]
    return out


def client_merge(shard_results, groupby_cols, agg_list, aggregate=False):
    """``RPC.uncompress_groupby_to_df`` (rpc.py:134-179) on already-decoded shard tables.

    ``shard_results`` are in the order the client globs them; ``''`` entries (empty shard
    replies) are dropped like the controller does (controller.py:175-179,196).
    Returns an OrderedDict of columns, or None for "no shard results" (empty DataFrame).
    """
    tables = [t for t in shard_results if not (isinstance(t, str) and t == '')]
    if not tables:
        return None
    names = list(tables[0].keys())
    cat = OrderedDict((n, np.concatenate([t[n] for t in tables])) for n in names)
    if not aggregate:
        return cat
    new_agg_list = [[x[2], 'sum', x[2]] for x in agg_list]
    return groupby(cat, groupby_cols, new_agg_list)
