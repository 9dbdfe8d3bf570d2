"""Host-side normalisation of bqueryd's where-terms and aggregation specs.

Mirrors the argument handling of bquery's ``ctable.where_terms`` (called at
``bqueryd/worker.py:303``) and ``create_agg_ctable`` (inside ``ct.groupby``, worker.py:313)
[ext-bquery, unverified -- bquery is not vendored; see SURVEY.md §8c], and reduces every term
to the typed, constant-folded form the gfx950 kernels evaluate (include/bqgpu.h ``bqg_term``):

* integer/bool columns compare against int64 values with Python's exact int/float rules
  (``int_col >= 2.5`` -> ``>= 3``; ``int_col == 2.5`` -> always false; out-of-range
  thresholds fold to constants);
* float columns compare after promotion to float64 (numpy-1.x scalar semantics).
"""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

from . import _lib as L

OPS = {
    '==': L.T_EQ, 'eq': L.T_EQ, '!=': L.T_NE, 'neq': L.T_NE, 'in': L.T_IN, 'nin': L.T_NIN,
    'not in': L.T_NIN, '>': L.T_GT, '>=': L.T_GE, '<': L.T_LT, '<=': L.T_LE,
}
AGG_OPS = ('sum', 'count', 'count_distinct', 'sorted_count_distinct', 'mean', 'std')


def parse_terms(names, term_list):
    """Validate a where-terms list like bquery (KeyError / ValueError on bad input)."""
    if type(term_list) not in (list, set, tuple):
        raise ValueError("Only term lists are supported")
    out = []
    for term in term_list:
        col, op, value = term[0], term[1], term[2]
        op = op.lower().strip(' ')
        if col not in names:
            raise KeyError(str(col) + ' not in table')
        if op not in OPS:
            raise KeyError(str(op) + ' is not an accepted operator for filtering')
        code = OPS[op]
        if code in (L.T_IN, L.T_NIN):
            if type(value) not in (list, set, tuple):
                raise ValueError("In selections need lists, sets or tuples")
            if len(value) < 1:
                raise ValueError("A value list needs to have values")
            if len(value) == 1:
                code = L.T_EQ if code == L.T_IN else L.T_NE
                value = list(value)[0]
            else:
                value = set(value)
        out.append((col, code, value))
    return out


def _fold(res):
    return L.T_TRUE if res else L.T_FALSE


def normalize(dtype, code, value):
    """-> (op, int64 list, float list) for one parsed term on a column of ``dtype``."""
    dtype = np.dtype(dtype)
    kind = dtype.kind
    if kind in 'biu':
        if kind == 'b':
            lo, hi = 0, 1
        else:
            info = np.iinfo(dtype)
            lo, hi = int(info.min), int(info.max)
        if code in (L.T_IN, L.T_NIN):
            members = set()
            for m in value:
                if isinstance(m, (bool, np.bool_)):
                    m = int(m)
                if isinstance(m, (float, np.floating)):
                    m = float(m)
                    if math.isnan(m) or math.isinf(m) or Fraction(m).denominator != 1:
                        continue
                    m = int(m)
                m = int(m)
                if lo <= m <= hi:
                    members.add(m)
            if not members:
                return _fold(code == L.T_NIN), [], []
            return code, sorted(members), []
        v = value
        if isinstance(v, (bool, np.bool_)):
            v = int(v)
        if isinstance(v, (float, np.floating)):
            v = float(v)
            if math.isnan(v):
                return _fold(code == L.T_NE), [], []
            if math.isinf(v):
                big = v > 0
                return _fold({L.T_EQ: False, L.T_NE: True, L.T_GT: not big, L.T_GE: not big,
                              L.T_LT: big, L.T_LE: big}[code]), [], []
            fr = Fraction(v)
            if code in (L.T_EQ, L.T_NE):
                if fr.denominator != 1:
                    return _fold(code == L.T_NE), [], []
                v = int(fr)
            elif code in (L.T_GT, L.T_LE):
                v = math.floor(fr)
            else:
                v = math.ceil(fr)
        v = int(v)
        if v > hi or v < lo:
            above = v > hi
            return _fold({L.T_EQ: False, L.T_NE: True, L.T_GT: not above, L.T_GE: not above,
                          L.T_LT: above, L.T_LE: above}[code]), [], []
        return code, [v], []
    if kind == 'f':
        if code in (L.T_IN, L.T_NIN):
            vals = sorted(set(float(m) for m in value if not (isinstance(m, float) and m != m)))
            if not vals:
                return _fold(code == L.T_NIN), [], []
            return code, [], vals
        return code, [], [float(value)]
    raise NotImplementedError('where_terms on a column of dtype %s' % dtype)


def parse_agg_list(dtypes, agg_list):
    """create_agg_ctable: -> [(in_col, out_col, op, out_dtype)].

    Accepted forms: 'col' (sum into col), ['col', op], ['col', op, 'out'].
    """
    ops = []
    for info in agg_list:
        if not isinstance(info, list):
            in_col, op, out_col = info, 'sum', info
        else:
            in_col, op = info[0], info[1]
            out_col = in_col if len(info) == 2 else info[2]
        if op not in AGG_OPS:
            raise NotImplementedError('Unknown Aggregation Type: ' + str(op))
        if in_col not in dtypes:
            raise KeyError(str(in_col))
        if op in ('count', 'count_distinct', 'sorted_count_distinct'):
            dt = np.dtype(np.int64)
        elif op in ('mean', 'std'):
            dt = np.dtype(np.float64)
        else:
            dt = np.dtype(dtypes[in_col])
        ops.append((in_col, out_col, op, dt))
    return ops


def any_value_satisfies(values, code, value):
    """True iff some element of ``values`` (a factor cache: the distinct values of a column)
    satisfies the parsed term -- the test ``ctable.where_terms_factorization_check`` applies
    to each term whose column has a ``<col>.values`` cache (worker.py:298) [ext-bquery,
    unverified].  Same exact int / float rules as the row predicate (``normalize``); host
    logic over a handful of cached values, not a row scan."""
    values = np.asarray(values)
    op, ivals, fvals = normalize(values.dtype, code, value)
    if op == L.T_TRUE:
        return len(values) > 0
    if op == L.T_FALSE or len(values) == 0:
        return False
    if values.dtype.kind == 'f':
        x = values.astype(np.float64)
        ref = np.asarray(fvals, np.float64)
    else:
        x = values.astype(np.uint64 if values.dtype == np.uint64 else np.int64)
        ref = np.asarray(ivals, x.dtype) if values.dtype != np.uint64 else np.asarray(
            [v & 0xFFFFFFFFFFFFFFFF for v in ivals], np.uint64)
    if op in (L.T_IN, L.T_NIN):
        hit = np.isin(x, ref)
        return bool(np.any(hit if op == L.T_IN else ~hit))
    v = ref[0]
    hit = {L.T_EQ: x == v, L.T_NE: x != v, L.T_GT: x > v, L.T_GE: x >= v, L.T_LT: x < v, L.T_LE: x <= v}[op]
    return bool(np.any(hit))
