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


def coerce_string(dtype, v):
    """A where-term value as an element of a string column of ``dtype``: bytes for 'S<n>' (a
    str is encoded latin-1 -- the py2 str values of bqueryd's pickled params decode to latin-1
    str, messages.py), str for 'U<n>'."""
    if np.dtype(dtype).kind == 'S':
        if isinstance(v, str):
            return v.encode('latin-1')
        return bytes(v) if isinstance(v, (bytes, bytearray, np.bytes_)) else v
    if isinstance(v, (bytes, bytearray, np.bytes_)):
        return bytes(v).decode('latin-1')
    return v


def string_mask(values, code, value):
    """Which elements of the string array ``values`` satisfy the parsed term (bytes / str
    comparisons, lexicographic; a value of another type never equals and never orders)."""
    values = np.asarray(values)
    dt = values.dtype
    if code in (L.T_IN, L.T_NIN):
        members = [coerce_string(dt, m) for m in value]
        members = [m for m in members if isinstance(m, (bytes, str))]
        # members keep their own width (a longer value must not truncate into a match)
        hit = np.isin(values, np.asarray(members)) if members else np.zeros(len(values), bool)
        return hit if code == L.T_IN else ~hit
    v = coerce_string(dt, value)
    if not isinstance(v, (bytes, str)):
        return np.full(len(values), code == L.T_NE)
    return {L.T_EQ: values == v, L.T_NE: values != v, L.T_GT: values > v, L.T_GE: values >= v,
            L.T_LT: values < v, L.T_LE: values <= v}[code]


def string_term(values_by_code, code, value):
    """A term on a string column as an integer term on its dictionary codes (engine.StringDict:
    ``values_by_code[c]`` is code c's string): the codes whose string satisfies the term, as
    ``in`` (or ``nin`` of the rest, whichever list is shorter), folded to a constant when none
    or all do."""
    hit = string_mask(values_by_code, code, value)
    codes = np.nonzero(hit)[0]
    if len(codes) == 0:
        return L.T_FALSE, [], []
    if len(codes) == len(hit):
        return L.T_TRUE, [], []
    if len(codes) * 2 <= len(hit):
        return L.T_IN, codes.tolist(), []
    return L.T_NIN, np.nonzero(~hit)[0].tolist(), []


def time_value(dtype, code, value):
    """A where-term value on a datetime64 / timedelta64 column as the column's int64 ticks (an
    in-list element by element); ints pass as ticks."""
    dtype = np.dtype(dtype)

    def one(v):
        if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
            return int(v)
        return int(np.asarray(v).astype(dtype).view(np.int64))
    if code in (L.T_IN, L.T_NIN):
        return set(one(v) for v in value)
    return one(value)


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
    if values.dtype.kind in 'SU':
        return bool(np.any(string_mask(values, code, value)))
    if values.dtype.kind in 'Mm':
        values, value = values.view(np.int64), time_value(values.dtype, code, value)
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
