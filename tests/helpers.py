"""Comparison helpers shared by the parity tests."""
from __future__ import annotations

import numpy as np

# north_star tolerances: bit-exact for keys / counts / distinct counts / integer sums;
# float64 sums and means within 1e-12 relative, float32 within 1e-6.
RTOL_F64 = 1e-12
RTOL_F32 = 1e-6


def assert_tables_equal(got, ref, exact_float_sums=False, ordered=True, rtol=None):
    """Compare two OrderedDicts of columns (same names, dtypes, row order).

    Integer/bool columns must match bit for bit.  Float columns match within the
    north_star tolerance (or exactly when ``exact_float_sums``).
    """
    assert list(got.keys()) == list(ref.keys()), (list(got.keys()), list(ref.keys()))
    for name in ref:
        g, r = np.asarray(got[name]), np.asarray(ref[name])
        assert g.dtype == r.dtype, (name, g.dtype, r.dtype)
        assert g.shape == r.shape, (name, g.shape, r.shape)
        if r.dtype.kind == 'f':
            tol = rtol if rtol is not None else (RTOL_F32 if r.dtype == np.float32 else RTOL_F64)
            if exact_float_sums:
                np.testing.assert_array_equal(g, r, err_msg=name)
            else:
                np.testing.assert_allclose(g, r, rtol=tol, atol=0, equal_nan=True, err_msg=name)
        else:
            np.testing.assert_array_equal(g, r, err_msg=name)


def sort_by_keys(table, keys):
    order = np.lexsort(tuple(table[k] for k in reversed(keys))) if keys else np.arange(
        len(next(iter(table.values()))))
    return type(table)((k, v[order]) for k, v in table.items())
