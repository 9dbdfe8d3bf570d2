"""Comparison helpers shared by the parity tests."""
from __future__ import annotations

import numpy as np

# north_star tolerances: bit-exact for keys / counts / distinct counts / integer sums;
# float64 sums and means within 1e-12 relative, float32 within 1e-6.
RTOL_F64 = 1e-12
RTOL_F32 = 1e-6


def assert_tables_equal(got, ref, exact_float_sums=False, ordered=True, rtol=None, exact_cols=None):
    """Compare two OrderedDicts of columns (same names, dtypes, row order).

    Integer/bool columns must match bit for bit.  Float columns match within the
    north_star tolerance, or exactly: all of them when ``exact_float_sums`` (and no
    ``exact_cols``), or the ones named in ``exact_cols``.
    """
    assert list(got.keys()) == list(ref.keys()), (list(got.keys()), list(ref.keys()))
    for name in ref:
        g, r = np.asarray(got[name]), np.asarray(ref[name])
        assert g.dtype == r.dtype, (name, g.dtype, r.dtype)
        assert g.shape == r.shape, (name, g.shape, r.shape)
        if r.dtype.kind == 'f':
            tol = rtol if rtol is not None else (RTOL_F32 if r.dtype == np.float32 else RTOL_F64)
            if (exact_float_sums and exact_cols is None) or (exact_cols is not None and name in exact_cols):
                np.testing.assert_array_equal(g, r, err_msg=name)
            else:
                # relative to the column's magnitude: bquery's incremental (Knuth) mean leaves a
                # ~1e-15 residue where the exact mean is 0, which a pure relative test reads as
                # a 100 % error
                finite = np.abs(r[np.isfinite(r)])
                scale = float(finite.max()) if finite.size else 0.0
                np.testing.assert_allclose(g, r, rtol=tol, atol=tol * scale, equal_nan=True, err_msg=name)
        else:
            np.testing.assert_array_equal(g, r, err_msg=name)


def sort_by_keys(table, keys):
    order = np.lexsort(tuple(table[k] for k in reversed(keys))) if keys else np.arange(
        len(next(iter(table.values()))))
    return type(table)((k, v[order]) for k, v in table.items())
