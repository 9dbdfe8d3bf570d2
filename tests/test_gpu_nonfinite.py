"""GPU parity of mean / std over float columns holding NaN or infinities.

bquery's mean is Knuth's row-order update ``c += 1; m += (x - m) / c`` and its std Welford's
(worker.py:313-314 [ext-bquery]; oracle/bquery_oracle.py ``aggregate_one``): once a group has
seen an infinity, the next row computes ``inf - inf`` and the mean becomes NaN, so a group's mean
is +-inf only when its one non-finite value is its LAST passing row, and NaN for any other
non-finite pattern; its std is NaN as soon as any non-finite value arrives.  libbqgpu gates this
on the column statistics and runs its nonfinite pass (last passing row per group, count and last
row of the non-finite values) -- these tests pin every placement, in every mode, against the C
and numpy restatements, with filters that drop or keep the decisive rows.
"""
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd.engine import ShardTable
from oracle import bquery_oracle as bo
from tests.helpers import assert_tables_equal

pytestmark = pytest.mark.gpu

MODES = {'private': 0, 'shared': 1, 'global_dense': 2, 'hash': 3, 'partitioned': 4}


def _keys(mode, rng, n):
    if mode == 'private':
        return rng.integers(0, 12, n).astype(np.int32)
    if mode == 'shared':
        return rng.integers(0, 700, n).astype(np.int32)
    if mode in ('global_dense', 'partitioned'):
        return rng.integers(0, 60_000, n).astype(np.int32)
    return rng.integers(-2**40, 2**40, 3_000)[rng.integers(0, 3_000, n)]  # sparse int64: hash mode


def _plant(k, v, t, rng):
    """Non-finite values at every placement that decides the row-order mean, each in its own
    group (rows of a group in row order); returns the groups used."""
    uniq, counts = np.unique(k, return_counts=True)
    groups = [g for g in uniq[counts >= 5]]
    rng.shuffle(groups)
    it = iter(groups)
    rows = {}

    def take():
        g = next(it)
        rows[g] = np.flatnonzero(k == g)
        return rows[g]

    inf, nan = np.inf, np.nan
    r = take(); v[r[0]] = inf                      # first row: NaN after the next row
    r = take(); v[r[len(r) // 2]] = -inf           # middle
    r = take(); v[r[-1]] = inf                     # last row: the mean stays +inf
    r = take(); v[r[-1]] = -inf                    # last row, negative: -inf
    r = take(); v[r[-2]] = inf; v[r[-1]] = inf     # two infinities at the end: NaN
    r = take(); v[r[-1]] = nan                     # NaN last
    r = take(); v[r[1]] = nan                      # NaN in the middle
    r = take(); v[r[0]] = -inf; v[r[-1]] = inf     # both signs
    r = take(); v[r[-2]] = inf; t[r[-1]] = 0       # the filter drops the row after it: +inf
    r = take(); v[r[-1]] = -inf; t[r[-1]] = 0      # the filter drops the infinity itself
    r = take(); v[r[0]] = inf; t[r[1:]] = 0        # the infinity is the group's only passing row
    r = take(); v[r[2]] = nan; t[r[2]] = 0         # a filtered NaN
    return rows


def _run(cols, keys, aggs, terms, oracle_c):
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(keys, aggs, where_terms=terms)
        info = t.dev.last_timing()
    finally:
        t.close()
    mask = oracle_c.where_terms(cols, terms) if terms else None
    ref_c = oracle_c.groupby(cols, keys, aggs, mask)
    ref_np = bo.groupby(cols, keys, aggs, bool_arr=mask)
    assert_tables_equal(got, ref_c)
    assert_tables_equal(got, ref_np)
    return got, info


@pytest.mark.parametrize('filtered', [False, True])
@pytest.mark.parametrize('mode', list(MODES))
def test_mean_std_nonfinite_placements(mode, filtered, oracle_c, engine_options):
    rng = np.random.default_rng(77 + MODES[mode])
    n = 150_000
    if mode == 'global_dense':
        engine_options(partition=0)
    k = _keys(mode, rng, n)
    v = rng.integers(-5_000, 90_000, n) / 100.0
    t = np.ones(n, np.int32)
    _plant(k, v, t, rng)
    cols = OrderedDict(k=k, v=v, t=t)
    aggs = [['v', 'sum', 's'], ['v', 'mean', 'm'], ['v', 'std', 'sd'], ['v', 'count', 'n']]
    got, info = _run(cols, ['k'], aggs, [('t', '==', 1)] if filtered else [], oracle_c)
    assert info['mode'] == MODES[mode], info
    m = got['m']
    assert np.isposinf(m).any() and np.isnan(m).any(), 'the planted placements did not reach the result'
    if filtered:
        assert np.isneginf(m).sum() == 1  # the -inf last row without a filter on it


@pytest.mark.parametrize('jit', [0, 1])
def test_mean_nonfinite_float32_and_jit(jit, oracle_c, engine_options):
    """A float32 column (means over its float64 values), the pass-1 scan specialised or not."""
    engine_options(jit=jit, jit_min_rows=0)
    rng = np.random.default_rng(5)
    n = 60_000
    k = rng.integers(0, 14, n).astype(np.int32)
    v = (rng.integers(-500, 900, n) / 4.0).astype(np.float32)
    t = np.ones(n, np.int32)
    _plant(k, v, t, rng)
    cols = OrderedDict(k=k, v=v, t=t)
    _run(cols, ['k'], [['v', 'mean', 'm'], ['v', 'std', 'sd'], ['v', 'count', 'n']], [('t', '>', 0)], oracle_c)


def test_mean_nonfinite_wide_keys(oracle_c):
    """Hash mode 2 (a float column in a multi-column key): the nonfinite pass looks each row's
    slot up by its representative row."""
    rng = np.random.default_rng(9)
    n = 80_000
    a = rng.integers(0, 40, n).astype(np.int32)
    b = rng.integers(0, 30, n) / 4.0
    k = a.astype(np.int64) * 1000 + (b * 4).astype(np.int64)  # one group id for the planting
    v = rng.integers(0, 10_000, n) / 100.0
    t = np.ones(n, np.int32)
    _plant(k, v, t, rng)
    cols = OrderedDict(a=a, b=b, v=v, t=t)
    _, info = _run(cols, ['a', 'b'], [['v', 'mean', 'm'], ['v', 'std', 'sd'], ['v', 'sum', 's']],
                   [('t', '!=', 0)], oracle_c)
    assert info['mode'] == 3, info


def test_mean_finite_column_skips_the_pass(oracle_c):
    """Finite data (every config): the plan has no nonfinite pass and the private inline emit
    stays (one launch fewer); results as before."""
    rng = np.random.default_rng(3)
    n = 50_000
    cols = OrderedDict(k=rng.integers(0, 5, n).astype(np.int32), v=rng.integers(0, 9_000, n) / 64.0)
    got, info = _run(cols, ['k'], [['v', 'mean', 'm'], ['v', 'count', 'n']], [], oracle_c)
    assert info['mode'] == 0 and np.isfinite(got['m']).all()
