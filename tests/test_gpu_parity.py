"""GPU parity: libbqgpu kernels vs the CPU restatement of bquery (oracle/).

Every comparison is order-sensitive: bquery emits groups in first-appearance order of the
passing rows, and so must the GPU.  Keys, counts, distinct counts and integer sums are
compared bit for bit; float sums are bit-exact on the dyadic ("exact") synthetic data and
within 1e-12 relative otherwise; means/std within 1e-12.
"""
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import synth
from bqueryd_amd.engine import ShardTable
from oracle import bquery_oracle as bo
from tests.helpers import assert_tables_equal

pytestmark = pytest.mark.gpu


def run_both(cols, keys, aggs, terms, oracle_c, exact=False, mask=None):
    t = ShardTable(cols)
    try:
        mname = None
        if mask is not None:
            mname = t.add_column('__m', np.bool_)
            t.push(mname, mask)
            t.sync()
        got, _ = t.groupby(keys, aggs, where_terms=terms, mask=mname)
    finally:
        t.close()
    if mask is not None:
        bool_arr = mask
        if terms:
            bool_arr = bool_arr & oracle_c.where_terms(cols, terms)
    else:
        bool_arr = oracle_c.where_terms(cols, terms) if terms else None
    ref = oracle_c.groupby(cols, keys, aggs, bool_arr)
    # exact data: float sums bit-exact; means / std within tolerance (bquery's Knuth / Welford)
    sums = {(a[2] if isinstance(a, list) and len(a) == 3 else (a[0] if isinstance(a, list) else a))
            for a in aggs if not isinstance(a, list) or a[1] == 'sum'}
    assert_tables_equal(got, ref, exact_cols=sums if exact else set())
    return got


C2 = synth.CONFIGS['c2']
C3 = synth.CONFIGS['c3']
C4 = synth.CONFIGS['c4']


@pytest.mark.parametrize('n', [1, 3, 1000, 1023, 1025, 200_003])
def test_c2_query_small(n, oracle_c):
    cols = synth.taxi_shard(n, config_id=2, columns=synth.query_columns(C2))
    got = run_both(cols, C2['groupby'], C2['aggs'], C2['where'], oracle_c)
    # exact variant: float sums are bit-exact
    ref = oracle_c.handle_work(cols, C2['groupby'], C2['aggs'], C2['where'])
    np.testing.assert_array_equal(got['fare_sum'], ref['fare_sum'])


def test_c3_multikey_dense(oracle_c):
    cols = synth.taxi_shard(300_000, config_id=3, columns=synth.query_columns(C3))
    run_both(cols, C3['groupby'], C3['aggs'], C3['where'], oracle_c, exact=True)


@pytest.mark.parametrize('sort_by', [None, ['pu_location_id', 'passenger_count']])
def test_c4_distinct(sort_by, oracle_c):
    cols = synth.taxi_shard(250_000, config_id=4, columns=synth.query_columns(C4), sort_by=sort_by)
    run_both(cols, C4['groupby'], C4['aggs'], C4['where'], oracle_c)


def test_c4_distinct_filtered(oracle_c):
    cols = synth.taxi_shard(100_000, config_id=4, columns=('pu_location_id', 'passenger_count', 'fare_amount'))
    run_both(cols, ['pu_location_id'], C4['aggs'], [('fare_amount', '>', 9.5)], oracle_c)
    # first row filtered out -> skip slot is label 0 (sorted_count_distinct init rule)
    cols['fare_amount'][0] = 1.0
    run_both(cols, ['pu_location_id'], C4['aggs'], [('fare_amount', '>', 9.5)], oracle_c)


def test_hash_mode_wide_keys(oracle_c):
    rng = np.random.default_rng(7)
    n = 50_000
    base = rng.integers(-2**62, 2**62, 300, dtype=np.int64)
    cols = OrderedDict(k=base[rng.integers(0, 300, n)], v=rng.integers(-1000, 1000, n).astype(np.int32),
                       w=np.round(rng.normal(size=n) * 64) / 64)
    run_both(cols, ['k'], [['v', 'sum', 'vs'], ['w', 'mean', 'wm'], ['v', 'count', 'c']], [], oracle_c)
    run_both(cols, ['k'], [['v', 'sum', 'vs']], [('v', '<', 10)], oracle_c)


def test_hash_mode_multi_key(oracle_c):
    """Two keys whose product exceeds the dense slot space: packed power-of-two fields whose
    ranges (500 000 and 200) are not powers of two."""
    rng = np.random.default_rng(12)
    n = 200_000
    cols = OrderedDict(a=rng.integers(0, 500_000, n).astype(np.int32), b=rng.integers(0, 200, n).astype(np.uint8),
                       v=np.round(rng.normal(size=n) * 64) / 64)
    run_both(cols, ['a', 'b'], [['v', 'sum', 's'], ['v', 'count', 'c']], [], oracle_c, exact=True)
    run_both(cols, ['b', 'a'], [['v', 'mean', 'm']], [('b', '>', 7)], oracle_c)


def _wide_key_cols(n, seed):
    rng = np.random.default_rng(seed)
    i64 = rng.integers(-2**63, 2**63 - 1, 400, dtype=np.int64)
    i64[:2] = [-2**63, 2**63 - 1]  # both ends of the range
    u64 = rng.integers(0, 2**64 - 1, 300, dtype=np.uint64)
    u64[:2] = [0, 2**64 - 1]
    f = np.array([0.5, -0.0, 0.0, np.nan, 3.25, -7.0, 1e300, -1e-300])
    return OrderedDict(a=i64[rng.integers(0, len(i64), n)], u=u64[rng.integers(0, len(u64), n)],
                       f=f[rng.integers(0, len(f), n)], g=rng.integers(0, 5, n).astype(np.int16),
                       v=rng.integers(-1000, 1000, n).astype(np.int64), w=np.round(rng.normal(size=n) * 64) / 64)


def _assert_float_key_tables(got, ref, float_keys):
    """keys compare by value (-0.0 == +0.0, NaN == NaN: bquery's khash identity); the rest exactly
    or within the float tolerance"""
    for k in float_keys:
        np.testing.assert_array_equal(got[k], ref[k])
    assert_tables_equal(OrderedDict((c, v) for c, v in got.items() if c not in float_keys),
                        OrderedDict((c, v) for c, v in ref.items() if c not in float_keys))


@pytest.mark.parametrize('keys', [['a'], ['u'], ['a', 'u'], ['f', 'g'], ['g', 'f', 'a'], ['u', 'f']])
def test_wide_key_spaces(keys, oracle_c):
    """Key spaces the packed 64-bit code cannot hold (hash mode 2): a full-range int64 or
    uint64 key, composite keys wider than 63 bits, float columns inside a multi-column key."""
    cols = _wide_key_cols(120_000, 21)
    aggs = [['v', 'sum', 'vs'], ['w', 'mean', 'wm'], ['v', 'count', 'n'], ['g', 'count_distinct', 'gcd'],
            ['w', 'std', 'wsd']]
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(keys, aggs)
        assert t.dev.last_timing()['mode'] == 3  # global hash
        got_f, _ = t.groupby(keys, aggs[:3], where_terms=[('v', '>', 100)])
    finally:
        t.close()
    ref = oracle_c.groupby(cols, keys, aggs)
    ref_f = oracle_c.groupby(cols, keys, aggs[:3], oracle_c.where_terms(cols, [('v', '>', 100)]))
    fk = [k for k in keys if k == 'f']
    _assert_float_key_tables(got, ref, fk)
    _assert_float_key_tables(got_f, ref_f, fk)


def test_float_key(oracle_c):
    rng = np.random.default_rng(8)
    n = 20_000
    vals = np.array([0.5, -0.0, 0.0, np.nan, 3.25, -7.0])
    cols = OrderedDict(k=vals[rng.integers(0, len(vals), n)], v=rng.integers(0, 9, n).astype(np.int64))
    t = ShardTable(cols)
    got, _ = t.groupby(['k'], [['v', 'sum', 'vs'], ['v', 'count', 'c']])
    ref = oracle_c.groupby(cols, ['k'], [['v', 'sum', 'vs'], ['v', 'count', 'c']])
    # -0.0 / +0.0 are one group; the representative bit pattern may differ
    np.testing.assert_array_equal(got['vs'], ref['vs'])
    np.testing.assert_array_equal(got['c'], ref['c'])
    np.testing.assert_array_equal(np.isnan(got['k']), np.isnan(ref['k']))
    ok = ~np.isnan(ref['k'])
    np.testing.assert_array_equal(got['k'][ok], ref['k'][ok])


@pytest.mark.parametrize('terms', [
    [('passenger_count', 'in', [1, 3, 5])],
    [('passenger_count', 'nin', [1, 3])],
    [('passenger_count', 'in', [2])],
    [('passenger_count', '!=', 1), ('fare_amount', '<=', 12.25)],
    [('passenger_count', '>', 1.5)],
    [('passenger_count', '==', 2.5)],
    [('passenger_count', '<', 100)],
    [('passenger_count', '>=', -5)],
    [('fare_amount', 'in', [10.0, 12.5, 7.25])],
    [('fare_amount', '>=', 8)],
    [('payment_type', 'eq', 0), ('passenger_count', 'neq', 1)],
])
def test_where_variants(terms, oracle_c):
    cols = synth.taxi_shard(60_000, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    run_both(cols, ['payment_type'], [['fare_amount', 'sum', 's'], ['fare_amount', 'count', 'c']], terms,
             oracle_c, exact=True)
    t = ShardTable(cols)
    m, npass = t.where(terms)
    ref = bo.where_terms(cols, terms)
    np.testing.assert_array_equal(t.read(m), ref)
    assert npass == int(ref.sum())


def test_zero_keys_and_empty(oracle_c):
    cols = synth.taxi_shard(10_000, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    aggs = [['fare_amount', 'sum', 's'], ['fare_amount', 'mean', 'm'], ['passenger_count', 'count', 'c']]
    run_both(cols, [], aggs, [], oracle_c)
    run_both(cols, [], aggs, [('passenger_count', '>', 3)], oracle_c)
    run_both(cols, [], aggs, [('passenger_count', '>', 30)], oracle_c)
    run_both(cols, ['payment_type'], aggs, [('passenger_count', '>', 30)], oracle_c)
    # no key, term or summed column: the scan still streams one column (count / distinct only)
    run_both(cols, [], [['passenger_count', 'count', 'c']], [], oracle_c)
    run_both(cols, [], [['passenger_count', 'count_distinct', 'cd'], ['fare_amount', 'count', 'c']], [], oracle_c)
    empty = OrderedDict((k, v[:0]) for k, v in cols.items())
    got, _ = ShardTable(empty).groupby([], aggs)
    ref = bo.groupby(empty, [], aggs)
    assert_tables_equal(got, ref)
    got, _ = ShardTable(empty).groupby(['payment_type'], aggs)
    ref = bo.groupby(empty, ['payment_type'], aggs)
    assert_tables_equal(got, ref)


def test_mask_column(oracle_c):
    cols = synth.taxi_shard(40_000, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    mask = np.random.default_rng(3).random(40_000) < 0.3
    run_both(cols, ['payment_type'], [['fare_amount', 'sum', 's']], [], oracle_c, mask=mask, exact=True)
    run_both(cols, ['payment_type'], [['fare_amount', 'sum', 's']], [('passenger_count', '>=', 2)], oracle_c,
             mask=mask, exact=True)


def test_std_and_dtypes(oracle_c):
    rng = np.random.default_rng(11)
    n = 30_000
    cols = OrderedDict(
        k8=rng.integers(-3, 3, n).astype(np.int8), k16=rng.integers(0, 40, n).astype(np.uint16),
        i8=rng.integers(-128, 127, n).astype(np.int8), u32=rng.integers(0, 2**32 - 1, n, dtype=np.uint32),
        f32=(np.round(rng.normal(size=n) * 16) / 16).astype(np.float32),
        f64=rng.normal(size=n) * 100.0, i64=rng.integers(-2**40, 2**40, n, dtype=np.int64))
    aggs = [['i8', 'sum', 'a'], ['u32', 'sum', 'b'], ['f32', 'sum', 'c'], ['f64', 'std', 'd']]
    run_both(cols, ['k8', 'k16'], aggs, [], oracle_c)
    run_both(cols, ['k8'], [['i64', 'mean', 'm'], ['f64', 'std', 's'], ['i8', 'std', 's2']], [('f64', '>', 0)],
             oracle_c)
    run_both(cols, ['k16'], [['i64', 'sum', 's'], 'f64', ['u32', 'count']], [], oracle_c)


def test_count_distinct_hash_set(oracle_c):
    rng = np.random.default_rng(5)
    n = 40_000
    cols = OrderedDict(k=rng.integers(0, 50, n).astype(np.int32),
                       v=rng.integers(-2**40, 2**40, 500, dtype=np.int64)[rng.integers(0, 500, n)])
    run_both(cols, ['k'], [['v', 'count_distinct', 'cd'], ['v', 'sorted_count_distinct', 'scd']], [], oracle_c)


def _distinct_value_cols(n, seed):
    rng = np.random.default_rng(seed)
    fv = np.concatenate([np.array([0.0, -0.0, np.nan, -np.nan, np.inf, -np.inf, 1e-300, -1e-300]),
                         np.round(rng.normal(size=600) * 64) / 64 + 0.001 * rng.integers(0, 3, 600)])
    i64 = rng.integers(-2**63, 2**63 - 1, 700, dtype=np.int64)
    i64[:2] = [-2**63, 2**63 - 1]
    u64 = rng.integers(0, 2**64 - 1, 500, dtype=np.uint64)
    u64[:2] = [0, 2**64 - 1]
    return OrderedDict(
        k1=rng.integers(0, 40, n).astype(np.int32), k2=rng.integers(0, 7, n).astype(np.int16),
        kw=rng.integers(-2**62, 2**62, 300, dtype=np.int64)[rng.integers(0, 300, n)],
        f64=fv[rng.integers(0, len(fv), n)], f32=fv[rng.integers(0, len(fv), n)].astype(np.float32),
        i64=i64[rng.integers(0, len(i64), n)], u64=u64[rng.integers(0, len(u64), n)],
        w41=rng.integers(-2**41, 2**41, 900, dtype=np.int64)[rng.integers(0, 900, n)],
        p=rng.integers(0, 10, n).astype(np.int32))


@pytest.mark.parametrize('keys', [['k1'], ['k1', 'k2'], ['kw'], ['kw', 'k2'], []])
@pytest.mark.parametrize('terms', [[], [('p', '>=', 3)]])
def test_count_distinct_float_and_wide_values(keys, terms, oracle_c):
    """count_distinct of float values under group keys (NaN one value, -0.0 == +0.0) and of
    integer values whose (slot x value range) pair space reaches 2^63 (full-range int64 /
    uint64, 2^42-wide values under a multi-key group): the pair set keyed by slot and
    representative row (bquery answers these with its per-group hash sets, worker.py:313)."""
    cols = _distinct_value_cols(60_000, 31 + len(keys))
    aggs = [['f64', 'count_distinct', 'cf'], ['f32', 'count_distinct', 'cf32'], ['i64', 'count_distinct', 'ci'],
            ['u64', 'count_distinct', 'cu'], ['w41', 'count_distinct', 'cw'], ['p', 'count', 'n']]
    run_both(cols, keys, aggs, terms, oracle_c)


def test_count_distinct_pair_set_grows(oracle_c, engine_options):
    """The pair set starts too small and is regrown (query re-run) until it holds every pair."""
    cols = _distinct_value_cols(80_000, 77)
    engine_options(distinct_slots=1024)
    run_both(cols, ['k1', 'k2'], [['f64', 'count_distinct', 'cf'], ['i64', 'count_distinct', 'ci']], [], oracle_c)


def test_count_distinct_c4_fare(oracle_c):
    """C4's query shape with fare_amount (float64, cent-rounded) as the distinct column."""
    cols = synth.taxi_shard(300_000, config_id=4, columns=('pu_location_id', 'passenger_count', 'fare_amount'),
                            variant='raw')
    run_both(cols, ['pu_location_id'], [['fare_amount', 'count_distinct', 'fcd'],
                                        ['passenger_count', 'sorted_count_distinct', 'pscd']], [], oracle_c)
    run_both(cols, ['pu_location_id'], [['fare_amount', 'count_distinct', 'fcd'],
                                        ['fare_amount', 'sorted_count_distinct', 'fscd']],
             [('passenger_count', '>', 1)], oracle_c)


@pytest.mark.parametrize('krange', [300, 20_000, 400_000])
def test_sorted_count_distinct_slot_spaces(krange, oracle_c):
    """Chunk-state combine over small, medium and large slot spaces (many runs of chunks per
    slot, a few, and one run per slot)."""
    rng = np.random.default_rng(krange)
    n = 600_000
    cols = OrderedDict(k=rng.integers(0, krange, n).astype(np.int32),
                       v=np.repeat(rng.integers(0, 3, n // 4 + 1), 4)[:n].astype(np.int64))
    run_both(cols, ['k'], [['v', 'sorted_count_distinct', 's'], ['v', 'sum', 'vs']], [], oracle_c)
    run_both(cols, ['k'], [['v', 'sorted_count_distinct', 's']], [], oracle_c)


def test_select_rows_and_expand(oracle_c):
    cols = synth.taxi_shard(50_000, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    terms = [('passenger_count', '>=', 2)]
    t = ShardTable(cols)
    got = t.select_rows(['payment_type', 'fare_amount'], where_terms=terms)
    ref = bo.handle_work(cols, ['payment_type'], [['fare_amount', 'sum', 'x']], terms, aggregate=False)
    assert_tables_equal(got, ref, exact_float_sums=True)
    # expand_filter_column
    m, _ = t.where(terms)
    e = t.expand_subgroups('payment_type', m)
    ref_e = bo.is_in_ordered_subgroups(cols['payment_type'], bo.where_terms(cols, terms))
    np.testing.assert_array_equal(t.read(e), ref_e)


@pytest.mark.parametrize('krange,terms', [(9_000, []), (100_000, [('f', '>', 3)]), (1_500_000, []),
                                          (3_000_000, [('f', 'in', [1, 2, 5])])])
def test_partitioned_mode(krange, terms, oracle_c):
    """Dense slot spaces above the shared-LDS limit: tile scatter -> aggregate."""
    rng = np.random.default_rng(krange)
    n = 400_000
    cols = OrderedDict(k=rng.integers(0, krange, n).astype(np.int32), k2=rng.integers(0, 2, n).astype(np.int8),
                       f=rng.integers(0, 9, n).astype(np.int16), v=np.round(rng.normal(size=n) * 64) / 64,
                       w=rng.integers(-50, 50, n).astype(np.int64))
    run_both(cols, ['k', 'k2'], [['v', 'sum', 'vs'], ['w', 'sum', 'ws'], ['v', 'count', 'c'], ['w', 'mean', 'wm']],
             terms, oracle_c, exact=True)
    mask = rng.random(n) < 0.5
    run_both(cols, ['k'], [['v', 'sum', 'vs']], [], oracle_c, exact=True, mask=mask)


def test_partitioned_four_sums(oracle_c):
    """Four summed columns: the scatter stages four value arrays per tile in LDS."""
    rng = np.random.default_rng(7)
    n = 300_001
    cols = OrderedDict(k=rng.integers(-700_000, 700_000, n).astype(np.int32),
                       a=np.round(rng.normal(size=n) * 64) / 64, b=rng.integers(-9, 9, n).astype(np.int8),
                       c=rng.integers(0, 1 << 40, n).astype(np.uint64), d=rng.random(n).astype(np.float32))
    run_both(cols, ['k'], [['a', 'sum', 'as'], ['b', 'sum', 'bs'], ['c', 'sum', 'cs'], ['d', 'mean', 'dm'],
                           ['a', 'count', 'n']], [('b', '!=', 0)], oracle_c, exact=True)


@pytest.mark.parametrize('jit', [False, True])
@pytest.mark.parametrize('n', [1, 255, 257, 70_001, 400_000])
def test_fused_distinct_pass(n, jit, oracle_c, engine_options):
    """count + count_distinct + sorted_count_distinct on different columns: one fused pass
    (k_scd_fused; precompiled or run-time specialised), checked against the oracle and against
    the unfused kernels."""
    if jit:
        engine_options(jit_min_rows=0)
    rng = np.random.default_rng(n)
    cols = OrderedDict(k=rng.integers(0, 50, n).astype(np.int16), a=rng.integers(-5, 40, n).astype(np.int32),
                       b=np.repeat(rng.integers(0, 4, (n + 9) // 10), 10)[:n].astype(np.int64),
                       f=rng.integers(0, 9, n).astype(np.uint8))
    aggs = [['a', 'count', 'n'], ['a', 'count_distinct', 'acd'], ['b', 'sorted_count_distinct', 'bscd']]
    for terms in ([], [('f', '>', 2)], [('f', 'in', [0, 8])]):
        got = run_both(cols, ['k'], aggs, terms, oracle_c)
        engine_options(fused_scd=0)
        t = ShardTable(cols)
        ref, _ = t.groupby(['k'], aggs, where_terms=terms)
        t.close()
        engine_options(fused_scd=1)
        assert_tables_equal(got, ref)
    # float value column for the sorted distinct, first row filtered out
    cols['b'] = (cols['b'] * 0.5).astype(np.float64)
    cols['f'][0] = 0
    run_both(cols, ['k'], [['b', 'sorted_count_distinct', 's'], ['b', 'count', 'c']], [('f', '>', 0)], oracle_c)


@pytest.mark.parametrize('case', range(6))
def test_specialised_private_scan(case, oracle_c, engine_options):
    """The run-time specialised (hiprtc) private scan against the oracle, forced on at small
    sizes; the precompiled generic kernel must give the same table."""
    engine_options(jit_min_rows=0)
    n = 300_001
    rng = np.random.default_rng(100 + case)
    cols = synth.taxi_shard(n, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    cols['k8'] = rng.integers(-3, 4, n).astype(np.int8)
    cols['u16'] = rng.integers(0, 7, n).astype(np.uint16)
    cols['i64'] = rng.integers(-2**40, 2**40, n)
    cols['f32'] = (np.round(rng.normal(size=n) * 16) / 16).astype(np.float32)
    cases = [
        (['payment_type'], C2['aggs'], C2['where']),
        (['k8'], [['fare_amount', 'sum', 's'], ['i64', 'sum', 'i'], ['f32', 'mean', 'm']],
         [('passenger_count', 'in', [1, 3, 5])]),
        (['u16'], [['fare_amount', 'std', 'sd'], ['passenger_count', 'count', 'c']], [('fare_amount', '<=', 12.25)]),
        ([], [['fare_amount', 'sum', 's'], ['k8', 'sum', 'k']], [('k8', '!=', 0), ('u16', '>', 1)]),
        (['k8'], [['i64', 'mean', 'm'], ['u16', 'sum', 'u']], []),
        (['payment_type'], [['f32', 'sum', 'f']], [('f32', '>', 0.5), ('passenger_count', 'nin', [2])]),
    ]
    keys, aggs, terms = cases[case]
    got = run_both(cols, keys, aggs, terms, oracle_c)
    t = ShardTable(cols)
    t.groupby(keys, aggs, where_terms=terms)
    assert t.dev.last_timing()['specialized'], 'specialised kernel did not run'
    engine_options(jit=0)
    ref, _ = t.groupby(keys, aggs, where_terms=terms)
    assert not t.dev.last_timing()['specialized']
    t.close()
    assert_tables_equal(got, ref, exact_float_sums=True)


@pytest.mark.parametrize('case', range(3))
def test_specialised_partitioned(case, oracle_c, engine_options):
    """The run-time specialised (hiprtc) partition scatter kernel against the oracle, forced on
    at small sizes; the precompiled generic kernel must give the same table."""
    engine_options(jit_min_rows=0)
    n = 500_003
    rng = np.random.default_rng(200 + case)
    cols = synth.taxi_shard(n, config_id=3, columns=synth.query_columns(C3) + ['passenger_count'])
    cols['k64'] = rng.integers(-2**20, 2**20, n)
    cols['u8'] = rng.integers(0, 200, n).astype(np.uint8)
    cases = [
        (C3['groupby'], C3['aggs'], C3['where']),
        (['k64'], [['fare_amount', 'mean', 'm'], ['u8', 'sum', 'u'], ['k64', 'count', 'c']],
         [('passenger_count', '>=', 2)]),
        (['pickup_location'], [['fare_amount', 'sum', 's']], [('u8', 'nin', [3, 4, 5])]),
    ]
    keys, aggs, terms = cases[case]
    got = run_both(cols, keys, aggs, terms, oracle_c)
    t = ShardTable(cols)
    t.groupby(keys, aggs, where_terms=terms)
    timing = t.dev.last_timing()
    assert timing['mode'] == 4 and timing['specialized'], timing
    engine_options(jit=0)
    ref, _ = t.groupby(keys, aggs, where_terms=terms)
    assert not t.dev.last_timing()['specialized']
    t.close()
    assert_tables_equal(got, ref, exact_float_sums=True)


@pytest.mark.parametrize('jit', [False, True])
@pytest.mark.parametrize('low_ranges', [(2, 4), (3,), (4, 3), (8192,), (16384,)])
def test_partition_key_layouts(jit, low_ranges, oracle_c, engine_options):
    """Multi-column keys whose trailing columns stay inside one partition (range products that
    are powers of two <= 2^wbits) and ones that do not; terms on a trailing key column."""
    if jit:
        engine_options(jit_min_rows=0)
    rng = np.random.default_rng(sum(low_ranges) + jit)
    n = 300_007
    kr = 40_000 if int(np.prod(low_ranges)) <= 8 else 500  # keep the slot space dense
    cols = OrderedDict(k=rng.integers(-kr, kr, n).astype(np.int32),
                       v=np.round(rng.normal(size=n) * 64) / 64)
    names = []
    for i, r in enumerate(low_ranges):
        cols['l%d' % i] = (rng.integers(0, r, n) + 7).astype(np.int16 if r > 100 else np.int8 if i else np.int32)
        names.append('l%d' % i)
    keys = ['k'] + names
    run_both(cols, keys, [['v', 'sum', 's'], ['v', 'count', 'c']], [], oracle_c, exact=True)
    run_both(cols, keys, [['v', 'sum', 's']], [(names[-1], '!=', 7)], oracle_c, exact=True)


@pytest.mark.parametrize('threads,splits,per_cu', [(256, None, None), (512, 3, 1), (1024, 64, 8), (1024, 1, 2)])
def test_partitioned_launch_shapes(threads, splits, per_cu, oracle_c, engine_options):
    """Tile sizes (256 / 512 / 1024 scatter threads: 1024- to 4096-row tiles), aggregate tile
    splits (one, three, more splits than some partitions have tiles) and scatter workgroups per
    CU give the same table; a partial last tile and a filter that empties whole tiles."""
    engine_options(part_threads=threads)
    if splits:
        engine_options(part_splits=splits)
    if per_cu:
        engine_options(part_per_cu=per_cu)
    rng = np.random.default_rng(threads + (splits or 0))
    n = 123_457
    cols = OrderedDict(k=rng.integers(0, 200_000, n).astype(np.int32), v=np.round(rng.normal(size=n) * 64) / 64,
                       f=np.where(np.arange(n) // 5000 % 3 == 1, 0, rng.integers(1, 5, n)).astype(np.int16))
    run_both(cols, ['k'], [['v', 'sum', 's'], ['v', 'count', 'c']], [], oracle_c, exact=True)
    run_both(cols, ['k'], [['v', 'sum', 's'], ['v', 'mean', 'm']], [('f', '>', 0)], oracle_c, exact=True)


@pytest.mark.parametrize('splits', [1, 2, 3])
@pytest.mark.parametrize('entries', ['packed', 'narrow', 'wide'])
def test_partitioned_aggregate_window_boundaries(splits, entries, oracle_c, engine_options):
    """The aggregate's window walk at its edges (k_part_aggregate: kAggWin = 1024 tiles of
    bounds per window, chunks of <= 8 tiles): 1024-row tiles (256 scatter threads, part_k 1)
    over 2,500,037 rows = 2442 tiles, so one split walks windows of 1024 + 1024 + 394 tiles and
    two splits 1024 + 197 each -- more tiles per split than one window, a last window that ends
    inside a chunk, a partial last tile -- and three splits (more splits than tiles / kAggWin)
    one window each; for packed, narrow (8-byte) and wide (12-byte) entries.  (Round-3 record:
    an illegal address in an aggregate experiment never committed; this pins the kept kernel's
    window / sentinel / granule indexing at these shapes.)"""
    engine_options(part_threads=256, part_k=1, part_splits=splits)
    if entries != 'packed':
        engine_options(part_pack=0)
    if entries == 'wide':
        engine_options(part_narrow=0)
    rng = np.random.default_rng(1000 + splits)
    n = 2_500_037
    cols = OrderedDict(k=rng.integers(0, 400_000, n).astype(np.int32),
                       v=np.round(rng.normal(size=n) * 300) / 64,
                       f=rng.integers(0, 4, n).astype(np.int8))
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['k'], [['v', 'sum', 'vs'], ['v', 'count', 'n']])
        info = t.dev.last_timing()
        got_f, _ = t.groupby(['k'], [['v', 'sum', 'vs']], where_terms=[('f', '>', 0)])
    finally:
        t.close()
    assert info['mode'] == 4 and bool(info['pack16']) == (entries == 'packed')
    assert bool(info['narrow']) == (entries != 'wide')
    ref = oracle_c.groupby(cols, ['k'], [['v', 'sum', 'vs'], ['v', 'count', 'n']], None)
    ref_f = oracle_c.groupby(cols, ['k'], [['v', 'sum', 'vs']], oracle_c.where_terms(cols, [('f', '>', 0)]))
    assert_tables_equal(got, ref, exact_cols={'vs'})
    assert_tables_equal(got_f, ref_f, exact_cols={'vs'})


@pytest.mark.parametrize('part_k', [1, 2, 4])
@pytest.mark.parametrize('part_win', [64, 1024, 4096])
def test_partitioned_window_and_tile_options(part_win, part_k, oracle_c, engine_options):
    """Every aggregate window (option part_win: tiles of bounds staged in LDS at once) with
    every tile size (option part_k: 4-row chunks per scatter thread; 4 = 16384-row tiles, packed
    entries only), run-time specialised kernels, against the C restatement -- including
    part_k=4 with part_win=4096, whose aggregate asked for more LDS than a CU has until the
    planner clamped the window (gpurun_out/r4d/c3_3.err, api.hip shape()); the planner now
    also checks every launch against the device limits (check_launch)."""
    engine_options(jit=1, jit_min_rows=0, part_win=part_win, part_k=part_k)
    rng = np.random.default_rng(part_win + part_k)
    n = 1_500_007
    cols = OrderedDict(k=rng.integers(0, 300_000, n).astype(np.int32),
                       g=rng.integers(1, 3, n).astype(np.int32),
                       v=np.round(rng.lognormal(2.3, 0.6, n).clip(2.5, 500) * 64) / 64)
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['k', 'g'], [['v', 'sum', 'vs'], ['v', 'count', 'n']])
        info = t.dev.last_timing()
    finally:
        t.close()
    assert info['mode'] == 4 and info['pack16'], info
    ref = oracle_c.groupby(cols, ['k', 'g'], [['v', 'sum', 'vs'], ['v', 'count', 'n']], None)
    assert_tables_equal(got, ref, exact_cols={'vs'})


@pytest.mark.parametrize('order', ['random', 'sorted', 'late'])
@pytest.mark.parametrize('part_first', [0, 1, 2])
def test_partitioned_first_rows_recorded(part_first, order, oracle_c, engine_options):
    """First appearances on the packed path: the tiles below PartLaunch::rit_tiles record each
    entry's row in tile, so the aggregate keys a slot by its exact first row; slots first seen
    in later tiles are keyed by their first tile and resolved by the first-row pass.  Option
    part_first: 0 auto (the tiles where first appearances fall on uniform keys), 1 none (every
    slot through the pass), 2 every tile (no pass) -- on random keys, keys sorted (first
    appearances spread over every tile) and keys whose first appearances come late (a block
    of new keys at the end), with and without a filter; group order must be bquery's."""
    engine_options(part_first=part_first, jit=1, jit_min_rows=0)
    rng = np.random.default_rng(40 + part_first)
    n = 1_200_000
    k = rng.integers(0, 150_000, n).astype(np.int32)
    if order == 'sorted':
        k = np.sort(k)
    elif order == 'late':
        k[-50_000:] = rng.integers(150_000, 260_000, 50_000)
    cols = OrderedDict(k=k, g=rng.integers(1, 3, n).astype(np.int32),
                       v=np.round(rng.lognormal(2.3, 0.6, n).clip(2.5, 500) * 64) / 64,
                       f=rng.integers(0, 5, n).astype(np.int8))
    aggs = [['v', 'sum', 'vs'], ['v', 'count', 'n']]
    for terms in ([], [('f', '>', 0)]):
        t = ShardTable(cols)
        try:
            got, _ = t.groupby(['k', 'g'], aggs, where_terms=terms)
            info = t.dev.last_timing()
        finally:
            t.close()
        assert info['mode'] == 4 and info['pack16'], info
        ref = oracle_c.groupby(cols, ['k', 'g'], aggs, oracle_c.where_terms(cols, terms) if terms else None)
        assert_tables_equal(got, ref, exact_cols={'vs'})


def _groupby_info(cols, keys, aggs, opts=None):
    t = ShardTable(cols)
    try:
        with t.dev.options(**(opts or {})):
            got, _ = t.groupby(keys, aggs)
            info = t.dev.last_timing()
    finally:
        t.close()
    return got, info


@pytest.mark.parametrize('kind', ['dyadic', 'cents', 'f32_dyadic', 'two_sums', 'neg_zero', 'nan', 'huge', 'int_sum',
                                  'int8_only', 'uint32_full', 'int64_wide', 'uint64'])
def test_partitioned_narrow_codes(kind, oracle_c, engine_options):
    """Partitioned sums over float columns whose values all have an exact 32-bit integer code
    (dyadic: v * 2^k; cents: rint(v * 100)) travel as 8-byte entries and are summed as
    integers: dyadic sums bit-exact (and bit-identical to the 64-bit entry path), cents within
    1e-12 of bquery's row-order sum; integer columns spanning fewer than 2^32 values travel
    as v - min (sums bit-exact, wrapping like the 64-bit path); columns without such a code
    (NaN, floats out of int32 range, integers spanning 2^32 or more, uint64) keep the 64-bit
    entries."""
    rng = np.random.default_rng(11)
    n = 300_000
    cols = OrderedDict(k=rng.integers(0, 700_000, n).astype(np.int32))
    aggs = [['v', 'sum', 'vs'], ['v', 'count', 'n']]
    narrow = True
    if kind == 'dyadic':
        cols['v'] = np.round(rng.normal(size=n) * 4000) / 64
    elif kind == 'cents':
        cols['v'] = np.round(rng.lognormal(2.3, 0.6, n) * np.where(rng.random(n) < 0.2, -1, 1), 2)
    elif kind == 'f32_dyadic':
        cols['v'] = (np.round(rng.normal(size=n) * 256) / 16).astype(np.float32)
    elif kind == 'two_sums':
        cols['v'] = np.round(rng.normal(size=n) * 640) / 64
        cols['w'] = np.round(rng.random(n) * 100, 2)
        aggs.append(['w', 'sum', 'ws'])
    elif kind == 'neg_zero':  # -0.0 codes as 0: bquery's sums start at +0.0 (+0.0 + -0.0 == +0.0)
        v = np.round(rng.normal(size=n) * 64) / 64
        v[::7] = -0.0
        v[cols['k'] < 1000] = -0.0  # whole groups of -0.0
        cols['v'] = v
    elif kind == 'nan':
        v = np.round(rng.normal(size=n) * 64) / 64
        v[5] = np.nan
        cols['v'] = v
        narrow = False
    elif kind == 'huge':
        cols['v'] = np.round(rng.normal(size=n) * 1e9, 2)
        narrow = False
    elif kind == 'int_sum':  # an integer summed column beside the float one
        cols['v'] = np.round(rng.normal(size=n) * 64) / 64
        cols['w'] = rng.integers(-9, 9, n).astype(np.int64) + (1 << 40)
        aggs.append(['w', 'sum', 'ws'])
    elif kind == 'int8_only':
        cols['v'] = rng.integers(-128, 128, n).astype(np.int8)
    elif kind == 'uint32_full':  # the whole uint32 range: codes up to 2^32 - 1
        cols['v'] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        cols['v'][:2] = [0, 0xFFFFFFFF]
    elif kind == 'int64_wide':  # spans more than 2^32 values
        cols['v'] = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
        narrow = False
    else:  # uint64
        cols['v'] = rng.integers(0, 1 << 40, n, dtype=np.uint64)
        narrow = False
    got, info = _groupby_info(cols, ['k'], aggs)
    assert info['mode'] == 4 and info['narrow'] == narrow
    ref = oracle_c.groupby(cols, ['k'], aggs, None)
    exact = {'vs'} if kind not in ('cents', 'two_sums', 'huge') else set()
    if kind == 'int_sum':
        exact.add('ws')
    assert_tables_equal(got, ref, exact_cols=exact)
    if narrow:
        wide, winfo = _groupby_info(cols, ['k'], aggs, {'part_narrow': 0})
        assert not winfo['narrow']
        if kind in ('dyadic', 'f32_dyadic', 'neg_zero', 'int_sum', 'int8_only', 'uint32_full'):
            np.testing.assert_array_equal(got['vs'], wide['vs'])
        else:
            np.testing.assert_allclose(got['vs'], wide['vs'], rtol=1e-12, atol=0)


@pytest.mark.parametrize('jit', [False, True])
@pytest.mark.parametrize('case', ['sorted_taxi', 'short_runs', 'wide_values', 'cd_other_column', 'int64_values',
                                  'one_key', 'ragged'])
def test_fused_distinct_runs_loop(case, jit, oracle_c, engine_options):
    """Clustered keys take the fused distinct pass's RUNS loop (256-row steps, 4 rows per lane):
    runs of several lengths (key boundaries inside and across steps and wave chunks), value
    codes above 2^16 (no packed first value), a count_distinct of another column, int64 values,
    a single key value and a ragged row count -- against the oracle and against the 64-row loop
    (scd_runs=0)."""
    if jit:
        engine_options(jit_min_rows=0)
    rng = np.random.default_rng(abs(hash(case)) % 997)
    n = 700_003 if case == 'ragged' else 600_000
    keys = ['k']
    if case == 'short_runs':  # runs of ~600 rows: many key boundaries per wave chunk
        k = np.repeat(rng.integers(0, 300, n // 600 + 1), 600)[:n]
    elif case == 'one_key':
        k = np.zeros(n, np.int64)
    else:
        k = np.sort(rng.integers(0, 265, n))
    cols = OrderedDict(k=k.astype(np.int32))
    v = np.repeat(rng.integers(0, 10, n // 37 + 1), 37)[:n]  # value runs inside key runs
    v[rng.random(n) < 0.05] = 7
    if case == 'wide_values':
        v = v * 30_000
    cols['v'] = v.astype(np.int64 if case == 'int64_values' else np.int32)
    cols['w'] = rng.integers(0, 12, n).astype(np.int16)
    cd_col = 'w' if case == 'cd_other_column' else 'v'
    aggs = [['v', 'sorted_count_distinct', 'scd'], [cd_col, 'count_distinct', 'cd'], ['v', 'count', 'n']]
    got = run_both(cols, keys, aggs, [], oracle_c)
    t = ShardTable(cols)
    try:
        t.groupby(keys, aggs)
        assert t.dev.last_timing()['mode'] == 5
        with t.dev.options(scd_runs=0):
            ref, _ = t.groupby(keys, aggs)
    finally:
        t.close()
    assert_tables_equal(got, ref)


@pytest.mark.parametrize('kind', ['count_only', 'dyadic', 'cents_neg', 'int_span_65535', 'int_span_65536', 'sorted_keys',
                                  'filtered', 'one_split', 'jit', 'flush'])
def test_partitioned_packed_entries(kind, oracle_c, engine_options):
    """Packed 4-byte partition entries {16-bit value code, slot}: no summed column, or one whose
    narrow codes span at most 2^16 values.  First appearance comes from each slot's first tile
    plus a re-read of the marked tiles (k_part_first_rows): group order, keys and counts
    bit-exact against the oracle, sums bit-exact on dyadic data and identical to the 8-byte
    entry path (part_pack=0); a span of 2^16 codes keeps the 8-byte entries; one aggregate
    split over every tile; 'flush': one split whose partition takes ~10.8 M entries, past the
    2^23 entries after which the aggregate flushes its packed accumulators into its record."""
    rng = np.random.default_rng(abs(hash(kind)) % 1000)
    n = 400_003 if kind != 'flush' else 12_000_003
    cols = OrderedDict(k=rng.integers(0, 300_000, n).astype(np.int32),
                       v=np.round(rng.normal(size=n) * 300) / 64)
    aggs = [['v', 'sum', 'vs'], ['v', 'count', 'n']]
    terms = []
    pack = True
    if kind == 'count_only':
        aggs = [['v', 'count', 'n']]
    elif kind == 'cents_neg':
        cols['v'] = np.round(rng.normal(size=n) * 30, 2)  # codes about -15000 .. 15000: base16 < 0
    elif kind == 'int_span_65535':
        cols['v'] = rng.integers(-7, 65_529, n).astype(np.int32)
        cols['v'][:2] = [-7, 65_528]
    elif kind == 'int_span_65536':
        cols['v'] = rng.integers(-7, 65_530, n).astype(np.int32)
        cols['v'][:2] = [-7, 65_529]
        pack = False
    elif kind == 'sorted_keys':  # every tile holds some group's first row
        order = np.argsort(cols['k'], kind='stable')
        cols = OrderedDict((c, a[order]) for c, a in cols.items())
    elif kind == 'filtered':
        cols['f'] = rng.integers(0, 5, n).astype(np.int8)
        terms = [('f', '>', 1)]
    elif kind == 'one_split':
        engine_options(part_splits=1)
        cols['v'] = rng.integers(0, 60_000, n).astype(np.int64)
    elif kind == 'jit':
        engine_options(jit_min_rows=0)
    elif kind == 'flush':
        engine_options(part_splits=1)
        hot = rng.random(n) < 0.9
        cols['k'][hot] = 7
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['k'], aggs, where_terms=terms)
        info = t.dev.last_timing()
        with t.dev.options(part_pack=0):
            wide, _ = t.groupby(['k'], aggs, where_terms=terms)
            winfo = t.dev.last_timing()
    finally:
        t.close()
    assert info['mode'] == 4 and info['pack16'] == pack, info
    assert not winfo['pack16']
    if kind == 'jit':
        assert info['specialized']
    ref = oracle_c.groupby(cols, ['k'], aggs, oracle_c.where_terms(cols, terms) if terms else None)
    exact = {'vs'} if kind not in ('cents_neg',) else set()
    assert_tables_equal(got, ref, exact_cols=exact)
    assert_tables_equal(got, wide, exact_float_sums=True)


@pytest.mark.parametrize('vrange,no_pack', [(7, False), (7, True), (65_536, False), (200_000, False)])
def test_fused_distinct_value_widths(vrange, no_pack, oracle_c, engine_options):
    """The fused distinct pass with 32-bit value codes: first value and first row share one
    LDS word when the codes fit 16 bits (value range <= 2^16), two words otherwise (or with
    option scd_pack16=0); every width against the oracle, at a size that runs the
    specialised kernel over several chunks."""
    engine_options(jit_min_rows=0)
    if no_pack:
        engine_options(scd_pack16=0)
    rng = np.random.default_rng(vrange)
    n = 600_000
    v = rng.integers(-3, vrange - 3, n).astype(np.int32)
    v[:2] = [-3, vrange - 4]  # the full range
    cols = OrderedDict(k=rng.integers(0, 200, n).astype(np.int16),
                       v=np.repeat(v[: n // 3], 3)[:n].astype(np.int32))
    run_both(cols, ['k'], [['v', 'count', 'n'], ['v', 'sorted_count_distinct', 'vscd']], [], oracle_c)


def _regrows_run(cols, keys, aggs, terms, oracle_c):
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(keys, aggs, where_terms=terms)
        timing = t.dev.last_timing()
    finally:
        t.close()
    ref = oracle_c.groupby(cols, keys, aggs, oracle_c.where_terms(cols, terms) if terms else None)
    assert_tables_equal(got, ref, exact_cols={a[2] for a in aggs if a[1] == 'sum'})
    return timing


@pytest.mark.parametrize('keys', [['k'], ['k', 'f']])
def test_hash_table_grows(keys, oracle_c, engine_options):
    """A group hash table started far too small (option hash_slots = 1024) for 40 k distinct
    keys fills past half: the query re-runs with twice the slots until it fits, as bquery's
    khash factorize has no cardinality ceiling (worker.py:313).  Packed keys (hash mode 1) and
    wide keys with a float column (mode 2), filtered and not, against the oracle."""
    engine_options(hash_slots=1024)
    rng = np.random.default_rng(len(keys))
    n = 200_000
    pool = rng.integers(-2**40, 2**40, 40_000)
    cols = OrderedDict(k=pool[rng.integers(0, len(pool), n)], f=np.round(rng.normal(size=n)) / 4,
                       v=np.round(rng.normal(size=n) * 64) / 64)
    aggs = [['v', 'sum', 's'], ['v', 'count', 'n'], ['v', 'mean', 'm']]
    for terms in ([], [('v', '>', -0.5)]):
        timing = _regrows_run(cols, keys, aggs, terms, oracle_c)
        assert timing['mode'] == 3 and timing['regrows'] >= 5, timing
    engine_options(hash_slots=0)
    assert _regrows_run(cols, keys, aggs, [], oracle_c)['regrows'] == 0


def test_distinct_set_grows(oracle_c, engine_options):
    """A count_distinct (group, value) set started at 1024 slots for ~50 k distinct pairs
    (the pair space is too wide for the bitmap) grows the same way."""
    engine_options(distinct_slots=1024)
    rng = np.random.default_rng(3)
    n = 150_000
    cols = OrderedDict(k=rng.integers(0, 12, n).astype(np.int32), w=rng.integers(0, 2**40, 5_000)[rng.integers(0, 5_000, n)])
    timing = _regrows_run(cols, ['k'], [['w', 'count_distinct', 'wcd'], ['w', 'count', 'n']], [], oracle_c)
    assert timing['regrows'] >= 5, timing


def test_engine_options_validate(gpu_device):
    from bqueryd_amd import _lib
    for name in _lib.OPTIONS:
        v = gpu_device.get_option(name)
        gpu_device.set_option(name, v)
    with pytest.raises(_lib.BqgError):
        gpu_device.set_option('no_such_option', 1)
    with pytest.raises(_lib.BqgError):
        gpu_device.set_option('part_threads', 300)
    with pytest.raises(_lib.BqgError):
        gpu_device.set_option('part_wbits', 3)
    gpu_device.reset_options()
    assert gpu_device.get_option('jit') in (0, 1) and gpu_device.get_option('part_narrow') == 1


def _fx_trunc(v, col):
    """v as the fixed-point sums see it: truncated toward zero at 2^-shift, the shift from the
    largest magnitude of the whole column (ScanParams::sum_fx_shift: 95 - frexp exponent)."""
    shift = 95 - int(np.frexp(np.max(np.abs(col)))[1])
    return np.ldexp(np.trunc(np.ldexp(v, shift)), -shift)


def _fsum_by_group(k, v, gk):
    """The correctly rounded exact sum of each group's values (math.fsum), in gk's order."""
    import math
    order = np.argsort(k, kind='stable')
    ks, vs = k[order], v[order]
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    ends = np.r_[starts[1:], len(ks)]
    sums = {ks[a]: math.fsum(vs[a:b]) for a, b in zip(starts, ends)}
    return np.array([sums[g] for g in gk], np.float64)


def _code_sums(keys_codes, ngroups, codes):
    out = np.zeros(ngroups, np.int64)
    np.add.at(out, keys_codes, codes)
    return out


@pytest.mark.parametrize('mode', ['shared', 'global_dense', 'hash', 'partitioned'])
@pytest.mark.parametrize('values', ['cents', 'dyadic', 'cents_big', 'dyadic_big', 'raw'])
def test_atomic_mode_float_sums_reproducible(mode, values, oracle_c, engine_options):
    """The shared / global / hashed atomic modes and the partitioned path's wide entries add
    a float column with an exact integer code per value (cents, dyadic; _big: codes beyond
    32 bits whose int64 sums cannot overflow) as int64 codes: the sums are the same bits on
    every run and equal the exact code sum scaled back once (one correctly rounded division per
    group); means follow.  Arbitrary doubles (raw) accumulate as fixed-point limbs (integer
    atomics, ScanParams::sum_enc 3): the same bits on every run, and -- no value of this data
    has bits below the fixed point -- the correctly rounded exact sum per group (math.fsum);
    their std's centred pass the same.  bquery sums in row order
    (/root/reference/bqueryd/worker.py:313 via bquery's groupby) -- within tolerance of it."""
    rng = np.random.default_rng(11)
    n = 1_500_000
    if mode == 'shared':
        ng = 1000
        k = rng.integers(0, ng, n).astype(np.int32)
    elif mode == 'partitioned':
        ng = 300_000
        k = rng.integers(0, ng, n).astype(np.int32)
    elif mode == 'global_dense':
        engine_options(partition=0)
        ng = 200_000
        k = rng.integers(0, ng, n).astype(np.int32)
    else:
        pool = np.unique(rng.integers(-2**40, 2**40, 30_000))
        ng = len(pool)
        k = pool[rng.integers(0, ng, n)]
    if values == 'cents':
        codes = rng.integers(-500_000, 5_000_000, n)
        v, mul = codes / 100.0, 100.0
    elif values == 'dyadic':
        codes = rng.integers(-2**20, 2**24, n)
        v, mul = np.ldexp(codes.astype(np.float64), -6), 64.0
    elif values == 'cents_big':
        codes = rng.integers(-10**11, 10**12, n)
        v, mul = codes / 100.0, 100.0
    elif values == 'dyadic_big':
        codes = rng.integers(-2**40, 2**41, n)
        v, mul = np.ldexp(codes.astype(np.float64), -6), 64.0
    else:
        v, mul = rng.normal(size=n) * 1e3, None
    cols = OrderedDict(k=k, v=v)
    aggs = [['v', 'sum', 's'], ['v', 'mean', 'm'], ['v', 'count', 'n']]
    if mul is None:
        aggs.append(['v', 'std', 'sd'])
    runs = []
    t = ShardTable(cols)
    try:
        for _ in range(3):
            got, _ = t.groupby(['k'], aggs)
            runs.append(got)
            info = t.dev.last_timing()
    finally:
        t.close()
    assert info['mode'] == {'shared': 1, 'global_dense': 2, 'hash': 3, 'partitioned': 4}[mode], info
    ref = oracle_c.groupby(cols, ['k'], aggs, None)
    assert_tables_equal(runs[0], ref)
    for r in runs[1:]:
        assert_tables_equal(r, runs[0], exact_float_sums=True)
        for name in ('s', 'm') + (('sd',) if mul is None else ()):
            np.testing.assert_array_equal(r[name].view(np.uint64), runs[0][name].view(np.uint64))
    if mul is None:
        np.testing.assert_array_equal(runs[0]['s'], _fsum_by_group(k, _fx_trunc(v, v), runs[0]['k']))
        return
    # the exact code sum per group, scaled back once
    gk = runs[0]['k']
    if mode == 'hash':
        idx = np.searchsorted(pool, k)
        exp = _code_sums(idx, ng, codes)[np.searchsorted(pool, gk)]
    else:
        exp = _code_sums(k, ng, codes)[gk]
    np.testing.assert_array_equal(runs[0]['s'], exp.astype(np.float64) / mul)
    np.testing.assert_array_equal(runs[0]['m'], (exp.astype(np.float64) / mul) / runs[0]['n'].astype(np.float64))


@pytest.mark.parametrize('splits', [0, 3])
@pytest.mark.parametrize('mode', ['shared', 'global_dense', 'hash', 'partitioned'])
def test_fixed_point_sums_mixed_columns(mode, splits, oracle_c, engine_options):
    """Fixed-point float sums (float64 over six decades, float32) beside integer-coded ones, with filters (an odd
    slot count in shared mode: the LDS limb table after an odd-length table stays 8-aligned); the
    partitioned path's split records (part_splits=3) add the limbs in split order; std of a
    coded column (pass 1 integer codes, the centred pass in fixed point); a column holding NaN
    and infinities sums its finite values in fixed point with the non-finite values as flags
    (NaN / +-inf groups whatever the order).  Every run the same bits; per-slot shifts
    (fx_sums=2) the same bits again; option fx_sums=0 restores the float64 atomics for all."""
    if splits and mode != 'partitioned':
        pytest.skip('split records are the partitioned path\'s')
    rng = np.random.default_rng(21 + splits)
    n = 900_000
    if mode == 'global_dense':
        engine_options(partition=0)
    if splits:
        engine_options(part_splits=splits)
    ng = {'shared': 399, 'global_dense': 150_000, 'hash': 0, 'partitioned': 150_000}[mode]
    if mode == 'hash':
        pool = np.unique(rng.integers(-2**40, 2**40, 20_000))
        k = pool[rng.integers(0, len(pool), n)]
    else:
        k = rng.integers(0, ng, n).astype(np.int32)
    raw = rng.normal(size=n) * 10.0 ** rng.integers(-2, 4, n)  # magnitudes over six decades
    raw32 = (rng.normal(size=n) * 7).astype(np.float32)
    cents = rng.integers(-90_000, 90_000, n) / 100.0
    withnan = rng.normal(size=n)
    withnan[rng.integers(0, n, 3)] = np.nan
    withnan[rng.integers(0, n, 3)] = np.inf
    withnan[rng.integers(0, n, 3)] = -np.inf
    t = (rng.random(n) < 0.8).astype(np.int32)
    cols = OrderedDict(k=k, raw=raw, raw32=raw32, cents=cents, withnan=withnan, t=t)
    aggs = [['raw', 'sum', 'a'], ['raw', 'mean', 'am'], ['raw32', 'sum', 'b'], ['cents', 'sum', 'c'],
            ['cents', 'std', 'csd'], ['withnan', 'sum', 'e'], ['raw', 'count', 'n']]
    terms = [('t', '==', 1)]
    if mode == 'partitioned':
        aggs = [a for a in aggs if a[1] != 'std']  # pass-2 std runs the global scan
    runs = []
    tb = ShardTable(cols)
    try:
        for _ in range(2):
            got, _ = tb.groupby(['k'], aggs, where_terms=terms)
            runs.append(got)
            info = tb.dev.last_timing()
        tb.dev.set_option('fx_sums', 2)
        slot, _ = tb.groupby(['k'], aggs, where_terms=terms)
        tb.dev.set_option('fx_sums', 0)
        off, _ = tb.groupby(['k'], aggs, where_terms=terms)
    finally:
        tb.close()
    assert info['mode'] == {'shared': 1, 'global_dense': 2, 'hash': 3, 'partitioned': 4}[mode], info
    # per-slot shifts (fx_sums=2) are never below the column's: the same exact sums, bit for bit
    for name in [a[2] for a in aggs]:
        assert slot[name].tobytes() == runs[0][name].tobytes(), name
    mask = oracle_c.where_terms(cols, terms)
    ref = oracle_c.groupby(cols, ['k'], aggs, mask)
    assert_tables_equal(runs[0], ref)
    assert_tables_equal(off, ref)
    for name in [a[2] for a in aggs]:
        assert runs[1][name].tobytes() == runs[0][name].tobytes(), name
    assert np.isnan(runs[0]['e']).any() and np.isinf(runs[0]['e']).any()
    sel = mask.astype(bool)
    np.testing.assert_array_equal(runs[0]['a'], _fsum_by_group(k[sel], _fx_trunc(raw[sel], raw), runs[0]['k']))


@pytest.mark.parametrize('mode', ['shared', 'global_dense'])
def test_std_of_timestamp_like_columns(mode, oracle_c, engine_options):
    """std's centred pass in fixed point over columns whose spread is far below their magnitude
    (1e12 + k / 8; epoch seconds with sub-millisecond spread): the limb shift leaves headroom for
    a centre an ulp outside [min, max].  Against the exact population std (the values
    minus their base are exact doubles): the centre is the mean rounded to a double, which biases
    the second moment by (mean - centre)^2 -- ~1e-8 of the variance here (DESIGN §4 states the
    bound); bquery's row-order Welford (the oracle) drifts further at such magnitudes."""
    rng = np.random.default_rng(57)
    n = 400_000
    if mode == 'global_dense':
        engine_options(partition=0)
    k = rng.integers(0, 300 if mode == 'shared' else 120_000, n).astype(np.int32)
    v = 1e12 + rng.integers(0, 16, n) * 0.125
    w = 1.7e9 + rng.normal(size=n) * 1e-3  # seconds-since-epoch-like, sub-millisecond spread
    cols = OrderedDict(k=k, v=v, w=w)
    aggs = [['v', 'std', 'vsd'], ['w', 'std', 'wsd'], ['v', 'mean', 'vm'], ['v', 'count', 'n']]
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['k'], aggs)
        info = t.dev.last_timing()
    finally:
        t.close()
    assert info['mode'] == {'shared': 1, 'global_dense': 2}[mode], info
    ref = oracle_c.groupby(cols, ['k'], aggs, None)
    np.testing.assert_array_equal(got['k'], ref['k'])
    np.testing.assert_array_equal(got['n'], ref['n'])
    np.testing.assert_allclose(got['vm'], ref['vm'], rtol=1e-12, atol=0)
    # std against the exact population std of the groups (the values shifted by their base are
    # exact doubles, two passes)
    for name, col, base in (('vsd', v, 1e12), ('wsd', w, 1.7e9)):
        x = col - base
        cnt = np.bincount(k, minlength=int(k.max()) + 1).astype(np.float64)
        mean = np.bincount(k, weights=x) / np.maximum(cnt, 1)
        var = np.bincount(k, weights=(x - mean[k]) ** 2) / np.maximum(cnt, 1)
        # the rounded centre's bias on the variance: (mean - centre)^2, the centre within ~1.5
        # ulp of the magnitude of the exact mean (the pass-1 sum is rounded to a float64 before
        # the division, then the quotient)
        bias = (2.0 * np.spacing(base)) ** 2
        np.testing.assert_allclose(got[name] ** 2, var[got['k']], rtol=1e-9, atol=bias, err_msg=name)


@pytest.mark.parametrize('mode', ['shared', 'global_dense', 'hash', 'partitioned'])
def test_fixed_point_sums_outlier_column(mode, oracle_c, engine_options):
    """A column of values near 1 with one 1e20 outlier: at the column-wide shift (from 1e20) the
    small values would lose their low bits, so its fixed point takes a shift per slot from the
    slot's own largest magnitude (an extra pass, ScanParams::fx_emax) -- every group without
    the outlier is again the correctly rounded exact sum (math.fsum), the outlier's group
    within tolerance of the row-order oracle, and every run the same bits."""
    rng = np.random.default_rng(33)
    n = 600_000
    if mode == 'global_dense':
        engine_options(partition=0)
    if mode == 'hash':
        pool = np.unique(rng.integers(-2**40, 2**40, 4_000))
        k = pool[rng.integers(0, len(pool), n)]
    else:
        k = rng.integers(0, {'shared': 500, 'global_dense': 120_000, 'partitioned': 120_000}[mode], n).astype(np.int32)
    v = rng.normal(size=n)
    out = rng.integers(0, n)
    v[out] = 1e20
    cols = OrderedDict(k=k, v=v)
    aggs = [['v', 'sum', 's'], ['v', 'mean', 'm'], ['v', 'count', 'n']]
    t = ShardTable(cols)
    try:
        runs = [t.groupby(['k'], aggs)[0] for _ in range(2)]
        info = t.dev.last_timing()
    finally:
        t.close()
    assert info['mode'] == {'shared': 1, 'global_dense': 2, 'hash': 3, 'partitioned': 4}[mode], info
    assert_tables_equal(runs[0], oracle_c.groupby(cols, ['k'], aggs, None))
    for name in ('s', 'm'):
        assert runs[1][name].tobytes() == runs[0][name].tobytes(), name
    exact = _fsum_by_group(k, v, runs[0]['k'])
    keep = runs[0]['k'] != k[out]
    np.testing.assert_array_equal(runs[0]['s'][keep], exact[keep])


@pytest.mark.parametrize('mode', ['private', 'shared', 'global_dense', 'partitioned', 'hash'])
def test_moments_of_wrapping_int64_and_coded_columns(mode, oracle_c, engine_options):
    """mean / std next to sum: of an int64 column whose sum wraps the 64-bit accumulator
    (bquery's typed sum wraps, its float64 incremental mean and std do not: the mean / std
    take a float64 sum state of their own), and of a cents column (integer-coded sums in the
    atomic modes and the wide partitioned entries: the std centres decode the codes exactly
    once).  Sums bit-exact (the integer one modulo 2^64), moments within 1e-12."""
    rng = np.random.default_rng(21)
    n = 200_000
    if mode == 'private':
        k = rng.integers(0, 6, n).astype(np.int32)
    elif mode == 'shared':
        k = rng.integers(0, 900, n).astype(np.int32)
    elif mode == 'global_dense':
        engine_options(partition=0)
        k = rng.integers(0, 150_000, n).astype(np.int32)
    elif mode == 'partitioned':
        k = rng.integers(0, 150_000, n).astype(np.int32)
    else:
        k = rng.integers(-2**40, 2**40, 5_000)[rng.integers(0, 5_000, n)]
    cols = OrderedDict(k=k, big=rng.integers(2**61, 2**62, n).astype(np.int64),
                       c=rng.integers(-10**11, 10**11, n) / 100.0)
    aggs = [['big', 'sum', 'bs'], ['big', 'mean', 'bm'], ['big', 'std', 'bsd'],
            ['c', 'sum', 'cs'], ['c', 'mean', 'cm'], ['c', 'std', 'csd'], ['c', 'count', 'n']]
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['k'], aggs)
        info = t.dev.last_timing()
    finally:
        t.close()
    assert info['mode'] == {'private': 0, 'shared': 1, 'global_dense': 2, 'hash': 3, 'partitioned': 4}[mode], info
    ref = bo.groupby(cols, ['k'], aggs)
    assert_tables_equal(got, ref, exact_cols={'bs'})


@pytest.mark.parametrize('compact', [1, 2])
@pytest.mark.parametrize('mode', ['shared', 'global_dense'])
def test_code_copies_without_narrow_codes(mode, compact, oracle_c, engine_options):
    """part_narrow=0 turns the atomic modes' integer-coded float sums off, so the plan gives a
    cents / dyadic column fixed-point limbs; the compact scan then still reads the column's code
    copy and sums the codes as integers -- that state is no limb sum any more and must not be
    finalized as one (the emit decoded a double's bits as a code sum).  Against the
    oracle and against the full-width scan."""
    rng = np.random.default_rng(41 + compact)
    n = 250_000
    engine_options(part_narrow=0, compact=compact)
    if mode == 'global_dense':
        engine_options(partition=0)
    k = rng.integers(0, 200 if mode == 'shared' else 140_000, n).astype(np.int32)
    cols = OrderedDict(k=k, c=rng.integers(-50_000, 90_000, n) / 100.0,
                       f=rng.integers(-20_000, 40_000, n) / 100.0,
                       d=np.ldexp(rng.integers(-2**20, 2**20, n).astype(np.float64), -5),
                       r=rng.normal(size=n) * 1e3, t=rng.integers(0, 4, n).astype(np.int32))
    aggs = [['c', 'sum', 'cs'], ['f', 'sum', 'fs'], ['f', 'mean', 'fm'], ['d', 'sum', 'ds'], ['r', 'sum', 'rs'],
            ['c', 'count', 'n']]
    terms = [('t', '!=', 2)]
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['k'], aggs, where_terms=terms)
        info = t.dev.last_timing()
        with t.dev.options(compact=0):
            full, _ = t.groupby(['k'], aggs, where_terms=terms)
    finally:
        t.close()
    assert info['mode'] == {'shared': 1, 'global_dense': 2}[mode], info
    assert info['bytes_read'] < info['bytes'], info  # the code copies were read
    ref = oracle_c.groupby(cols, ['k'], aggs, oracle_c.where_terms(cols, terms))
    assert_tables_equal(got, ref, exact_cols={'ds'})
    assert_tables_equal(full, ref, exact_cols={'ds'})
    np.testing.assert_array_equal(got['ds'], full['ds'])  # dyadic: the exact sum either way
    # the code copies sum the cents codes exactly: the correctly rounded DECIMAL sum (the
    # full-width limbs give the correctly rounded sum of the float64 inputs -- within tolerance
    # of it, not bit-equal)
    sel = oracle_c.where_terms(cols, terms).astype(bool)
    for name, col in (('cs', 'c'), ('fs', 'f')):
        codes = np.rint(cols[col] * 100).astype(np.int64)
        sums = np.zeros(int(k.max()) + 1, np.int64)
        np.add.at(sums, k[sel], codes[sel])
        np.testing.assert_array_equal(got[name], sums[got['k']].astype(np.float64) / 100.0)


@pytest.mark.parametrize('mode', ['private', 'shared', 'global_dense'])
def test_compact_resident_copies(mode, oracle_c, engine_options):
    """Compact resident copies (option compact): narrow integer offsets for keys / terms /
    integer sums (negative minima, every width), exact int32 codes for a float64 column that is
    only summed (cents and dyadic) -- the same answers as the full-width scan and the oracle,
    fewer algorithmic bytes; a pushed column rebuilds its copy (the next query sees the new
    values); a float column in a term keeps its full width."""
    rng = np.random.default_rng(31)
    n = 300_000
    if mode == 'private':
        k = rng.integers(-5, 3, n).astype(np.int64)              # 8 values of an int64 key
    elif mode == 'shared':
        k = rng.integers(-400, 500, n).astype(np.int32)
    else:
        engine_options(partition=0)
        k = rng.integers(-70_000, 60_000, n).astype(np.int32)
    cols = OrderedDict(k=k, t=rng.integers(-30_000, 30_000, n).astype(np.int32),
                       i=rng.integers(-2**40, -2**40 + 200, n).astype(np.int64),
                       c=rng.integers(-50_000, 90_000, n) / 100.0,
                       d=np.ldexp(rng.integers(-2**20, 2**20, n).astype(np.float64), -5),
                       f=rng.integers(-20_000, 40_000, n) / 100.0,       # cents spanning < 2^16: 2-byte codes
                       g=np.ldexp(rng.integers(-100, 100, n).astype(np.float64), -2))  # 1-byte dyadic codes
    aggs = [['c', 'sum', 'cs'], ['c', 'mean', 'cm'], ['d', 'sum', 'ds'], ['i', 'sum', 'is'], ['i', 'count', 'n']]
    terms = [('t', '>=', -12_345)]
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['k'], aggs, where_terms=terms)
        info = t.dev.last_timing()
        with t.dev.options(compact=0):
            full, _ = t.groupby(['k'], aggs, where_terms=terms)
            finfo = t.dev.last_timing()
        assert info['mode'] == finfo['mode'] == {'private': 0, 'shared': 1, 'global_dense': 2}[mode], (info, finfo)
        # k: 1 B / 2 B / 4 B offsets (from 8 / 4 / 4), t 2 B (from 4), i 1 B (from 8), c / d 4 B (from 8)
        # algorithmic bytes are the stored widths either way; the copies read fewer
        assert info['bytes'] == finfo['bytes'] == finfo['bytes_read'], (info, finfo)
        assert info['bytes_read'] < finfo['bytes_read'], (info['bytes_read'], finfo['bytes_read'])
        ref = oracle_c.groupby(cols, ['k'], aggs, oracle_c.where_terms(cols, terms))
        assert_tables_equal(got, ref, exact_cols={'ds', 'is'})
        assert_tables_equal(full, ref, exact_cols={'ds', 'is'})
        # float64 sums over codes spanning fewer than 2^16 / 2^8: 2 / 1-byte offsets from the
        # smallest code
        aggs4 = [['f', 'sum', 'fs'], ['f', 'mean', 'fm'], ['g', 'sum', 'gs'], ['g', 'count', 'n']]
        got4, _ = t.groupby(['k'], aggs4, where_terms=terms)
        info4 = t.dev.last_timing()
        with t.dev.options(compact=0):
            full4, _ = t.groupby(['k'], aggs4, where_terms=terms)
            finfo4 = t.dev.last_timing()
        # f 8 -> 2 B, g 8 -> 1 B, t 4 -> 2 B per row, k as above
        kd = {'private': 7, 'shared': 2, 'global_dense': 0}[mode]
        assert finfo4['bytes_read'] - info4['bytes_read'] == (kd + 6 + 7 + 2) * n, (info4, finfo4)
        ref4 = oracle_c.groupby(cols, ['k'], aggs4, oracle_c.where_terms(cols, terms))
        assert_tables_equal(got4, ref4, exact_cols={'gs'})
        assert_tables_equal(full4, ref4, exact_cols={'gs'})
        # new values in a column: its copy is rebuilt
        cols['t'] = rng.integers(-100, 100_000, n).astype(np.int32)
        t.push('t', cols['t'])
        t.sync()
        got2, _ = t.groupby(['k'], aggs, where_terms=terms)
        ref2 = oracle_c.groupby(cols, ['k'], aggs, oracle_c.where_terms(cols, terms))
        assert_tables_equal(got2, ref2, exact_cols={'ds', 'is'})
        # a float column in a term is read at full width (its value, not its code, compares)
        got3, _ = t.groupby(['k'], [['c', 'sum', 'cs']], where_terms=[('c', '>', 12.34)])
        ref3 = oracle_c.groupby(cols, ['k'], [['c', 'sum', 'cs']], oracle_c.where_terms(cols, [('c', '>', 12.34)]))
        assert_tables_equal(got3, ref3)
    finally:
        t.close()


@pytest.mark.gpu
@pytest.mark.parametrize('jit', [1, 0])
def test_compact_term_bounds(jit, oracle_c, engine_options):
    """Scalar terms on a compact integer column compare in the copy's domain (stored = value -
    min, a 32-bit compare in specialised kernels): every operator at and around the column's
    minimum and maximum, beyond both, and at the int64 extremes -- the same rows pass as in the
    oracle, in the private scan and in the shared scan."""
    engine_options(jit=jit, jit_min_rows=0)
    rng = np.random.default_rng(77)
    n = 50_000
    for kvals, vlo, vhi in ((6, -5, 300), (700, 1000, 1200)):
        cols = OrderedDict(k=rng.integers(0, kvals, n).astype(np.int32),
                           t=rng.integers(vlo, vhi + 1, n).astype(np.int64),
                           x=rng.integers(-1000, 1000, n).astype(np.int64))
        t = ShardTable(cols)
        try:
            consts = [vlo - 1, vlo, vlo + 1, vhi - 1, vhi, vhi + 1, -2**40, 2**40, 2**33 + vlo,
                      -2**63, 2**63 - 1, 0, -1]
            for op in ('==', '!=', '<', '<=', '>', '>='):
                for c in consts:
                    terms = [('t', op, c)]
                    got, _ = t.groupby(['k'], [['x', 'sum', 'xs'], ['x', 'count', 'n']], where_terms=terms)
                    ref = oracle_c.groupby(cols, ['k'], [['x', 'sum', 'xs'], ['x', 'count', 'n']],
                                           oracle_c.where_terms(cols, terms))
                    assert_tables_equal(got, ref, exact_cols={'xs', 'n'})
        finally:
            t.close()


def test_compact_copies_accounting(oracle_c):
    """The compact copies' HBM is visible (bqg_table_device_bytes: what ShardCache budgets), they
    can be built ahead of a query and released, the timing reports their build on the query
    that made them, and a query answers the same with or without them."""
    rng = np.random.default_rng(12)
    n = 400_000
    cols = OrderedDict(k=rng.integers(0, 9, n).astype(np.int32), p=rng.integers(0, 10, n).astype(np.int32),
                       v=np.round(rng.lognormal(2.3, 0.6, n).clip(2.5, 500) * 64) / 64)
    aggs = [['v', 'sum', 's'], ['v', 'mean', 'm'], ['v', 'count', 'n']]
    terms = [('p', '>=', 2)]
    ref = oracle_c.groupby(cols, ['k'], aggs, oracle_c.where_terms(cols, terms))
    t = ShardTable(cols)
    try:
        base = t.device_bytes()
        assert base >= sum(a.nbytes for a in cols.values())
        t.dev.enable_timing(True)
        with t.dev.options(compact=1):
            got, _ = t.groupby(['k'], aggs, where_terms=terms)
            first = t.dev.last_timing()
            again, _ = t.groupby(['k'], aggs, where_terms=terms)
            second = t.dev.last_timing()
        with t.dev.options(compact=0):
            full, _ = t.groupby(['k'], aggs, where_terms=terms)
            finfo = t.dev.last_timing()
        t.dev.enable_timing(False)
        assert first['compact_ms'] > 0 and second['compact_ms'] == 0, (first, second)
        assert first['bytes'] == finfo['bytes'] == finfo['bytes_read'] > first['bytes_read'], (first, finfo)
        grown = t.device_bytes()
        assert grown > base
        t.drop_compact()
        assert t.device_bytes() == base
        assert t.build_compact(['k', 'p', 'v']) == 3 and t.device_bytes() > base  # (pooled blocks: caps may differ)
        for g in (got, again, full):
            assert_tables_equal(g, ref, exact_cols={'s'})
    finally:
        t.close()


def test_column_memory_budget(oracle_c):
    """Option mem_cap_mb (a context's budget for resident column memory): compact copies that do
    not fit are not built -- the scan reads the columns as stored, same answer; a table that
    fits only without another table's copies releases them (a rebuildable cache) instead of
    failing, and the copies are not rebuilt past the budget; a table that cannot fit fails with
    an out-of-memory error and leaves the context and its tables usable (the shadow
    allocation failure path)."""
    from bqueryd_amd._lib import BqgError
    from bqueryd_amd.engine import Device
    rng = np.random.default_rng(13)
    n = 2_000_000
    MB = 1 << 20

    def shard():
        return OrderedDict(k=rng.integers(0, 9, n).astype(np.int32), p=rng.integers(0, 10, n).astype(np.int32),
                           v=np.round(rng.lognormal(2.3, 0.6, n).clip(2.5, 500) * 64) / 64)
    aggs = [['v', 'sum', 's'], ['v', 'count', 'n']]
    terms = [('p', '>=', 2)]
    dev = Device(0)  # a context of its own: its pool holds this test's columns only
    tables = []
    try:
        dev.set_option('compact', 1)
        a_cols = shard()
        ref = oracle_c.groupby(a_cols, ['k'], aggs, oracle_c.where_terms(a_cols, terms))
        a = ShardTable(a_cols, device=dev)
        tables.append(a)
        base = a.device_bytes()  # 16 B/row; the copies take 4 B/row (1 + 1 + 2-byte codes)
        # (budgets in whole MiB: base + 0.5 MiB rounded up leaves less headroom than the smallest
        # copy, 2 M one-byte codes)
        dev.set_option('mem_cap_mb', -(-(base + MB // 2) // MB))
        dev.enable_timing(True)
        got, _ = a.groupby(['k'], aggs, where_terms=terms)
        info = dev.last_timing()
        assert info['bytes_read'] == info['bytes'] and a.device_bytes() == base, info
        assert_tables_equal(got, ref, exact_cols={'s'})
        # room for A and its copies, and for B only without them
        dev.set_option('mem_cap_mb', -(-(2 * base + MB // 2) // MB))
        got, _ = a.groupby(['k'], aggs, where_terms=terms)
        assert dev.last_timing()['bytes_read'] < info['bytes'] and a.device_bytes() > base
        b_cols = shard()
        b = ShardTable(b_cols, device=dev)
        tables.append(b)
        assert a.device_bytes() == base and b.device_bytes() == base
        for t, c in ((a, a_cols), (b, b_cols)):
            got, _ = t.groupby(['k'], aggs, where_terms=terms)
            assert dev.last_timing()['bytes_read'] == info['bytes']  # no room to rebuild the copies
            assert_tables_equal(got, oracle_c.groupby(c, ['k'], aggs, oracle_c.where_terms(c, terms)), exact_cols={'s'})
        with pytest.raises(BqgError, match='allocation'):
            tables.append(ShardTable(shard(), device=dev))
        got, _ = b.groupby(['k'], aggs, where_terms=terms)
        assert_tables_equal(got, oracle_c.groupby(b_cols, ['k'], aggs, oracle_c.where_terms(b_cols, terms)),
                            exact_cols={'s'})
    finally:
        for t in tables:
            t.close()
        dev.close()


@pytest.mark.parametrize('opt,val', [('part_wbits', 6), ('part_wbits', 10), ('part_wbits', 13), ('scd_compact', 0),
                                     ('priv_ahead', 1), ('priv_ahead', 2), ('priv_ahead', 4),
                                     ('private_per_cu', 1), ('private_per_cu', 3), ('small_emit', 0),
                                     ('part_ring', 1), ('part_ring', 2), ('slot_emit', 0)])
def test_remaining_engine_options(opt, val, oracle_c, engine_options):
    """The engine options no other test sets, each at non-default values, on the query shape
    it steers (partition width and the scatter's ring: a partitioned C3-shaped query; the fused distinct pass's value
    codes: C4; the private scan's tiles in flight and workgroups per CU, run-time specialised:
    C2; the one-workgroup emit off: a shared-mode query), against the C restatement -- so that
    every option value the header lists has run against the oracle."""
    engine_options(**{opt: val, 'jit': 1, 'jit_min_rows': 0})
    rng = np.random.default_rng(sum(map(ord, opt)) * 16 + val)
    n = 400_003
    if opt in ('part_wbits', 'part_ring', 'slot_emit'):  # (part_ring: packed entries, each block's spare tile)
        cols = OrderedDict(k=rng.integers(0, 90_000, n).astype(np.int32), g=rng.integers(1, 3, n).astype(np.int32),
                           v=np.round(rng.normal(size=n) * 64) / 64)
        keys, aggs, terms, mode = ['k', 'g'], [['v', 'sum', 's'], ['v', 'count', 'n']], [], 4
    elif opt == 'scd_compact':
        cols = synth.taxi_shard(n, config_id=4, columns=synth.query_columns(C4))
        keys, aggs, terms, mode = C4['groupby'], C4['aggs'], C4['where'], 5
    elif opt == 'small_emit':
        cols = OrderedDict(k=rng.integers(0, 900, n).astype(np.int32), v=rng.integers(-50, 50, n).astype(np.int64))
        keys, aggs, terms, mode = ['k'], [['v', 'sum', 's'], ['v', 'mean', 'm'], ['v', 'count', 'n']], [('v', '!=', 3)], 1
    else:
        cols = synth.taxi_shard(n, config_id=2, columns=synth.query_columns(C2))
        keys, aggs, terms, mode = C2['groupby'], C2['aggs'], C2['where'], 0
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(keys, aggs, where_terms=terms)
        info = t.dev.last_timing()
    finally:
        t.close()
    assert info['mode'] == mode, info
    ref = oracle_c.groupby(cols, keys, aggs, oracle_c.where_terms(cols, terms) if terms else None)
    assert_tables_equal(got, ref)


def _same_bits(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and (a.dtype.kind == 'O' and list(a) == list(b) or
                                                          a.dtype.kind != 'O' and a.tobytes() == b.tobytes())


@pytest.mark.parametrize('shape', ['partitioned', 'hash', 'wide_keys', 'nonfinite_std', 'distinct', 'filtered_empty',
                                   'device_table'])
def test_slot_emit_matches_compaction_emit(shape, oracle_c, engine_options):
    """Round 6's large-result emit (option slot_emit: the first-row bitmap set straight from the
    slot arrays, the group count left on the device for the emit's column layout and read by
    the host while the emit runs -- no compaction pass, no host round trip before the emit)
    against the compaction emit it replaces, bit for bit, on each slot mode with more than 8192
    slots (slot_emit 1: first rows marked in the epoch row map; 2: per-group records, then the
    columns; 3: first rows marked by bitmap atomics), and
    against the C restatement.  (nonfinite_std: a std over a column holding NaN / infinities
    keeps the fixed-point limbs, so its finite groups are the same bits run to run.)"""
    rng = np.random.default_rng(sum(map(ord, shape)))
    n = 300_007
    terms = []
    if shape == 'partitioned':
        cols = OrderedDict(k=rng.integers(0, 90_000, n).astype(np.int32), g=rng.integers(1, 3, n).astype(np.int32),
                           v=np.round(rng.normal(size=n) * 64) / 64)
        keys, aggs = ['k', 'g'], [['v', 'sum', 's'], ['v', 'count', 'n']]
    elif shape == 'hash':
        pool = rng.integers(-2**40, 2**40, 40_000)
        cols = OrderedDict(k=pool[rng.integers(0, pool.size, n)], v=rng.integers(-1000, 1000, n).astype(np.int64))
        keys, aggs = ['k'], [['v', 'sum', 's'], ['v', 'mean', 'm']]
    elif shape == 'wide_keys':
        pool = rng.normal(size=30_000) * 1e6
        cols = OrderedDict(f=pool[rng.integers(0, pool.size, n)], i=rng.integers(0, 3, n).astype(np.int64) << 40,
                           v=rng.integers(0, 100, n).astype(np.int32))
        keys, aggs = ['f', 'i'], [['v', 'sum', 's'], ['v', 'count', 'n']]
    elif shape == 'nonfinite_std':
        v = np.round(rng.normal(size=n) * 16) / 16
        v[rng.integers(0, n, 300)] = np.nan
        v[rng.integers(0, n, 300)] = np.inf
        cols = OrderedDict(k=rng.integers(0, 20_000, n).astype(np.int32), v=v)
        keys, aggs = ['k'], [['v', 'mean', 'm'], ['v', 'std', 'sd'], ['v', 'sum', 's']]
    elif shape == 'distinct':
        cols = OrderedDict(k=rng.integers(0, 20_000, n).astype(np.int32), d=rng.integers(0, 7, n).astype(np.int32))
        keys, aggs = ['k'], [['d', 'count_distinct', 'cd'], ['d', 'sorted_count_distinct', 'scd']]
    else:
        cols = OrderedDict(k=rng.integers(0, 50_000, n).astype(np.int32), v=rng.integers(0, 100, n).astype(np.int64))
        keys, aggs = ['k'], [['v', 'sum', 's'], ['v', 'count', 'n']]
        if shape == 'filtered_empty':
            terms = [('v', '>', 1000)]
    t = ShardTable(cols)
    try:
        runs = []
        for se in (1, 2, 3, 0):
            engine_options(slot_emit=se)
            if shape == 'device_table':
                r = t.groupby_table(keys, aggs)
                try:
                    runs.append((r.to_host(), False))
                finally:
                    r.close()
            else:
                runs.append(t.groupby(keys, aggs, where_terms=terms))
    finally:
        t.close()
    old, fold = runs[-1]
    for got, fgot in runs[:-1]:
        assert fgot == fold and list(got) == list(old)
        for c in got:
            assert _same_bits(got[c], old[c]), c
    new, fnew = runs[0]
    if shape == 'filtered_empty':
        assert fnew and all(len(x) == 0 for x in new.values())
        return
    ref = oracle_c.groupby(cols, keys, aggs, None)
    assert_tables_equal(new, ref)


def test_slot_emit_row_map_epochs(oracle_c, engine_options):
    """The row map of the large-result emit holds one byte per row, the query's epoch (1..255),
    and is cleared only when the epoch wraps or the map grows: 300 large-result queries on one
    context -- past a wrap -- alternating two tables whose first rows differ, then a larger
    table (the map grows) and the first again, each against the C restatement."""
    rng = np.random.default_rng(255)

    def shard(n, k):
        return OrderedDict(k=rng.integers(0, k, n).astype(np.int32), v=rng.integers(0, 100, n).astype(np.int64))

    a_cols, b_cols, big_cols = shard(40_000, 20_000), shard(30_000, 15_000), shard(120_000, 30_000)
    aggs = [['v', 'sum', 's'], ['v', 'count', 'n']]
    refs = {}
    tables = {}
    try:
        for name, cols in (('a', a_cols), ('b', b_cols), ('big', big_cols)):
            tables[name] = ShardTable(cols)
            refs[name] = oracle_c.groupby(cols, ['k'], aggs, None)
        for q in range(300):
            name = 'a' if q % 2 == 0 else 'b'
            got, _ = tables[name].groupby(['k'], aggs)
            if q % 37 == 0 or q >= 250:
                assert_tables_equal(got, refs[name])
        for name in ('big', 'a', 'big'):
            got, _ = tables[name].groupby(['k'], aggs)
            assert_tables_equal(got, refs[name])
    finally:
        for t in tables.values():
            t.close()
