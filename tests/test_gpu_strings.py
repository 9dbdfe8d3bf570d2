"""String (numpy 'S<n>' / 'U<n>') and datetime64 columns on the GPU path.

The reference's own fixture builds its shards from the full taxi frame (string flags, parse_dates
datetimes: /root/reference/tests/test_simple_rpc.py:22-26,79), and bquery factorizes string keys
and compares strings in where_terms [ext-bquery, unverified].  Here a string column lives in HBM
as INT32 dictionary codes made on the GPU (bqg_encode_bytes: code 0 = the empty string, r + 1 =
first-appearance rank r) and a datetime64 column as its int64 ticks; the results must equal the
numpy restatement (oracle/bquery_oracle.py), whose string semantics are pinned against pandas in
tests/test_oracle.py.  Keys, counts and distinct counts bit-exact; first-appearance group order.
"""
import os
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import bcolz_io, messages, rpc, synth
from bqueryd_amd.engine import ShardTable
from oracle import bquery_oracle as bo
from tests.helpers import assert_tables_equal, sort_by_keys

pytestmark = pytest.mark.gpu

COLS = ('payment_type', 'store_and_fwd_flag', 'vendor_name', 'pickup_datetime', 'fare_amount', 'passenger_count')


def _shard(n=120_000, seed_shard=0):
    return synth.taxi_shard(n, config_id=2, n_shards=4, shard=seed_shard, columns=COLS)


def _run(cols, keys, aggs, terms):
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(keys, aggs, where_terms=terms)
    finally:
        t.close()
    ref = bo.handle_work(cols, keys, aggs, terms)
    assert_tables_equal(got, ref)
    return got


@pytest.mark.parametrize('keys', [['store_and_fwd_flag'], ['vendor_name'], ['vendor_name', 'payment_type'],
                                  ['store_and_fwd_flag', 'vendor_name'], ['pickup_datetime']])
def test_string_and_datetime_keys(keys):
    cols = _shard()
    aggs = [['fare_amount', 'sum', 'fs'], ['fare_amount', 'count', 'n'], ['passenger_count', 'count_distinct', 'pcd']]
    got = _run(cols, keys, aggs, [])
    assert got[keys[0]].dtype == cols[keys[0]].dtype


@pytest.mark.parametrize('terms', [
    [('store_and_fwd_flag', '==', 'Y')],
    [('store_and_fwd_flag', '==', b'Y')],
    [('store_and_fwd_flag', '!=', 'N')],
    [('store_and_fwd_flag', '==', '')],
    [('store_and_fwd_flag', 'in', ['Y', 'Q'])],
    [('store_and_fwd_flag', 'nin', ['N', ''])],
    [('store_and_fwd_flag', '==', 'NN')],          # longer than the column's width: no row
    [('vendor_name', '>=', 'DDS'), ('vendor_name', '<', 'VTS')],
    [('vendor_name', 'in', ['CMT', 'VeriFone'])],
    [('vendor_name', '!=', 'nobody')],
    [('pickup_datetime', '>=', np.datetime64('2016-01-15T00:00:00')),
     ('pickup_datetime', '<', np.datetime64('2016-01-20'))],
    [('pickup_datetime', 'in', [np.datetime64('2016-01-01T06:09:49', 'ns'), np.datetime64('2017-01-01')])],
])
def test_string_and_datetime_terms(terms):
    cols = _shard(80_000, 1)
    _run(cols, ['payment_type'], [['fare_amount', 'sum', 'fs'], ['fare_amount', 'count', 'n']], terms)
    t = ShardTable(cols)
    try:
        m, npass = t.where(terms)
        ref = bo.where_terms(cols, terms)
        np.testing.assert_array_equal(t.read(m), ref)
        assert npass == int(ref.sum())
    finally:
        t.close()


def test_distinct_counts_of_strings_and_times():
    """count_distinct and sorted_count_distinct of string and datetime columns -- the empty
    string and the epoch compare like bquery's zero-initialised last value."""
    cols = _shard(150_000, 2)
    rng = np.random.default_rng(3)
    cols['store_and_fwd_flag'] = np.array([b'', b'N', b'Y'], dtype='S1')[rng.integers(0, 3, len(cols['payment_type']))]
    aggs = [['store_and_fwd_flag', 'count_distinct', 'fcd'], ['store_and_fwd_flag', 'sorted_count_distinct', 'fscd'],
            ['vendor_name', 'count_distinct', 'vcd'], ['vendor_name', 'sorted_count_distinct', 'vscd'],
            ['pickup_datetime', 'count_distinct', 'tcd'], ['pickup_datetime', 'sorted_count_distinct', 'tscd']]
    _run(cols, ['payment_type'], aggs, [])
    _run(cols, ['payment_type'], aggs, [('passenger_count', '>', 1)])


def test_cached_string_term_after_repush():
    """A where-term on a string column is planned as a list of dictionary codes and the plan is
    cached per query text; pushing the column again builds a new dictionary, so the cached plan
    must not survive it (engine.ShardTable._touch drops the plans)."""
    rng = np.random.default_rng(4)
    n = 50_000
    cols = OrderedDict(s=np.array([b'A', b'B', b'C'], dtype='S1')[rng.integers(0, 3, n)],
                       v=rng.integers(0, 100, n).astype(np.int64))
    terms = [('s', '==', 'C')]
    aggs = [['v', 'sum', 'vs'], ['v', 'count', 'n']]
    t = ShardTable(cols)
    try:
        for _ in range(2):  # the second query runs the cached plan
            got, _ = t.groupby([], aggs, where_terms=terms)
            assert_tables_equal(got, bo.handle_work(cols, [], aggs, terms))
        # new data, different first-appearance order: 'C' gets another dictionary code
        cols['s'] = np.array([b'C', b'Z', b'A'], dtype='S1')[rng.integers(0, 3, n)]
        t.push('s', cols['s'])
        t.sync()
        got, _ = t.groupby([], aggs, where_terms=terms)
        assert_tables_equal(got, bo.handle_work(cols, [], aggs, terms))
    finally:
        t.close()


def test_wide_strings_many_values_and_select_rows():
    """40-byte keys with ~20 K distinct values (a dictionary larger than the first guess of the
    binding), values that differ only in their last byte, and raw-row selection of strings."""
    rng = np.random.default_rng(9)
    n = 200_000
    base = np.array([('k%036d' % i).encode() + bytes([65 + (i % 3)]) for i in range(20_000)], dtype='S40')
    cols = OrderedDict(k=base[rng.integers(0, len(base), n)], v=rng.integers(0, 100, n).astype(np.int64),
                       u=np.array(['α', 'β', 'αβ', ''], dtype='U2')[rng.integers(0, 4, n)])
    _run(cols, ['k'], [['v', 'sum', 'vs'], ['u', 'count_distinct', 'ucd']], [])
    _run(cols, ['u', 'k'], [['v', 'count', 'n']], [('u', '!=', '')])
    t = ShardTable(cols)
    try:
        got = t.select_rows(['k', 'u', 'v'], where_terms=[('u', '==', 'αβ')])
        ref = bo.handle_work(cols, ['k', 'u'], [['v', 'sum', 'v']], [('u', '==', 'αβ')], aggregate=False)
        assert_tables_equal(got, ref)
        lab, vals = t.factorize('k')
        ref_lab, ref_vals = bo.factorize(cols['k'])
        np.testing.assert_array_equal(lab, ref_lab)
        np.testing.assert_array_equal(vals, ref_vals)
    finally:
        t.close()


def _write_shards(tmp_path, n_shards, rows):
    files, shards = [], []
    for i in range(n_shards):
        s = synth.taxi_shard(rows, config_id=1, n_shards=n_shards, shard=i, columns=COLS)
        fn = 'taxi-%d.bcolzs' % i
        bcolz_io.write_ctable(os.path.join(str(tmp_path), fn), s)
        files.append(fn)
        shards.append(s)
    return files, shards


def _df_cols(df, like):
    """DataFrame columns as arrays of the reference table's dtypes (pandas holds bytes / str
    columns as objects)."""
    return OrderedDict((c, np.asarray(df[c].values.tolist(), dtype=like[c].dtype) if like[c].dtype.kind in 'SU'
                        else df[c].values) for c in df.columns)


def _msg(fn, keys, aggs, where, **kw):
    m = messages.CalcMessage({'payload': 'groupby', 'token': 'cd' * 8, 'filename': fn if isinstance(fn, str) else fn[0]})
    m.set_args_kwargs([fn, keys, aggs, where], kw)
    return m


def test_worker_path_with_string_and_datetime_shards(tmp_path):
    """bcolz shards holding string and datetime columns through the worker (ctable open, factor
    caches, result tar), the controller's tar of tars and the client merge -- per-file messages
    and one node-level message (string keys merge on the host values) against the reference
    client merge of the oracle's per-shard results; then the factorization-check early-out on a
    string value no shard holds."""
    from bqueryd_amd.worker import CalcPath
    files, shards = _write_shards(tmp_path, 3, 40_000)
    keys = ['vendor_name', 'store_and_fwd_flag']
    aggs = [['fare_amount', 'sum', 'fs'], ['fare_amount', 'count', 'n']]
    where = [('pickup_datetime', '>=', np.datetime64('2016-01-05'))]
    calc = CalcPath(str(tmp_path))
    replies = OrderedDict((fn, calc.handle_work(_msg(fn, keys, aggs, where, aggregate=True))['data']) for fn in files)
    per = [bo.handle_work(s, keys, aggs, where) for s in shards]
    ref = bo.client_merge(per, keys, aggs, aggregate=True)
    got = _df_cols(rpc.uncompress_groupby_to_df(rpc.tar_of_tars(replies), keys, aggs, where, aggregate=True), ref)
    assert_tables_equal(sort_by_keys(got, keys), sort_by_keys(ref, keys))
    node = calc.handle_work(_msg(list(files), keys, aggs, where, aggregate=True))
    got_n = _df_cols(rpc.uncompress_groupby_to_df(rpc.tar_of_tars({files[0]: node['data']}), keys, aggs, where,
                                                  aggregate=True), ref)
    assert_tables_equal(sort_by_keys(got_n, keys), sort_by_keys(ref, keys))
    # the factor caches the first groupby wrote (auto_cache) prove 'ZZZ' absent: '' replies
    for fn in files:
        calc.cache.open(os.path.join(str(tmp_path), fn)).flush_caches()
    reply = calc.handle_work(_msg(files[0], keys, aggs, [('vendor_name', '==', 'ZZZ')], aggregate=True))
    assert reply['data'] == ''
