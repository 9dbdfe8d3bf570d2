"""Randomised differential tests: random shard shapes and random bquery queries through the GPU
path (ShardTable: the library's planner picks the mode) against the numpy restatement of
bquery's calc (oracle/bquery_oracle.py, worker.py:291-323).

Every case is seeded (the parametrize id is the seed): key columns of every kind the worker
meets -- small / wide / unsigned integers, floats with NaN and -0.0, bools, fixed-width bytes
and unicode, datetime64 -- 1-3 of them per query; 1-4 aggregations over value columns (integer
sums wrap like bquery's typed loops, float sums on cents and raw data, NaN / infinities, means,
std, count_distinct and sorted_count_distinct, also of key-like columns); 0-2 where terms of
every operator on values drawn from the column (and values it lacks); row counts from empty to
70 K (past a tile and a private-mode chunk).  Keys, counts, distinct counts and integer sums
bit-exact; float sums, means and std within the north_star 1e-12 (relative to the column's
magnitude); first-appearance group order exact.  Raw-row selection (aggregate=False) on a third
of the cases.
"""
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd.engine import ShardTable
from oracle import bquery_oracle as bo
from tests.helpers import assert_tables_equal

pytestmark = pytest.mark.gpu

N_CASES = 60
SIZES = [0, 1, 5, 257, 4999, 70_001]


def _key_column(rng, kind, n):
    if kind == 'i4':
        return rng.integers(-3, 6, n).astype(np.int32)
    if kind == 'i1':
        return rng.integers(-128, 128, n).astype(np.int8)
    if kind == 'i8w':
        return rng.integers(-2**62, 2**62, 40)[rng.integers(0, 40, n)].astype(np.int64)
    if kind == 'u2':
        return rng.integers(0, 2000, n).astype(np.uint16)
    if kind == 'f8':
        return np.array([-0.0, 0.0, 1.5, np.nan, -2.25, 1e300, 7.0])[rng.integers(0, 7, n)]
    if kind == 'b1':
        return rng.random(n) < 0.3
    if kind == 'S3':
        return np.array([b'', b'a', b'ab', b'abc', b'b', b'zz'], dtype='S3')[rng.integers(0, 6, n)]
    if kind == 'U2':
        return np.array(['', 'x', 'αβ', 'yy'], dtype='U2')[rng.integers(0, 4, n)]
    if kind == 'M8':
        base = np.datetime64('2016-01-01T00:00:00', 's')
        return base + rng.integers(0, 5, n).astype('timedelta64[h]')
    raise ValueError(kind)


def _value_column(rng, kind, n):
    if kind == 'cents':
        return rng.integers(-100_000, 100_000, n) / 100.0
    if kind == 'raw':
        return rng.normal(size=n) * 100.0
    if kind == 'special':
        v = rng.normal(size=n)
        pick = rng.random(n)
        v[pick < 0.02] = np.nan
        v[(pick >= 0.02) & (pick < 0.03)] = np.inf
        v[(pick >= 0.03) & (pick < 0.04)] = -0.0
        return v
    if kind == 'i4':
        return rng.integers(-1000, 1000, n).astype(np.int32)
    if kind == 'i8':
        return rng.integers(-2**62, 2**62, n).astype(np.int64)  # sums wrap modulo 2^64
    if kind == 'u4':
        return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if kind == 'f4':
        return (rng.integers(0, 50, n) / 4.0).astype(np.float32)
    if kind == 'small':
        return rng.integers(0, 4, n).astype(np.int32)  # distinct counts over few values
    raise ValueError(kind)


KEY_KINDS = ['i4', 'i1', 'i8w', 'u2', 'f8', 'b1', 'S3', 'U2', 'M8']
VALUE_KINDS = ['cents', 'raw', 'special', 'i4', 'i8', 'u4', 'f4', 'small']
SUMMABLE = {'cents', 'raw', 'special', 'i4', 'i8', 'u4', 'small'}
# mean / std of a group holding an infinity: bquery's incremental mean turns NaN as soon as any
# row follows the first infinity (inf - inf), where sum / count stays infinite -- a documented
# deviation, so infinities only meet sum / count / distinct counts here
MOMENTS = SUMMABLE - {'special'}
DISTINCTABLE = {'cents', 'i4', 'i8', 'u4', 'f4', 'small', 'special'}


def _term(rng, name, arr):
    """A where term on column ``name`` with a value drawn from the column (or one it lacks)."""
    ops = ['==', '!=', 'in', 'nin', '>', '>=', '<', '<=']
    if arr.dtype.kind == 'b':
        ops = ['==', '!=']
    op = ops[rng.integers(0, len(ops))]
    vals = arr[~np.isnan(arr)] if arr.dtype.kind == 'f' else arr
    if len(vals) == 0 or rng.random() < 0.15:
        absent = {'i': 99, 'u': 1999, 'f': 123.25, 'S': b'qq', 'U': 'qq', 'b': True,
                  'M': np.datetime64('2017-06-01T00:00:00', 's')}
        pool = [absent[arr.dtype.kind]]
    else:
        pool = [vals[i] for i in rng.integers(0, len(vals), 3)]

    def scalar(v):
        if arr.dtype.kind in 'iu':
            return int(v)
        if arr.dtype.kind == 'f':
            return float(v)
        if arr.dtype.kind == 'b':
            return bool(v)
        if arr.dtype.kind == 'S':
            return bytes(v)
        if arr.dtype.kind == 'U':
            return str(v)
        return np.datetime64(v, 's')
    if op in ('in', 'nin'):
        return (name, op, [scalar(v) for v in pool[:int(rng.integers(1, 4))]])
    return (name, op, scalar(pool[0]))


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    n = SIZES[int(rng.integers(0, len(SIZES)))]
    nkeys = int(rng.integers(1, 4))
    key_kinds = [KEY_KINDS[i] for i in rng.choice(len(KEY_KINDS), nkeys, replace=False)]
    val_kinds = [VALUE_KINDS[i] for i in rng.choice(len(VALUE_KINDS), 3, replace=False)]
    cols = OrderedDict()
    for i, k in enumerate(key_kinds):
        cols['k%d_%s' % (i, k)] = _key_column(rng, k, n)
    for i, k in enumerate(val_kinds):
        cols['v%d_%s' % (i, k)] = _value_column(rng, k, n)
    keys = list(cols)[:nkeys]
    aggs = []
    for j in range(int(rng.integers(1, 5))):
        vi = int(rng.integers(0, len(val_kinds)))
        name, kind = 'v%d_%s' % (vi, val_kinds[vi]), val_kinds[vi]
        ops = ['count']
        if kind in SUMMABLE:
            ops += ['sum']
        if kind in MOMENTS:
            ops += ['mean', 'std']
        if kind in DISTINCTABLE:
            ops += ['count_distinct', 'sorted_count_distinct']
        op = ops[int(rng.integers(0, len(ops)))]
        aggs.append([name, op, 'o%d_%s' % (j, op)])
    if rng.random() < 0.3:  # a distinct count of a key-like column
        kname = keys[int(rng.integers(0, nkeys))]
        if cols[kname].dtype.kind in 'iuSUM':
            aggs.append([kname, 'count_distinct', 'okcd'])
    terms = []
    for _ in range(int(rng.integers(0, 3))):
        name = list(cols)[int(rng.integers(0, len(cols)))]
        if cols[name].dtype.kind == 'f' and np.isnan(cols[name]).any() and rng.random() < 0.5:
            continue
        terms.append(_term(rng, name, cols[name]))
    return cols, keys, aggs, terms, rng.random() < 0.33


@pytest.mark.parametrize('seed', range(N_CASES))
def test_random_queries_match_the_oracle(seed, engine_options):
    """A third of the cases run the run-time specialised (hiprtc) kernels at these small
    sizes (option jit_min_rows=0); cases with terms also run bquery's expand_filter_column
    (worker.py:306-307: the mask widened to whole runs of a key column)."""
    cols, keys, aggs, terms, raw_rows = _case(seed)
    if seed % 3 == 1:
        engine_options(jit_min_rows=0)
    elif seed % 3 == 2:
        engine_options(fx_sums=2)  # fixed-point float sums with per-slot shifts
    ref = bo.handle_work(cols, keys, aggs, terms)
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(keys, aggs, where_terms=terms)
        assert_tables_equal(got, ref)
        if terms and len(cols[keys[0]]):
            basket = keys[int(seed) % len(keys)]
            if cols[basket].dtype.kind in 'iub':
                m, _ = t.where(terms)
                e = t.expand_subgroups(basket, m)
                got_e, _ = t.groupby(keys, aggs, mask=e)
                ref_e = bo.handle_work(cols, keys, aggs, terms, expand_filter_column=basket)
                assert_tables_equal(got_e, ref_e)
        if raw_rows:
            sel = list(keys) + [a[0] for a in aggs if a[0] not in keys]
            sel = list(OrderedDict.fromkeys(sel))
            got_rows = t.select_rows(sel, where_terms=terms)
            mask = bo.where_terms(cols, terms) if terms else np.ones(len(cols[keys[0]]), bool)
            ref_rows = OrderedDict((c, cols[c][mask]) for c in sel)
            assert_tables_equal(got_rows, ref_rows, exact_float_sums=True)
    finally:
        t.close()


MERGE_KEY_KINDS = ['i4', 'i1', 'i8w', 'u2', 'f8', 'b1', 'M8']
N_MERGE_CASES = 25


def _merge_case(seed):
    rng = np.random.default_rng(5000 + seed)
    world = int(rng.integers(1, 5))
    n_shards = int(rng.integers(1, 7))
    nkeys = int(rng.integers(1, 3))
    key_kinds = [MERGE_KEY_KINDS[i] for i in rng.choice(len(MERGE_KEY_KINDS), nkeys, replace=False)]
    val_kinds = [VALUE_KINDS[i] for i in rng.choice(len(VALUE_KINDS), 2, replace=False)]
    shards = []
    for _ in range(n_shards):
        n = [0, 3, 900, 12_000, 30_001][int(rng.integers(0, 5))]
        cols = OrderedDict()
        for i, k in enumerate(key_kinds):
            cols['k%d_%s' % (i, k)] = _key_column(rng, k, n)
        for i, k in enumerate(val_kinds):
            cols['v%d_%s' % (i, k)] = _value_column(rng, k, n)
        shards.append(cols)
    keys = list(shards[0])[:nkeys]
    aggs = []
    for j in range(int(rng.integers(1, 4))):
        vi = int(rng.integers(0, 2))
        name, kind = 'v%d_%s' % (vi, val_kinds[vi]), val_kinds[vi]
        ops = ['count']
        if kind in SUMMABLE:
            ops += ['sum']
        if kind in MOMENTS:
            ops += ['mean', 'std']
        if kind in DISTINCTABLE:
            ops += ['count_distinct']
        op = ops[int(rng.integers(0, len(ops)))]
        aggs.append([name, op, 'o%d_%s' % (j, op)])
    terms = []
    if rng.random() < 0.4:
        name = keys[0]
        if shards[0][name].dtype.kind != 'f' and len(shards[0][name]):
            terms.append(_term(rng, name, shards[0][name]))
    return world, shards, keys, aggs, terms


@pytest.mark.parametrize('seed', range(N_MERGE_CASES))
def test_random_merges_match_the_client_merge(seed):
    """The co-located merge (bqg_merge_group_host over in-process ranks: hash partition, pack,
    exchange, receive reduce, per-rank slices into one host result) of random shard results --
    1-6 shards of 0-30 K rows over 1-4 ranks, numeric / bool / datetime keys (NaN and -0.0
    among the float ones), every op whose client merge is a sum of finalized values -- against
    the reference client's merge (rpc.py:164-173) of the oracle's per-shard results, compared
    after sorting by the keys (the merged order is key-hash order at world > 1)."""
    from bqueryd_amd import dist as bdist
    from bqueryd_amd.engine import Device
    from tests.helpers import sort_by_keys
    world, shards, keys, aggs, terms = _merge_case(seed)
    devs = [Device(0) for _ in range(world)]
    tables = [[ShardTable(s, device=devs[r]) for i, s in enumerate(shards) if i % world == r] for r in range(world)]
    per = [[t.groupby_table(keys, aggs, where_terms=terms) for t in ts] for ts in tables]
    dtypes = OrderedDict((k, np.dtype(v)) for k, v in next(p for ps in per for p in ps).dtypes.items())
    group = bdist.CommGroup(devs, transport='local')
    try:
        merged = bdist.merge_group_device(per, keys, aggs, dtypes, group)
    finally:
        group.close()
        for ps in per:
            for p in ps:
                p.close()
        for ts in tables:
            for t in ts:
                t.close()
    ref = bo.client_merge([bo.handle_work(s, keys, aggs, terms) for s in shards], keys, aggs, aggregate=True)
    if ref is None:
        assert merged is None or len(next(iter(merged.values()))) == 0
        return
    got = OrderedDict((k, np.asarray(merged[k])) for k in ref)
    assert_tables_equal(sort_by_keys(got, keys), sort_by_keys(ref, keys))


N_WORKER_CASES = 10
WORKER_KEY_KINDS = ['i4', 'u2', 'f8', 'S3', 'U2', 'M8', 'i8w']


@pytest.mark.parametrize('seed', range(N_WORKER_CASES))
def test_random_worker_messages_match_the_reference_path(seed, tmp_path):
    """The whole drop-in path on random bcolz shards: 1-4 shard files (string, datetime and
    numeric columns) written by bcolz_io, one CalcPath.handle_work per file (worker.py:269-348:
    ctable open, factor caches, where terms, groupby, result ctable + tar) and, for
    aggregate=True, one node-level message over all of them; the controller's tar of tars and
    the client's uncompress_groupby_to_df (rpc.py:134-179) -- against the reference client
    merge of the oracle's per-shard results (sorted by the keys: the reference's own order is
    the glob order, rpc.py:151)."""
    import os
    from bqueryd_amd import bcolz_io, messages, rpc
    from bqueryd_amd.worker import CalcPath
    from tests.helpers import sort_by_keys
    rng = np.random.default_rng(9000 + seed)
    n_files = int(rng.integers(1, 5))
    nkeys = int(rng.integers(1, 3))
    key_kinds = [WORKER_KEY_KINDS[i] for i in rng.choice(len(WORKER_KEY_KINDS), nkeys, replace=False)]
    val_kinds = [VALUE_KINDS[i] for i in rng.choice(len(VALUE_KINDS), 2, replace=False)]
    files, shards = [], []
    for f in range(n_files):
        n = [1, 700, 9_000, 20_001][int(rng.integers(0, 4))]
        cols = OrderedDict()
        for i, k in enumerate(key_kinds):
            cols['k%d_%s' % (i, k)] = _key_column(rng, k, n)
        for i, k in enumerate(val_kinds):
            cols['v%d_%s' % (i, k)] = _value_column(rng, k, n)
        fn = 'shard-%d.bcolzs' % f
        bcolz_io.write_ctable(os.path.join(str(tmp_path), fn), cols)
        files.append(fn)
        shards.append(cols)
    keys = list(shards[0])[:nkeys]
    aggs = []
    for j in range(int(rng.integers(1, 4))):
        vi = int(rng.integers(0, 2))
        name, kind = 'v%d_%s' % (vi, val_kinds[vi]), val_kinds[vi]
        ops = ['count'] + (['sum'] if kind in SUMMABLE else []) + (['mean'] if kind in MOMENTS else []) + \
              (['count_distinct'] if kind in DISTINCTABLE else [])
        aggs.append([name, ops[int(rng.integers(0, len(ops)))], 'o%d' % j])
    terms = []
    if rng.random() < 0.5 and len(shards[0][keys[0]]):
        terms.append(_term(rng, keys[0], shards[0][keys[0]]))
    aggregate = bool(rng.random() < 0.7)

    def msg(fn):
        m = messages.CalcMessage({'payload': 'groupby', 'token': 'ab' * 8, 'filename': fn if isinstance(fn, str) else fn[0]})
        m.set_args_kwargs([fn, keys, aggs, terms], {'aggregate': aggregate})
        return m

    def as_cols(df, like):
        return OrderedDict((c, np.asarray(df[c].values.tolist(), dtype=like[c].dtype) if like[c].dtype.kind in 'SU'
                            else np.asarray(df[c].values).astype(like[c].dtype)) for c in df.columns)

    calc = CalcPath(str(tmp_path))
    per = [bo.handle_work(s, keys, aggs, terms, aggregate=aggregate) for s in shards]
    ref = bo.client_merge(per, keys, aggs, aggregate=aggregate)
    replies = OrderedDict((fn, calc.handle_work(msg(fn))['data']) for fn in files)
    df = rpc.uncompress_groupby_to_df(rpc.tar_of_tars(replies), keys, aggs, terms, aggregate=aggregate)
    if ref is None or len(next(iter(ref.values()))) == 0:
        assert len(df) == 0
        return
    got = as_cols(df, ref)
    if aggregate:
        assert_tables_equal(sort_by_keys(got, keys), sort_by_keys(ref, keys))
    else:
        # raw rows: the per-file results concatenated in file order
        assert_tables_equal(got, ref, exact_float_sums=True)
    if aggregate and n_files > 1:
        node = calc.handle_work(msg(list(files)))
        df_n = rpc.uncompress_groupby_to_df(rpc.tar_of_tars({files[0]: node['data']}), keys, aggs, terms,
                                            aggregate=True)
        assert_tables_equal(sort_by_keys(as_cols(df_n, ref), keys), sort_by_keys(ref, keys))


N_LARGE_CASES = 8


def _large_key(rng, kind, n):
    if kind == 'dense_i4':  # 100 K - 1.5 M groups alone: the partitioned path
        return rng.integers(0, int(rng.integers(100_000, 1_500_000)), n).astype(np.int32)
    if kind == 'pair_u2':
        return rng.integers(0, 700, n).astype(np.uint16)
    if kind == 'pair_i1':
        return rng.integers(-100, 100, n).astype(np.int8)
    if kind == 'wide_i8':
        return rng.integers(-2**50, 2**50, 200_000)[rng.integers(0, 200_000, n)].astype(np.int64)
    if kind == 'sorted_i4':  # clustered keys: every tile holds some group's first row
        return np.sort(rng.integers(0, 300_000, n)).astype(np.int32)
    raise ValueError(kind)


@pytest.mark.parametrize('seed', range(N_LARGE_CASES))
def test_random_large_queries_match_the_c_oracle(seed, oracle_c, engine_options):
    """Random queries at 4.5 M rows -- past the hiprtc threshold, so the run-time specialised
    kernels run -- with 10^5-10^6 groups (the partitioned tile-scatter path, dense or packed
    entries by the value column's codes; sorted keys; hashed wide keys), random numeric value
    dtypes and terms, against the C restatement (oracle/cbquery.c); odd seeds take the
    fixed-point float sums' per-slot shifts (option fx_sums=2)."""
    rng = np.random.default_rng(7000 + seed)
    if seed % 2:
        engine_options(fx_sums=2)
    n = 4_500_000
    layouts = [['dense_i4'], ['pair_u2', 'pair_i1'], ['wide_i8'], ['sorted_i4'], ['pair_i1', 'dense_i4']]
    kinds = layouts[seed % len(layouts)]
    cols = OrderedDict(('k%d' % i, _large_key(rng, k, n)) for i, k in enumerate(kinds))
    val_kinds = [('cents', 'i4'), ('small', 'i8'), ('raw', 'cents'), ('i4', 'f4'), ('cents', 'small'),
                 ('u4', 'raw'), ('cents', 'i8'), ('i8', 'raw')][seed % 8]
    for i, k in enumerate(val_kinds):
        cols['v%d' % i] = _value_column(rng, k, n)
    keys = list(cols)[:len(kinds)]
    aggs = []
    for j in range(int(rng.integers(1, 4))):
        vi = int(rng.integers(0, 2))
        kind = val_kinds[vi]
        ops = ['count'] + (['sum', 'mean'] if kind in SUMMABLE else []) + \
              (['count_distinct', 'sorted_count_distinct'] if kind in DISTINCTABLE else [])
        aggs.append(['v%d' % vi, ops[int(rng.integers(0, len(ops)))], 'o%d' % j])
    terms = []
    if rng.random() < 0.5:
        name = ['v0', 'v1'][int(rng.integers(0, 2))]
        if cols[name].dtype.kind in 'iu':
            op = ['>', '<=', '!=', 'in'][int(rng.integers(0, 4))]
            terms.append((name, op, [int(x) for x in cols[name][:3]] if op == 'in' else int(cols[name][0])))
        else:
            terms.append((name, ['>', '<='][int(rng.integers(0, 2))], float(np.median(cols[name][:1000]))))
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(keys, aggs, where_terms=terms)
    finally:
        t.close()
    ref = oracle_c.groupby(cols, keys, aggs, oracle_c.where_terms(cols, terms) if terms else None)
    assert_tables_equal(got, ref)
