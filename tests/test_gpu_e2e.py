"""GPU end to end: golden fixtures through the bquery-compatible ctable API, the worker calc
path (CalcPath.handle_work) over bcolz shards, the controller's tar-of-tars and the client
merge, and full-size (BASELINE) parity for config C2."""
import json
import os
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import bcolz_io, messages, rpc, synth
from bqueryd_amd.ctable import ctable
from bqueryd_amd.worker import CalcPath
from oracle import bquery_oracle as bo
from tests.helpers import assert_tables_equal, sort_by_keys

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
with open(os.path.join(GOLDEN, 'cases.json')) as _f:
    CASES = json.load(_f)
SINGLE = [k for k in CASES if k != 'c1_multishard']


def load_case(name):
    q = CASES[name]
    z = np.load(os.path.join(GOLDEN, name + '.npz'))
    cols = OrderedDict((c, z['in__' + c]) for c in q['inputs'])
    out = OrderedDict((c, z['out__' + c]) for c in q['outputs'])
    return q, cols, out


@pytest.mark.parametrize('name', SINGLE)
def test_golden_via_ctable_api(name):
    q, cols, out = load_case(name)
    ct = ctable(columns=cols)
    try:
        where = [tuple(t) for t in q['where']]
        bool_arr = ct.where_terms(where, cache=True) if where else None
        if q.get('expand'):
            bool_arr = ct.is_in_ordered_subgroups(basket_col=q['expand'], bool_arr=bool_arr)
        if q.get('aggregate', True):
            got = ct.groupby(q['groupby'], q['aggs'], bool_arr=bool_arr).columns
        else:
            got = ct.select(list(q['groupby']) + [x[0] for x in q['aggs']], bool_arr=bool_arr).columns
    finally:
        ct.close()
    assert_tables_equal(got, out)


def _calc_msg(filename, groupby, aggs, where, **kwargs):
    m = messages.CalcMessage({'payload': 'groupby', 'token': 'ab' * 8, 'filename': filename})
    m.set_args_kwargs([filename, groupby, aggs, where], kwargs)
    return m


def test_worker_controller_client_path(tmp_path):
    q = CASES['c1_multishard']
    z = np.load(os.path.join(GOLDEN, 'c1_multishard.npz'))
    data_dir = str(tmp_path)
    files = []
    for i in range(q['shards']):
        shard = OrderedDict((c, z['shard%d__%s' % (i, c)]) for c in q['inputs'])
        fn = 'tripdata-%d.bcolzs' % i
        bcolz_io.write_ctable(os.path.join(data_dir, fn), shard)
        files.append(fn)
    calc = CalcPath(data_dir)
    replies = OrderedDict()
    for fn in files:
        msg = calc.handle_work(_calc_msg(fn, q['groupby'], q['aggs'], []))
        assert isinstance(msg['data'], bytes) and msg['data']
        replies[fn] = msg['data']
    blob = rpc.tar_of_tars(replies)
    ref_merged = OrderedDict((c, z['merged__' + c]) for c in q['outputs'])
    got = rpc.uncompress_groupby_to_df(blob, q['groupby'], q['aggs'], [], aggregate=True)
    got = OrderedDict((c, got[c].values) for c in got.columns)
    assert_tables_equal(sort_by_keys(got, q['groupby']), sort_by_keys(ref_merged, q['groupby']))
    # default (no aggregate kwarg at the client): per-shard tables concatenated
    concat = rpc.uncompress_groupby_to_df(blob, q['groupby'], q['aggs'], [])
    ref_concat = OrderedDict((c, z['concat__' + c]) for c in ref_merged)
    assert_tables_equal(OrderedDict((c, concat[c].values) for c in concat.columns), ref_concat)
    # aggregate=False at the worker: raw filtered rows
    msg = calc.handle_work(_calc_msg(files[0], ['payment_type'], [['fare_amount', 'sum', 'x']],
                                     [('passenger_count', '>=', 2)], aggregate=False))
    back = rpc.read_shard_results(rpc.tar_of_tars({files[0]: msg['data']}))[0]
    shard0 = OrderedDict((c, z['shard0__' + c]) for c in q['inputs'])
    ref = bo.handle_work(shard0, ['payment_type'], [['fare_amount', 'sum', 'x']], [('passenger_count', '>=', 2)],
                         aggregate=False)
    assert_tables_equal(back, ref, exact_float_sums=True)


@pytest.mark.parametrize('variant', ['exact', 'raw'])
def test_c1_full_shape_end_to_end(tmp_path, variant, oracle_c):
    """C1 at its stated shape (BASELINE.json configs[0]): 10 bcolz shards x 1 M rows on disk,
    one per-file calc message per shard through CalcPath.handle_work (cold, then warm from the
    resident shard cache), the controller's tar of tars and the client's aggregate=True merge
    -- against the reference client merge (rpc.py:164-173) of bquery's per-shard results
    (the C restatement): keys exact, sums bit-exact on dyadic data, 1e-12 on cents."""
    cfg = synth.CONFIGS['c1']
    data_dir = str(tmp_path)
    files, results = [], []
    for i in range(cfg['shards']):
        cols = synth.taxi_shard(cfg['rows'] // cfg['shards'], config_id=1, n_shards=cfg['shards'], shard=i,
                                variant=variant, columns=synth.query_columns(cfg))
        fn = 'tripdata-%d.bcolzs' % i
        bcolz_io.write_ctable(os.path.join(data_dir, fn), cols)
        files.append(fn)
        results.append(oracle_c.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where']))
    ref = bo.client_merge(results, cfg['groupby'], cfg['aggs'], aggregate=True)
    calc = CalcPath(data_dir)
    for rep in ('cold', 'warm'):
        replies = OrderedDict()
        for fn in files:
            replies[fn] = calc.handle_work(_calc_msg(fn, cfg['groupby'], cfg['aggs'], cfg['where']))['data']
        df = rpc.uncompress_groupby_to_df(rpc.tar_of_tars(replies), cfg['groupby'], cfg['aggs'], cfg['where'],
                                          aggregate=True)
        got = OrderedDict((c, df[c].values) for c in df.columns)
        got, exp = sort_by_keys(got, cfg['groupby']), sort_by_keys(ref, cfg['groupby'])
        assert_tables_equal(got, exp, exact_cols={'fare_amount'} if variant == 'exact' else set())


def test_worker_factorization_check_and_errors(tmp_path):
    cols = synth.taxi_shard(5000, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    root = os.path.join(str(tmp_path), 's.bcolzs')
    bcolz_io.write_ctable(root, cols)
    # a bquery factor cache of payment_type values (auto_cache side effect of earlier queries)
    bcolz_io.write_carray(os.path.join(root, 'payment_type.values'), np.unique(cols['payment_type']))
    calc = CalcPath(str(tmp_path))
    msg = calc.handle_work(_calc_msg('s.bcolzs', ['passenger_count'], [['fare_amount', 'sum', 'f']],
                                     [('payment_type', '==', 42)]))
    assert msg['data'] == ''  # worker.py:298-301 early out
    msg = calc.handle_work(_calc_msg('s.bcolzs', ['passenger_count'], [['fare_amount', 'sum', 'f']],
                                     [('payment_type', 'in', [1, 42])]))
    assert msg['data']
    with pytest.raises(Exception, match='does not exist'):
        calc.handle_work(_calc_msg('missing.bcolzs', ['a'], [['b', 'sum', 'b']], []))
    with pytest.raises(KeyError):
        calc.handle_work(_calc_msg('s.bcolzs', ['nope'], [['fare_amount', 'sum', 'f']], []))


def _write_shards(tmp_path, n_shards, rows, extra=None):
    files, shards = [], []
    for i in range(n_shards):
        s = synth.taxi_shard(rows, config_id=5, n_shards=n_shards, shard=i,
                             columns=('pickup_location', 'vendor_id', 'passenger_count', 'fare_amount'))
        s['pickup_location'] = (s['pickup_location'] % 5_000).astype(np.int32)
        if extra:
            extra(s)
        fn = 'tripdata-%d.bcolzs' % i
        bcolz_io.write_ctable(os.path.join(str(tmp_path), fn), s)
        files.append(fn)
        shards.append(s)
    return files, shards


@pytest.mark.parametrize('aggs, where, expand', [
    ([['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']], [], None),
    ([['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']], [('passenger_count', '>=', 2)], None),
    ([['fare_amount', 'mean', 'fm'], ['passenger_count', 'count_distinct', 'pcd']], [('vendor_id', '==', 2)], None),
    ([['fare_amount', 'sum', 'fare_sum']], [('passenger_count', '==', 3)], 'basket'),
])
def test_node_level_calc_matches_per_shard_replies(tmp_path, aggs, where, expand):
    """One message with the node's files (args[0] a list, aggregate=True) -> ONE result tar
    holding the GPU-merged table (bqg_merge over RCCL); the unchanged client merge of that tar
    equals the client merge of the per-file replies (controller.py:471-508, rpc.py:164-173)."""
    def add_basket(s):
        s['basket'] = (np.arange(len(s['vendor_id'])) // 5).astype(np.int32)
    files, shards = _write_shards(tmp_path, 5, 30_000, extra=add_basket)
    keys = ['pickup_location', 'vendor_id']
    calc = CalcPath(str(tmp_path))
    kwargs = {'aggregate': True}
    if expand:
        kwargs['expand_filter_column'] = expand
    msg = calc.handle_work(_calc_msg(files, keys, aggs, where, **kwargs))
    assert msg['filenames'] == files and msg['data']
    got = rpc.uncompress_groupby_to_df(rpc.tar_of_tars({'node': msg['data']}), keys, aggs, where, aggregate=True)
    got = OrderedDict((c, got[c].values) for c in got.columns)
    per = [bo.handle_work(s, keys, aggs, where, expand_filter_column=expand) for s in shards]
    ref = bo.client_merge(per, keys, aggs, aggregate=True)
    assert_tables_equal(sort_by_keys(got, keys), sort_by_keys(ref, keys))
    # the same answer through the per-file path (the default)
    replies = OrderedDict((fn, calc.handle_work(_calc_msg(fn, keys, aggs, where, **kwargs))['data']) for fn in files)
    per_file = rpc.uncompress_groupby_to_df(rpc.tar_of_tars(replies), keys, aggs, where, aggregate=True)
    per_file = OrderedDict((c, per_file[c].values) for c in per_file.columns)
    assert_tables_equal(sort_by_keys(per_file, keys), sort_by_keys(ref, keys))
    # the patched controller (restated in rpc.fan_out / rpc.route /
    # rpc.CalcSegment): files 0-2 on the GPU worker (one message pinned to it, one reply), files
    # 3-4 per file on a CPU worker; file 0 is replicated on the CPU worker too, so an unpinned
    # node message could have reached a worker without files 1-2.  The RPC completes when every
    # file is covered and the client merge of the gathered tar is the same answer
    workers = {'gpu-w': {'workertype': 'calc', 'gpu_node': True}, 'cpu-w': {'workertype': 'calc'}}
    fmap = {f: {'gpu-w'} for f in files[:3]}
    fmap.update({f: {'cpu-w'} for f in files[3:]})
    fmap[files[0]] = {'gpu-w', 'cpu-w'}
    seg = rpc.CalcSegment(files)
    sent = rpc.fan_out([files, keys, aggs, where], kwargs, workers, fmap)
    assert sent[0]['args'][0] == files[:3] and len(sent) == 3
    assert [rpc.route(m, workers, fmap) for m in sent] == ['gpu-w', 'cpu-w', 'cpu-w']
    for m in reversed(sent):
        assert not seg.complete
        reply = calc.handle_work(_calc_msg(m['args'][0], keys, aggs, where, **kwargs))
        done = seg.add_reply(reply.get_args_kwargs()[0], reply['data'])
    assert done
    mixed = rpc.uncompress_groupby_to_df(seg.tar(), keys, aggs, where, aggregate=True)
    mixed = OrderedDict((c, mixed[c].values) for c in mixed.columns)
    assert_tables_equal(sort_by_keys(mixed, keys), sort_by_keys(ref, keys))


def test_node_level_calc_needs_explicit_aggregate(tmp_path):
    files, _ = _write_shards(tmp_path, 2, 1000)
    calc = CalcPath(str(tmp_path))
    with pytest.raises(ValueError, match='aggregate=True'):
        calc.handle_work(_calc_msg(files, ['vendor_id'], [['fare_amount', 'sum', 'f']], []))


def test_auto_cache_factor_files_and_check(tmp_path):
    """A groupby with auto_cache=True writes bquery's <col>.factor / <col>.values caches
    (labels = first-appearance rank over all rows, values in label order); the factorization
    check over them agrees with the oracle's on every term shape (worker.py:291, 298-301)."""
    files, shards = _write_shards(tmp_path, 1, 40_000)
    root = os.path.join(str(tmp_path), files[0])
    calc = CalcPath(str(tmp_path))
    calc.handle_work(_calc_msg(files[0], ['passenger_count', 'vendor_id'], [['fare_amount', 'sum', 'f']], []))
    ct = calc.cache.open(root)
    ct.flush_caches()
    for col in ('passenger_count', 'vendor_id'):
        labels, uniq = bo.factorize(shards[0][col])
        np.testing.assert_array_equal(bcolz_io.read_carray(os.path.join(root, col + '.factor')), labels)
        np.testing.assert_array_equal(bcolz_io.read_carray(os.path.join(root, col + '.values')), uniq)
        assert ct.cache_valid(col)
    assert not ct.cache_valid('fare_amount')  # not a groupby column: no cache
    values = {c: bcolz_io.read_carray(os.path.join(root, c + '.values')) for c in ('passenger_count', 'vendor_id')}
    for terms in ([('passenger_count', '==', 42)], [('passenger_count', '==', 3)], [('passenger_count', '>', 9)],
                  [('passenger_count', '>=', 9)], [('passenger_count', '<', 0)], [('passenger_count', '<=', 0.5)],
                  [('passenger_count', 'in', [11, 12])], [('passenger_count', 'in', [11, 2])],
                  [('passenger_count', 'nin', list(range(10)))], [('vendor_id', '!=', 1)],
                  [('vendor_id', '==', 1.5)], [('fare_amount', '>', 1e9), ('vendor_id', '==', 7)],
                  [('vendor_id', '==', 7), ('fare_amount', '>', 1e9)]):
        assert ct.where_terms_factorization_check(terms) == bo.factorization_check(values, shards[0], terms), terms
    msg = calc.handle_work(_calc_msg(files[0], ['vendor_id'], [['fare_amount', 'sum', 'f']],
                                     [('passenger_count', 'in', [11, 12])]))
    assert msg['data'] == ''


def test_factor_cache_float_and_wide_columns(tmp_path):
    """Factor caches of groupby columns the lookup table cannot cover -- a float column (with
    -0.0 / +0.0 and NaN: khash identity) and an int64 column spanning more than 2^27 values --
    through a hash of the canonical key bits; labels and values against the oracle's factorize,
    and the factorization check over a float term column then answers the '' early-out."""
    rng = np.random.default_rng(17)
    n = 60_000
    fl = np.array([2.5, -0.0, 0.0, np.nan, 7.25, 1e300, -3.5])
    cols = OrderedDict(f=fl[rng.integers(0, len(fl), n)],
                       w=rng.integers(-(1 << 40), 1 << 40, 900)[rng.integers(0, 900, n)].astype(np.int64),
                       v=rng.integers(0, 9, n).astype(np.int32))
    root = os.path.join(str(tmp_path), 's.bcolzs')
    bcolz_io.write_ctable(root, cols)
    calc = CalcPath(str(tmp_path))
    calc.handle_work(_calc_msg('s.bcolzs', ['f', 'w'], [['v', 'sum', 'vs']], []))
    ct = calc.cache.open(root)
    ct.flush_caches()
    for col in ('f', 'w'):
        labels, uniq = bo.factorize(cols[col])
        np.testing.assert_array_equal(bcolz_io.read_carray(os.path.join(root, col + '.factor')), labels)
        np.testing.assert_array_equal(bcolz_io.read_carray(os.path.join(root, col + '.values')), uniq)
        assert ct.cache_valid(col)
    msg = calc.handle_work(_calc_msg('s.bcolzs', ['v'], [['v', 'count', 'n']], [('f', '==', 3.0)]))
    assert msg['data'] == ''
    msg = calc.handle_work(_calc_msg('s.bcolzs', ['v'], [['v', 'count', 'n']], [('f', '==', 7.25)]))
    assert msg['data'] != ''


def test_worker_mask_columns_stay_flat(tmp_path):
    """Repeated filtered + basket-expanded queries on one resident shard reuse the shard's
    scratch mask columns (no HBM growth per query, plan cache kept)."""
    n = 20_000
    cols = synth.taxi_shard(n, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    cols['basket'] = (np.arange(n) // 7).astype(np.int32)
    root = os.path.join(str(tmp_path), 's.bcolzs')
    bcolz_io.write_ctable(root, cols)
    calc = CalcPath(str(tmp_path))
    where = [('passenger_count', '>=', 2)]
    ref = bo.handle_work(cols, ['payment_type'], [['fare_amount', 'sum', 'f']], where, expand_filter_column='basket')
    scratch = []
    for _ in range(6):
        msg = calc.handle_work(_calc_msg('s.bcolzs', ['payment_type'], [['fare_amount', 'sum', 'f']], where,
                                         expand_filter_column='basket'))
        got = rpc.read_shard_results(rpc.tar_of_tars({'s.bcolzs': msg['data']}))[0]
        assert_tables_equal(got, ref, exact_float_sums=True)
        scratch.append(len(calc.cache.open(root)._table._scratch))
    assert scratch[-1] == scratch[0] <= 2, scratch


def test_c2_full_size_parity(oracle_c):
    """BASELINE configs[1] at full size (100 M rows) against the C restatement."""
    cfg = synth.CONFIGS['c2']
    cols = synth.taxi_shard(cfg['rows'], config_id=2, columns=synth.query_columns(cfg))
    ct = ctable(columns=cols)
    try:
        got = ct.groupby(cfg['groupby'], cfg['aggs'], bool_arr=ct.where_terms(cfg['where'])).columns
    finally:
        ct.close()
    ref = oracle_c.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where'])
    assert_tables_equal(got, ref)
    np.testing.assert_array_equal(got['fare_sum'], ref['fare_sum'])  # dyadic data: exact sums
    assert int(got['fare_cnt'].sum()) == int(np.count_nonzero(cols['passenger_count'] >= 2))
