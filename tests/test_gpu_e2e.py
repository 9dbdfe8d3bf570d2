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
