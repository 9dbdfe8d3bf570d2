#!/usr/bin/env python3
"""Generates the golden fixtures in tests/golden/ from the CPU restatement of bquery.

The reference's own arithmetic (bquery/bcolz) is absent from this container and the
reference is Python-2 only, so the fixtures are produced by
oracle/bquery_oracle.py; the subset pandas can pin (single-key sum/mean/count, the reference's
own test oracle at tests/test_simple_rpc.py:139-190) is cross-checked against pandas by
tests/test_oracle.py.  Each case is one .npz (inputs ``in__<col>``, expected outputs
``out__<col>``, no pickles) plus an entry in cases.json with the query.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from bqueryd_amd import synth  # noqa: E402
from oracle import bquery_oracle as bo  # noqa: E402


def case_list():
    cases = []
    c2 = synth.CONFIGS['c2']
    cols = synth.taxi_shard(6000, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount',
                                                        'trip_distance'))
    cases.append(('c2_filtered', cols, dict(groupby=c2['groupby'], aggs=c2['aggs'], where=c2['where'])))
    cases.append(('pandas_sum', cols, dict(groupby=['payment_type'], aggs=[['fare_amount', 'sum', 'fare_amount']],
                                           where=[])))
    cases.append(('pandas_mean', cols, dict(groupby=['payment_type'],
                                            aggs=[['fare_amount', 'mean', 'fare_amount']], where=[])))
    cases.append(('pandas_count', cols, dict(groupby=['payment_type'],
                                             aggs=[['passenger_count', 'count', 'passenger_count']], where=[])))
    raw = synth.taxi_shard(5000, config_id=2, variant='raw', columns=('payment_type', 'passenger_count',
                                                                       'fare_amount', 'trip_distance'))
    cases.append(('raw_mean_std', raw, dict(groupby=['passenger_count'],
                                            aggs=[['fare_amount', 'mean', 'm'], ['trip_distance', 'std', 's'],
                                                  ['fare_amount', 'sum', 'fs'], 'trip_distance'],
                                            where=[('payment_type', 'in', [0, 1, 2])])))
    c3 = synth.CONFIGS['c3']
    cols3 = synth.taxi_shard(5000, config_id=3, columns=synth.query_columns(c3))
    cols3['pickup_location'] = (cols3['pickup_location'] % 700).astype(np.int32)
    cases.append(('c3_multikey', cols3, dict(groupby=c3['groupby'], aggs=c3['aggs'], where=[])))
    c4 = synth.CONFIGS['c4']
    cols4 = synth.taxi_shard(8000, config_id=4, columns=synth.query_columns(c4))
    cases.append(('c4_distinct_random', cols4, dict(groupby=c4['groupby'], aggs=c4['aggs'], where=[])))
    cols4s = synth.taxi_shard(8000, config_id=4, columns=synth.query_columns(c4),
                              sort_by=['pu_location_id', 'passenger_count'])
    cases.append(('c4_distinct_sorted', cols4s, dict(groupby=c4['groupby'], aggs=c4['aggs'], where=[])))
    f = synth.taxi_shard(4000, config_id=4, columns=('pu_location_id', 'passenger_count', 'fare_amount'))
    f['fare_amount'][0] = 1.0  # first row filtered: the skip slot takes label 0
    cases.append(('scd_first_row_filtered', f, dict(groupby=['pu_location_id'], aggs=c4['aggs'],
                                                     where=[('fare_amount', '>', 9.5)])))
    w = synth.taxi_shard(3000, config_id=2, columns=('payment_type', 'passenger_count', 'fare_amount'))
    terms_variants = [
        [('passenger_count', 'nin', [1, 3])],
        [('passenger_count', 'in', [2])],
        [('passenger_count', '!=', 1), ('fare_amount', '<=', 12.25)],
        [('passenger_count', '>', 1.5)],
        [('passenger_count', '==', 2.5)],
        [('fare_amount', 'in', [10.0, 12.5, 7.25])],
        [('payment_type', 'eq', 0), ('passenger_count', 'neq', 1)],
    ]
    for i, tv in enumerate(terms_variants):
        cases.append(('where_%d' % i, w, dict(groupby=['payment_type'],
                                               aggs=[['fare_amount', 'sum', 's'], ['fare_amount', 'count', 'c']],
                                               where=tv)))
    cases.append(('zero_keys', w, dict(groupby=[], aggs=[['fare_amount', 'sum', 's'], ['fare_amount', 'mean', 'm'],
                                                         ['passenger_count', 'count', 'c']], where=[])))
    cases.append(('no_rows_pass', w, dict(groupby=['payment_type'], aggs=[['fare_amount', 'sum', 's']],
                                          where=[('passenger_count', '>', 30)])))
    empty = OrderedDict((k, v[:0]) for k, v in w.items())
    cases.append(('empty_zero_keys', empty, dict(groupby=[], aggs=[['fare_amount', 'sum', 's'],
                                                                    ['passenger_count', 'count', 'c']], where=[])))
    rng = np.random.default_rng(12)
    n = 3000
    dt = OrderedDict(k8=rng.integers(-3, 3, n).astype(np.int8), k16=rng.integers(0, 9, n).astype(np.uint16),
                     i8=rng.integers(-128, 127, n).astype(np.int8),
                     u32=rng.integers(0, 2**32 - 1, n, dtype=np.uint32),
                     f32=(np.round(rng.normal(size=n) * 16) / 16).astype(np.float32),
                     i64=rng.integers(-2**40, 2**40, n, dtype=np.int64))
    cases.append(('dtypes_wrap', dt, dict(groupby=['k8', 'k16'], aggs=[['i8', 'sum', 'a'], ['u32', 'sum', 'b'],
                                                                        ['f32', 'sum', 'c'], ['i64', 'mean', 'd']],
                                          where=[('i64', '>', 0)])))
    cases.append(('raw_rows', w, dict(groupby=['payment_type'], aggs=[['fare_amount', 'sum', 'x']],
                                      where=[('passenger_count', '>=', 2)], aggregate=False)))
    cases.append(('expand_basket', w, dict(groupby=['payment_type'], aggs=[['fare_amount', 'sum', 's']],
                                           where=[('passenger_count', '>=', 5)], expand='payment_type')))
    return cases


def run_case(cols, q):
    if q.get('expand'):
        return bo.handle_work(cols, q['groupby'], q['aggs'], q['where'], aggregate=q.get('aggregate', True),
                              expand_filter_column=q['expand'])
    return bo.handle_work(cols, q['groupby'], q['aggs'], q['where'], aggregate=q.get('aggregate', True))


def multishard_case():
    """C1-shaped: 3 shards -> per-shard results -> client merge (rpc.py:164-175)."""
    aggs = [['fare_amount', 'sum', 'fare_amount'], ['fare_amount', 'mean', 'fm'], ['passenger_count', 'count', 'pc']]
    shards = [synth.taxi_shard(2000, config_id=1, n_shards=3, shard=i,
                               columns=('payment_type', 'passenger_count', 'fare_amount')) for i in range(3)]
    per = [bo.handle_work(s, ['payment_type'], aggs, []) for s in shards]
    merged = bo.client_merge(per, ['payment_type'], aggs, aggregate=True)
    concat = bo.client_merge(per, ['payment_type'], aggs, aggregate=False)
    return shards, per, merged, concat, aggs


def main():
    manifest = OrderedDict()
    for name, cols, q in case_list():
        out = run_case(cols, q)
        arrs = {}
        for k, v in cols.items():
            arrs['in__' + k] = v
        for k, v in out.items():
            arrs['out__' + k] = v
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **arrs)
        manifest[name] = dict(q, inputs=list(cols.keys()), outputs=list(out.keys()))
    shards, per, merged, concat, aggs = multishard_case()
    arrs = {}
    for i, s in enumerate(shards):
        for k, v in s.items():
            arrs['shard%d__%s' % (i, k)] = v
        for k, v in per[i].items():
            arrs['result%d__%s' % (i, k)] = v
    for k, v in merged.items():
        arrs['merged__' + k] = v
    for k, v in concat.items():
        arrs['concat__' + k] = v
    np.savez_compressed(os.path.join(HERE, 'c1_multishard.npz'), **arrs)
    manifest['c1_multishard'] = dict(groupby=['payment_type'], aggs=aggs, where=[], shards=3,
                                     inputs=list(shards[0].keys()), outputs=list(merged.keys()))
    with open(os.path.join(HERE, 'cases.json'), 'w') as f:
        json.dump(manifest, f, indent=1)
    print('wrote %d cases' % len(manifest))


if __name__ == '__main__':
    main()
