"""aggregate=True merge of co-located shard results on one GPU (bqueryd_amd/dist.py): the
device reduce of the row-concatenated finalized tables must equal the reference client merge
(rpc.py:164-173), including its first-appearance group order."""
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import dist as bdist
from bqueryd_amd import synth
from bqueryd_amd.engine import ShardTable
from oracle import bquery_oracle as bo
from tests.helpers import assert_tables_equal

pytestmark = pytest.mark.gpu

KEYS = ['pickup_location', 'vendor_id']


@pytest.mark.parametrize('aggs', [
    [['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']],
    [['fare_amount', 'mean', 'fm'], ['passenger_count', 'count_distinct', 'pcd']],
])
def test_gpu_single_rank_merge(aggs):
    cols = ('pickup_location', 'vendor_id', 'fare_amount', 'passenger_count')
    shards = [synth.taxi_shard(150_000, config_id=5, n_shards=6, shard=i, columns=cols) for i in range(6)]
    for s in shards:
        s['pickup_location'] = (s['pickup_location'] % 20_000).astype(s['pickup_location'].dtype)
    per = []
    for s in shards:
        t = ShardTable(s)
        out, _ = t.groupby(KEYS, aggs)
        t.close()
        per.append(out)
    dtypes = OrderedDict((k, np.asarray(v).dtype) for k, v in per[0].items())
    merged = bdist.merge_partials(per, KEYS, aggs, dtypes, bdist.GpuBackend(), bdist.LocalExchange())
    ref = bo.client_merge([bo.handle_work(s, KEYS, aggs, []) for s in shards], KEYS, aggs, aggregate=True)
    assert_tables_equal(merged, ref)


def test_from_parts_matches_concatenation():
    rng = np.random.default_rng(4)
    parts = [OrderedDict(a=rng.integers(0, 9, n).astype(np.int32), b=rng.normal(size=n))
             for n in (0, 5, 300_000, 1, 70_000)]
    t = ShardTable.from_parts(parts)
    np.testing.assert_array_equal(t.read('a'), np.concatenate([p['a'] for p in parts]))
    np.testing.assert_array_equal(t.read('b'), np.concatenate([p['b'] for p in parts]))
    # a query result (page-locked block) pushed back by DMA
    out, _ = t.groupby(['a'], [['b', 'sum', 'b']])
    t2 = ShardTable.from_parts([out, out])
    np.testing.assert_array_equal(t2.read('b'), np.concatenate([out['b'], out['b']]))
