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
from tests.helpers import assert_tables_equal, sort_by_keys

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


def _shards(n_shards, rows, mod):
    cols = ('pickup_location', 'vendor_id', 'fare_amount')
    out = [synth.taxi_shard(rows, config_id=5, n_shards=n_shards, shard=i, columns=cols) for i in range(n_shards)]
    for s in out:
        s['pickup_location'] = (s['pickup_location'] % mod).astype(s['pickup_location'].dtype)
    return out


AGGS_SC = [['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']]


def test_device_resident_single_rank_merge():
    """Per-shard results kept in HBM (groupby_table), concatenated device to device, summed:
    the reference client merge, in its group order."""
    shards = _shards(5, 120_000, 30_000)
    per = []
    for s in shards:
        t = ShardTable(s)
        per.append(t.groupby_table(KEYS, AGGS_SC))
        t.close()
    dtypes = OrderedDict((k, per[0].dtypes[k]) for k in per[0].names)
    merged = bdist.merge_partials_device(per, KEYS, AGGS_SC, dtypes, bdist.GpuBackend(), bdist.LocalExchange())
    for p in per:
        p.close()
    ref = bo.client_merge([bo.handle_work(s, KEYS, AGGS_SC, []) for s in shards], KEYS, AGGS_SC, aggregate=True)
    assert_tables_equal(merged, ref)


def test_groupby_table_and_select_rows_table_match_host_results():
    shards = _shards(1, 200_003, 7_000)
    t = ShardTable(shards[0])
    try:
        host, _ = t.groupby(KEYS, AGGS_SC, where_terms=[('fare_amount', '>', 9)])
        dev = t.groupby_table(KEYS, AGGS_SC, where_terms=[('fare_amount', '>', 9)])
        assert_tables_equal(dev.to_host(), host, exact_float_sums=True)
        dev.close()
        sel = t.select_rows_table(['vendor_id', 'fare_amount'], where_terms=[('vendor_id', '==', 2)])
        ref = t.select_rows(['vendor_id', 'fare_amount'], where_terms=[('vendor_id', '==', 2)])
        assert_tables_equal(sel.to_host(), ref, exact_float_sums=True)
        sel.close()
        empty = t.groupby_table(KEYS, AGGS_SC, where_terms=[('fare_amount', '<', 0)])
        assert empty.nrows == 0
        empty.close()
    finally:
        t.close()


class _ThreadExchange:
    """World of ``world`` ranks as threads of one process on one GPU: the collectives are
    host copies between threads (test harness for the device merge protocol; the product
    exchange is DeviceExchange over RCCL)."""

    def __init__(self, rank, world, shared):
        self.rank, self.world, self.sh = rank, world, shared

    def counts(self, send_counts):
        self.sh['counts'][self.rank] = np.asarray(send_counts, np.int64)
        self.sh['barrier'].wait()
        r = np.array([self.sh['counts'][src][self.rank] for src in range(self.world)], np.int64)
        self.sh['barrier'].wait()
        return r

    def column_device(self, parts, name, dtype, recv_counts):
        self.sh['cols'][self.rank] = [p.read(name) if p.nrows else np.zeros(0, dtype) for p in parts]
        self.sh['barrier'].wait()
        mine = np.concatenate([self.sh['cols'][src][self.rank] for src in range(self.world)]).astype(dtype)
        self.sh['barrier'].wait()
        # the receive buffer: a device column (torch is not imported in this process)
        buf = ShardTable(OrderedDict(x=np.concatenate([mine.view(np.uint8), np.zeros(1, np.uint8)])),
                         device=parts[0].dev)
        return buf.column_ptr('x'), buf

    def host_bytes(self, buf, nbytes):
        return buf.read('x')[:nbytes]


def test_device_merge_protocol_two_ranks_as_threads():
    import threading
    from bqueryd_amd.engine import Device
    shards = _shards(6, 50_000, 9_000)
    world = 2
    shared = {'barrier': threading.Barrier(world), 'counts': [None] * world, 'cols': [None] * world}
    results, errors = [None] * world, []

    def rank_main(rank):
        try:
            dev = Device(0)
            per = []
            for i, s in enumerate(shards):
                if i % world == rank:
                    t = ShardTable(s, device=dev)
                    per.append(t.groupby_table(KEYS, AGGS_SC))
                    t.close()
            dtypes = OrderedDict((k, per[0].dtypes[k]) for k in per[0].names)
            results[rank] = bdist.merge_partials_device(per, KEYS, AGGS_SC, dtypes, bdist.GpuBackend(dev),
                                                        _ThreadExchange(rank, world, shared))
            for p in per:
                p.close()
        except Exception as e:  # noqa: BLE001 -- re-raised in the main thread
            errors.append(e)
            shared['barrier'].abort()

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    assert results[1] is None
    ref = bo.client_merge([bo.handle_work(s, KEYS, AGGS_SC, []) for s in shards], KEYS, AGGS_SC, aggregate=True)
    assert_tables_equal(sort_by_keys(results[0], KEYS), sort_by_keys(ref, KEYS))


@pytest.mark.parametrize('aggs, where', [
    (AGGS_SC, []),
    (AGGS_SC, [('vendor_id', '==', 2)]),
    ([['fare_amount', 'mean', 'fm'], ['fare_amount', 'count', 'n']], []),  # not decomposable: per shard
])
def test_colocated_shards_single_rank(aggs, where):
    """A rank's shards aggregated in one pass over their union (sum / count) or per shard
    (anything else): the reference client merge of the per-shard results, in its group order
    (rpc.py:164-173)."""
    shards = _shards(5, 120_000, 30_000)
    tables = [ShardTable(s) for s in shards]
    colo = bdist.ColocatedShards(tables)
    per, reduced = colo.groupby_tables(KEYS, aggs, where_terms=where)
    assert reduced == bdist.decomposable(aggs)
    dtypes = OrderedDict((k, per[0].dtypes[k]) for k in per[0].names)
    for p in per:
        p.close()
    merged = colo.groupby_merged(KEYS, aggs, dtypes, bdist.GpuBackend(), bdist.LocalExchange(), where_terms=where)
    colo.close()
    for t in tables:
        t.close()
    ref = bo.client_merge([bo.handle_work(s, KEYS, aggs, where) for s in shards], KEYS, aggs, aggregate=True)
    assert_tables_equal(merged, ref)


def test_colocated_shards_two_ranks_as_threads():
    import threading
    from bqueryd_amd.engine import Device
    shards = _shards(6, 50_000, 9_000)
    world = 2
    shared = {'barrier': threading.Barrier(world), 'counts': [None] * world, 'cols': [None] * world}
    results, errors = [None] * world, []
    dtypes = OrderedDict([('pickup_location', np.dtype(np.int32)), ('vendor_id', np.dtype(np.int32)),
                          ('fare_sum', np.dtype(np.float64)), ('n', np.dtype(np.int64))])

    def rank_main(rank):
        try:
            dev = Device(0)
            tables = [ShardTable(s, device=dev) for i, s in enumerate(shards) if i % world == rank]
            colo = bdist.ColocatedShards(tables)
            results[rank] = colo.groupby_merged(KEYS, AGGS_SC, dtypes, bdist.GpuBackend(dev),
                                                _ThreadExchange(rank, world, shared))
            colo.close()
            for t in tables:
                t.close()
        except Exception as e:  # noqa: BLE001 -- re-raised in the main thread
            errors.append(e)
            shared['barrier'].abort()

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    assert results[1] is None
    ref = bo.client_merge([bo.handle_work(s, KEYS, AGGS_SC, []) for s in shards], KEYS, AGGS_SC, aggregate=True)
    assert_tables_equal(sort_by_keys(results[0], KEYS), sort_by_keys(ref, KEYS))
