"""aggregate=True merge of co-located shard results (bqueryd_amd/dist.py, libbqgpu bqg_merge):
the reduce of the row-concatenated finalized tables must equal the reference client merge
(rpc.py:164-173) -- in its first-appearance group order on one rank, after sorting by the keys
across ranks (the client's own order is file-system glob order, rpc.py:151)."""
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
    """The product merge (bqg_merge at world 1) of six shards' device-resident results, every
    aggregation's finalized values summed as the client does -- in its first-appearance order."""
    from bqueryd_amd.engine import get_device
    cols = ('pickup_location', 'vendor_id', 'fare_amount', 'passenger_count')
    shards = [synth.taxi_shard(150_000, config_id=5, n_shards=6, shard=i, columns=cols) for i in range(6)]
    for s in shards:
        s['pickup_location'] = (s['pickup_location'] % 20_000).astype(s['pickup_location'].dtype)
    per = _device_results(shards, aggs=aggs)
    comm = bdist.RcclComm(get_device())
    try:
        merged = bdist.merge_partials_device(per, KEYS, aggs, _dtypes(aggs), comm)
    finally:
        comm.close()
        for p in per:
            p.close()
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


def _device_results(shards, dev=None, aggs=AGGS_SC):
    per = []
    for s in shards:
        t = ShardTable(s, device=dev)
        per.append(t.groupby_table(KEYS, aggs))
        t.close()
    return per


def _dtypes(aggs=AGGS_SC):
    d = OrderedDict([('pickup_location', np.dtype(np.int32)), ('vendor_id', np.dtype(np.int32))])
    for a in aggs:
        d[a[2]] = np.dtype(np.float64) if a[1] in ('sum', 'mean', 'std') else np.dtype(np.int64)
    return d


def test_rccl_merge_world_one():
    """bqg_merge over a one-rank RCCL communicator (bqg_comm_init): partition, RCCL
    all-gather of the row counts, RCCL send/recv of the rows, reduce and gather all run; with
    one rank the result keeps the client's first-appearance group order (rpc.py:164-173)."""
    from bqueryd_amd.engine import get_device
    shards = _shards(5, 120_000, 30_000)
    per = _device_results(shards)
    comm = bdist.RcclComm(get_device())
    try:
        merged = bdist.merge_partials_device(per, KEYS, AGGS_SC, _dtypes(), comm)
        again = bdist.merge_partials_device(per, KEYS, AGGS_SC, _dtypes(), comm)  # buffers reused
        empty = bdist.merge_partials_device([], KEYS, AGGS_SC, _dtypes(), comm)
    finally:
        comm.close()
        for p in per:
            p.close()
    ref = bo.client_merge([bo.handle_work(s, KEYS, AGGS_SC, []) for s in shards], KEYS, AGGS_SC, aggregate=True)
    assert_tables_equal(merged, ref)
    assert_tables_equal(again, ref)
    assert all(len(v) == 0 for v in empty.values())


def test_shared_host_merge_world_one():
    """bqg_merge_shared_host at world 1 (dist.SharedResult: a POSIX shared-memory block, as the
    node's rank processes map it): the same rows as bqg_merge_host in the client's order; a
    block too small reports the rows it needs and leaves the communicator usable; the block
    is registered once and reused across merges; an empty merge writes no row."""
    import os
    from bqueryd_amd.engine import get_device
    shards = _shards(4, 100_000, 25_000)
    per = _device_results(shards)
    dts = _dtypes()
    names = list(dts)
    comm = bdist.RcclComm(get_device())
    small = big = None
    try:
        ref = bdist.merge_partials_device(per, KEYS, AGGS_SC, dts, comm)
        small = bdist.SharedResult('bqgpu-test-small-%d' % os.getpid(), 100, names, dts, create=True)
        with pytest.raises(ValueError) as ei:
            bdist.merge_partials_shared(per, KEYS, AGGS_SC, dts, comm, small)
        need = ei.value.args[1]
        assert need == len(ref['n'])
        big = bdist.SharedResult('bqgpu-test-big-%d' % os.getpid(), need + 7, names, dts, create=True)
        for _ in range(2):  # the second merge reuses the registration
            rows = bdist.merge_partials_shared(per, KEYS, AGGS_SC, dts, comm, big)
            got = {n: np.array(v) for n, v in big.columns(rows).items()}
            for n in names:
                np.testing.assert_array_equal(got[n], ref[n], err_msg=n)
        assert bdist.merge_partials_shared([], KEYS, AGGS_SC, dts, comm, big) == 0
    finally:
        comm.close()
        for p in per:
            p.close()
        for b in (small, big):
            if b is not None:
                b.close()


def test_comm_progress_counts_merges():
    """bqg_comm_progress (what bench.py's watchdog reports for a rank whose collective does not
    return): idle between merges, one more merge begun and ended per call, failures included;
    readable from another thread while a merge runs."""
    import threading
    from bqueryd_amd.engine import get_device
    dev = get_device()
    shards = _shards(3, 80_000, 20_000)
    per = _device_results(shards)
    comm = bdist.RcclComm(dev)
    seen = []
    try:
        p0 = bdist.merge_progress(dev)
        assert p0['phase'] == 'idle' and p0['merges_started'] == p0['merges_done']
        stop = threading.Event()

        def poll():
            while not stop.is_set():
                seen.append(bdist.merge_progress(dev)['phase'])
        th = threading.Thread(target=poll)
        th.start()
        try:
            for _ in range(3):
                bdist.merge_partials_device(per, KEYS, AGGS_SC, _dtypes(), comm)
        finally:
            stop.set()
            th.join()
        p1 = bdist.merge_progress(dev)
        assert p1['phase'] == 'idle'
        assert p1['merges_started'] == p0['merges_started'] + 3 and p1['merges_done'] == p0['merges_done'] + 3
        with pytest.raises(Exception):  # a bad schema fails inside the merge: counted as ended
            bdist.merge_partials_device(per, KEYS, AGGS_SC + [['fare_amount', 'sum', 'x']],
                                        dict(_dtypes(), x=np.dtype(np.float64)), comm)
        p2 = bdist.merge_progress(dev)
        assert p2['phase'] == 'idle' and p2['merges_done'] - p2['merges_started'] == p1['merges_done'] - p1['merges_started']
    finally:
        comm.close()
        for p in per:
            p.close()
    assert set(seen) <= set(bdist.MERGE_PHASES) | {'idle'}, set(seen)


def test_rccl_comm_init_all_one_gpu():
    """bqg_comm_init_all (a process owning the node's GPUs) with the one GPU of this box."""
    from bqueryd_amd.engine import Device
    dev = Device(0)
    shards = _shards(4, 60_000, 8_000)
    per = _device_results(shards, dev)
    group = bdist.CommGroup([dev], transport='rccl')
    try:
        merged = bdist.merge_group_device([per], KEYS, AGGS_SC, _dtypes(), group)
    finally:
        group.close()
        for p in per:
            p.close()
    ref = bo.client_merge([bo.handle_work(s, KEYS, AGGS_SC, []) for s in shards], KEYS, AGGS_SC, aggregate=True)
    assert_tables_equal(merged, ref)


@pytest.mark.parametrize('world, nshards', [(2, 6), (3, 7), (4, 3)])
def test_merge_in_process_ranks(world, nshards):
    """World 2-4 on one GPU: every rank a libbqgpu context, the exchange by device copies
    (bqg_comm_init_local) -- the same partition / pack / reduce / gather code as over RCCL,
    including a rank that holds no shard (world 4, 3 shards)."""
    from bqueryd_amd.engine import Device
    devs = [Device(0) for _ in range(world)]
    shards = _shards(nshards, 50_000, 9_000)
    per = [_device_results([s for i, s in enumerate(shards) if i % world == r], devs[r]) for r in range(world)]
    group = bdist.CommGroup(devs, transport='local')
    try:
        merged = bdist.merge_group_device(per, KEYS, AGGS_SC, _dtypes(), group)
    finally:
        group.close()
        for tabs in per:
            for p in tabs:
                p.close()
    ref = bo.client_merge([bo.handle_work(s, KEYS, AGGS_SC, []) for s in shards], KEYS, AGGS_SC, aggregate=True)
    assert_tables_equal(sort_by_keys(merged, KEYS), sort_by_keys(ref, KEYS))


def test_colocated_in_process_ranks():
    """Co-located one-pass groupby per rank (reduced=True) merged across 3 in-process ranks."""
    from bqueryd_amd.engine import Device
    world = 3
    devs = [Device(0) for _ in range(world)]
    shards = _shards(7, 40_000, 6_000)
    tables = [[ShardTable(s, device=devs[r]) for i, s in enumerate(shards) if i % world == r] for r in range(world)]
    colos = [bdist.ColocatedShards(t) for t in tables]
    per = []
    for c in colos:
        p, reduced = c.groupby_tables(KEYS, AGGS_SC)
        assert reduced
        per.append(p)
    group = bdist.CommGroup(devs, transport='local')
    try:
        merged = bdist.merge_group_device(per, KEYS, AGGS_SC, _dtypes(), group, reduced=True)
    finally:
        group.close()
        for tabs in per:
            for p in tabs:
                p.close()
        for c in colos:
            c.close()
        for ts in tables:
            for t in ts:
                t.close()
    ref = bo.client_merge([bo.handle_work(s, KEYS, AGGS_SC, []) for s in shards], KEYS, AGGS_SC, aggregate=True)
    assert_tables_equal(sort_by_keys(merged, KEYS), sort_by_keys(ref, KEYS))


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
    comm = bdist.RcclComm(tables[0].dev)
    merged = colo.groupby_merged(KEYS, aggs, dtypes, comm, where_terms=where)
    comm.close()
    colo.close()
    for t in tables:
        t.close()
    ref = bo.client_merge([bo.handle_work(s, KEYS, aggs, where) for s in shards], KEYS, aggs, aggregate=True)
    assert_tables_equal(merged, ref)


def _rank_tables(world, seed, n_tables=3, rows=40_000):
    """Finalized per-shard tables of mixed dtypes (each table's keys unique, as a shard result
    is): an int16 and a float64 key (-0.0 / +0.0 and NaN among them), an int32 sum that wraps,
    a float32 sum, a raw (non-dyadic) float64 sum and an int64 count."""
    rng = np.random.default_rng(seed)
    fkeys = np.array([0.0, -0.0, np.nan, 1.5, -2.25, 1e300, 3.0])
    out = []
    for r in range(world):
        tabs = []
        for _ in range(n_tables):
            a = rng.integers(-300, 300, rows).astype(np.int16)
            f = fkeys[rng.integers(0, len(fkeys), rows)]
            t = OrderedDict(a=a, f=f)
            # unique keys per table: keep each (a, canonical f) once
            code = (a.astype(np.int64) + 300) * 8 + np.searchsorted(np.array([-2.25, 0.0, 1.5, 3.0, 1e300]), np.nan_to_num(f, nan=9e300))
            _, first = np.unique(code, return_index=True)
            first.sort()
            t = OrderedDict((k, v[first]) for k, v in t.items())
            m = len(first)
            t['s32'] = rng.integers(-2**31, 2**31 - 1, m).astype(np.int32)
            t['f32'] = (rng.normal(size=m) * 100).astype(np.float32)
            t['f64'] = np.round(rng.lognormal(2.3, 0.6, m), 2)
            t['n'] = rng.integers(0, 1000, m).astype(np.int64)
            tabs.append(t)
        out.append(tabs)
    return out


@pytest.mark.parametrize('world', [1, 2, 3, 5])
def test_merge_reduce_dtypes_and_determinism(world):
    """The receive-side reduce (MergeReduce: one hash table, partials added in source-rank
    order) over mixed key / value dtypes: keys compare by value (-0.0 == +0.0, NaN == NaN),
    int32 sums wrap, float32 sums round once; the same merge twice gives bit-identical rows in
    the same order (deterministic sums and order), and the device-table variant (gather to
    rank 0, bqg_merge_group) gives the same rows."""
    from bqueryd_amd.engine import Device
    keys = ['a', 'f']
    aggs = [['s32', 'sum', 's32'], ['f32', 'sum', 'f32'], ['f64', 'sum', 'f64'], ['n', 'sum', 'n']]
    host = _rank_tables(world, 50 + world)
    dtypes = OrderedDict((k, v.dtype) for k, v in host[0][0].items())
    devs = [Device(0) for _ in range(world)]
    per = [[ShardTable(t, device=devs[r]) for t in host[r]] for r in range(world)]
    group = bdist.CommGroup(devs, transport='local')
    try:
        m1 = bdist.merge_group_device(per, keys, aggs, dtypes, group)
        m2 = bdist.merge_group_device(per, keys, aggs, dtypes, group)
        t3 = bdist.merge_group_device_table(per, keys, aggs, dtypes, group)
        m3 = t3.to_host()
        t3.close()
    finally:
        group.close()
        for tabs in per:
            for p in tabs:
                p.close()
    for c in m1:
        np.testing.assert_array_equal(m1[c].view(np.uint8), m2[c].view(np.uint8), err_msg=c)
    flat = [t for tabs in host for t in tabs]
    ref = bo.client_merge(flat, keys, aggs, aggregate=True)
    for got in (m1, m3):
        g, r = sort_by_keys(got, keys), sort_by_keys(ref, keys)
        assert list(g) == list(r)
        for c in r:
            if c in ('f32', 'f64'):
                tol = 1e-6 if c == 'f32' else 1e-12
                np.testing.assert_allclose(g[c], r[c], rtol=tol, atol=tol * float(np.abs(r[c]).max()), err_msg=c)
            else:
                np.testing.assert_array_equal(g[c], r[c], err_msg=c)
