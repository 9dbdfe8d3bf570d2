"""Cross-rank merge protocol under gloo, world_size 2, on CPU.

``tests/merge_protocol.py`` is the host-side specification of the protocol libbqgpu's
``bqg_merge`` runs on device buffers (partition, count exchange, row exchange, reduce, gather);
here its per-rank partition / reduce steps use the oracle as the backend and the exchange runs
over torch.distributed (gloo).  The merged result must equal the reference client merge
(rpc.py:164-173) of all shards."""
import os
import socket
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import dist as bdist
from bqueryd_amd import synth
from oracle import bquery_oracle as bo
from tests import merge_protocol as mp_
from tests.helpers import assert_tables_equal, sort_by_keys

AGGS = [['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n'], ['fare_amount', 'mean', 'fm']]
KEYS = ['pickup_location', 'vendor_id']
NSHARDS = 5


class OracleBackend:
    def reduce(self, table, groupby_cols, agg_list):
        if isinstance(table, list):
            table = mp_.concat_tables(table)
        return bo.groupby(table, groupby_cols, bdist.sum_spec(agg_list))

    def partition(self, table, groupby_cols, nparts):
        h = np.zeros(len(table[groupby_cols[0]]), np.uint64)
        for c in groupby_cols:
            h = (h * np.uint64(1000003)) ^ table[c].astype(np.int64).view(np.uint64)
        p = (h % np.uint64(nparts)).astype(np.int64)
        return [OrderedDict((n, v[p == i]) for n, v in table.items()) for i in range(nparts)]


def shard_results():
    out = []
    for i in range(NSHARDS):
        s = synth.taxi_shard(3000, config_id=5, n_shards=NSHARDS, shard=i,
                             columns=('pickup_location', 'vendor_id', 'fare_amount'))
        s['pickup_location'] = (s['pickup_location'] % 300).astype(np.int32)
        out.append(bo.handle_work(s, KEYS, AGGS, []))
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        results = shard_results()
        mine = [r for i, r in enumerate(results) if i % world == rank]
        dtypes = OrderedDict((k, v.dtype) for k, v in results[0].items())
        merged = mp_.merge_partials(mine, KEYS, AGGS, dtypes, OracleBackend(), mp_.Exchange(dist))
        q.put((rank, None if merged is None else {k: v.tolist() for k, v in merged.items()}))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('world', [2])
def test_merge_partials_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[1] is None
    results = shard_results()
    ref = bo.client_merge(results, KEYS, AGGS, aggregate=True)
    merged = OrderedDict((k, np.array(v, dtype=ref[k].dtype)) for k, v in got[0].items())
    assert_tables_equal(sort_by_keys(merged, KEYS), sort_by_keys(ref, KEYS))


def test_merge_partials_single_rank():
    """World of one: the merge is one reduce of every local table, in client order."""
    results = shard_results()
    dtypes = OrderedDict((k, v.dtype) for k, v in results[0].items())
    merged = mp_.merge_partials(results + [''], KEYS, AGGS, dtypes, OracleBackend(), mp_.LocalExchange())
    ref = bo.client_merge(results, KEYS, AGGS, aggregate=True)
    # same first-appearance order as the client's appended-then-regrouped table
    assert_tables_equal(merged, ref)
    empty = mp_.merge_partials([], KEYS, AGGS, dtypes, OracleBackend(), mp_.LocalExchange())
    assert all(len(v) == 0 and v.dtype == dtypes[k] for k, v in empty.items())


def test_decomposable_aggregations():
    from bqueryd_amd.dist import decomposable
    assert decomposable([['f', 'sum', 'a'], ['f', 'count', 'b']])
    assert decomposable([])
    assert not decomposable([['f', 'sum', 'a'], ['f', 'mean', 'b']])
    assert not decomposable([['f', 'count_distinct', 'a']])
    assert not decomposable([['f', 'sorted_count_distinct', 'a']])
    assert not decomposable([['f', 'std', 'a']])
    assert not decomposable(['f'])  # aggregate=True needs 3-element specs (rpc.py:171)
    assert not decomposable([['f', 'sum']])


def _shared_result_rank(rank, port, name, q):
    import os
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist
    from bqueryd_amd import dist as bdist
    dist.init_process_group('gloo', rank=rank, world_size=2)
    dts = {'k': np.dtype(np.int32), 's': np.dtype(np.float64)}
    try:
        if rank == 0:
            blk = bdist.SharedResult(name, 1000, ['k', 's'], dts, create=True)
        dist.barrier()
        if rank == 1:
            blk = bdist.SharedResult(name, 1000, ['k', 's'], dts, create=False)
            # the library's layout: column j at sum of align256(capacity x itemsize) before it
            assert blk.offsets == [0, (1000 * 4 + 255) & ~255]
            cols = blk.columns(5)
            cols['k'][:] = np.arange(5, dtype=np.int32) + 10
            cols['s'][:] = 0.5
            del cols
        dist.barrier()
        if rank == 0:
            got = blk.columns(5)
            q.put((got['k'].tolist(), got['s'].tolist()))
            del got
        dist.barrier()
        blk.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shared_result_block_between_ranks():
    """dist.SharedResult (the host block bqg_merge_shared_host writes): rank 0 creates it, rank 1
    attaches by name, the column layout is the library's, writes of one process are the other's
    reads, and the creator unlinks it (no GPU: plain shared memory between two gloo ranks)."""
    import multiprocessing as mp
    import os
    import socket
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    name = 'bqgpu-test-%d' % os.getpid()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_shared_result_rank, args=(r, port, name, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert [p.exitcode for p in ps] == [0, 0]
    assert q.get(timeout=10) == ([10, 11, 12, 13, 14], [0.5] * 5)
    assert not os.path.exists('/dev/shm/' + name)
