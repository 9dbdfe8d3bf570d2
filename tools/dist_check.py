#!/usr/bin/env python3
"""GPU merge check, launched under torch.distributed.run (one process per GPU).

torch.distributed (gloo, CPU) only hands rank 0's RCCL unique id to the other ranks and
provides the final barrier; the merge itself is libbqgpu's bqg_merge over RCCL on device
buffers (bqueryd_amd.dist.RcclComm / merge_partials_device).  Each rank runs per-shard
groupbys into HBM tables and, separately, one co-located pass over its shards
(ColocatedShards); rank 0 checks both merges against the oracle's client merge
(rpc.py:164-173).  Exit code 0 = parity.
"""
import os
import sys

import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from bqueryd_amd import dist as bdist  # noqa: E402
from bqueryd_amd import synth  # noqa: E402
from bqueryd_amd.engine import Device, ShardTable  # noqa: E402


def _check(merged, ref):
    order_g = np.lexsort((merged['vendor_id'], merged['pickup_location']))
    order_r = np.lexsort((ref['vendor_id'], ref['pickup_location']))
    ok = len(merged['n']) == len(ref['n'])
    for c in ref:
        if not ok:
            break
        g, r = merged[c][order_g], ref[c][order_r]
        same = np.array_equal(g, r) if r.dtype.kind != 'f' else np.allclose(g, r, rtol=1e-12, atol=0)
        ok &= bool(same) and g.dtype == r.dtype
    return ok


def one_gpu_rccl_env(rank):
    """Every rank on GPU 0 over real RCCL (BQGPU_DIST_ONE_GPU=1): RCCL refuses two ranks on one
    device of one host ("Duplicate GPU detected"), so each rank claims a host of its own
    (NCCL_HOSTID) and the ranks talk over RCCL's socket transport on the loopback interface --
    the merge's RCCL calls (grouped send / recv, all-gather) at world > 1 on a one-GPU box,
    slowly.  Set before librccl initialises (the unique id below)."""
    os.environ['NCCL_HOSTID'] = 'bqgpu-rank%d' % rank
    os.environ.setdefault('NCCL_SOCKET_IFNAME', 'lo')
    os.environ.setdefault('NCCL_IB_DISABLE', '1')
    return 0


def main():
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    if os.environ.get('BQGPU_DIST_ONE_GPU') == '1':
        local = one_gpu_rccl_env(rank)
    uid = [bdist.new_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    dev = Device(local)
    comm = bdist.RcclComm(dev, rank, world, uid[0])
    keys = ['pickup_location', 'vendor_id']
    aggs = [['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']]
    nshards = 4 * world
    shards = [synth.taxi_shard(200_000, config_id=5, n_shards=nshards, shard=i,
                               columns=('pickup_location', 'vendor_id', 'fare_amount')) for i in range(nshards)]
    tables = [ShardTable(shards[i], device=dev) for i in range(rank, nshards, world)]
    per = [t.groupby_table(keys, aggs) for t in tables]
    dtypes = {'pickup_location': np.dtype(np.int32), 'vendor_id': np.dtype(np.int32),
              'fare_sum': np.dtype(np.float64), 'n': np.dtype(np.int64)}
    merged = bdist.merge_partials_device(per, keys, aggs, dtypes, comm)
    colo = bdist.ColocatedShards(tables)
    merged_colo = colo.groupby_merged(keys, aggs, dtypes, comm)
    # the same merge into node-shared host memory (bqg_merge_shared_host): rank 0 creates the
    # block, every rank writes its partition into it; started too small, so the first call
    # reports the rows it needs on every rank and the block grows
    names = keys + [a[2] for a in aggs]
    sh_name = ['bqgpu-dist-%d' % os.getpid() if rank == 0 else None]
    dist.broadcast_object_list(sh_name, src=0)
    cap = 1000
    while True:
        if rank == 0:
            shared = bdist.SharedResult(sh_name[0] + '-%d' % cap, cap, names, dtypes, create=True)
        dist.barrier()  # the other ranks attach after rank 0 created it
        if rank != 0:
            shared = bdist.SharedResult(sh_name[0] + '-%d' % cap, cap, names, dtypes, create=False)
        try:
            rows = bdist.merge_partials_shared(per, keys, aggs, dtypes, comm, shared)
            break
        except ValueError as e:
            dist.barrier()  # every rank is done with the block before rank 0 unlinks it
            shared.close()
            cap = e.args[1]
    ok = True
    if rank == 0:
        from oracle import bquery_oracle as bo
        ref = bo.client_merge([bo.handle_work(s, keys, aggs, []) for s in shards], keys, aggs, aggregate=True)
        merged_shared = {n: np.array(v) for n, v in shared.columns(rows).items()}
        ok = _check(merged, ref) and _check(merged_colo, ref) and _check(merged_shared, ref) and cap > 1000
        print('dist_check world=%d groups=%d shared_rows=%d ok=%s' % (world, len(ref['n']), rows, ok), flush=True)
    else:
        ok = merged is None and merged_colo is None
    dist.barrier()
    shared.close()
    for p in per:
        p.close()
    colo.close()
    for t in tables:
        t.close()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
