#!/usr/bin/env python3
"""GPU merge check, launched under torch.distributed.run (one process per GPU).

Imports torch first (so libbqgpu binds the HIP runtime torch loaded), initialises the nccl
(RCCL) process group, runs per-shard groupbys on the GPU, merges them with
bqueryd_amd.dist.merge_partials over RCCL, and on rank 0 checks the result against the
oracle's client merge (rpc.py:164-173).  Exit code 0 = parity.
"""
import os
import sys

import torch  # noqa: F401  (must precede libbqgpu: one HIP runtime per process)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from bqueryd_amd import dist as bdist  # noqa: E402
from bqueryd_amd import synth  # noqa: E402
from bqueryd_amd.engine import Device, ShardTable  # noqa: E402


def main():
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dist.init_process_group('nccl')
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = Device(local)
    keys = ['pickup_location', 'vendor_id']
    aggs = [['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']]
    nshards = 4 * world
    shards = [synth.taxi_shard(200_000, config_id=5, n_shards=nshards, shard=i,
                               columns=('pickup_location', 'vendor_id', 'fare_amount')) for i in range(nshards)]
    mine = []
    for i in range(rank, nshards, world):
        t = ShardTable(shards[i], device=dev)
        out, _ = t.groupby(keys, aggs)
        t.close()
        mine.append(out)
    dtypes = {'pickup_location': np.dtype(np.int32), 'vendor_id': np.dtype(np.int32),
              'fare_sum': np.dtype(np.float64), 'n': np.dtype(np.int64)}
    merged = bdist.merge_partials(mine, keys, aggs, dtypes, bdist.GpuBackend(dev),
                                  bdist.Exchange(dist, device=torch.device('cuda', local)))
    ok = True
    if rank == 0:
        from oracle import bquery_oracle as bo
        per = [bo.handle_work(s, keys, aggs, []) for s in shards]
        ref = bo.client_merge(per, keys, aggs, aggregate=True)
        order_g = np.lexsort((merged['vendor_id'], merged['pickup_location']))
        order_r = np.lexsort((ref['vendor_id'], ref['pickup_location']))
        for c in ref:
            g, r = merged[c][order_g], ref[c][order_r]
            same = np.array_equal(g, r) if r.dtype.kind != 'f' else np.allclose(g, r, rtol=1e-12, atol=0)
            ok &= bool(same) and g.dtype == r.dtype
        print('dist_check world=%d groups=%d ok=%s' % (world, len(ref['n']), ok), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
