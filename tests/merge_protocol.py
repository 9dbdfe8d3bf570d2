"""Host-side specification of the co-located merge protocol -- TEST CODE.

The product merge is libbqgpu's ``bqg_merge`` (``bqueryd_amd/csrc/comm.hip``, called through
``bqueryd_amd.dist.merge_partials_device``).  This module restates the same five steps --
local reduce, hash partition, count exchange, row exchange, reduce, gather to rank 0 -- on host
tables over torch.distributed, against a small backend interface (``partition`` / ``reduce``),
so the CPU suite can run the protocol at world 2 under gloo with the oracle as the backend
(``tests/test_dist.py``).  The client merge it must reproduce is ``bqueryd/rpc.py:164-173``.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from bqueryd_amd.dist import sum_spec


def concat_tables(tables, names=None):
    tables = [t for t in tables if t is not None and not (isinstance(t, str) and t == '')]
    if not tables:
        return None
    names = names or list(tables[0].keys())
    return OrderedDict((n, np.concatenate([np.asarray(t[n]) for t in tables])) for n in names)


class LocalExchange:
    """World of one (no torch): the exchange is the identity."""
    world = 1
    rank = 0

    def counts(self, send_counts):
        return np.asarray(send_counts, np.int64)

    def column(self, parts, dtype, recv_counts):
        return np.ascontiguousarray(parts[0], dtype=np.dtype(dtype))


class Exchange:
    """Byte all-to-all over torch.distributed (nccl = RCCL on ROCm, or gloo)."""

    def __init__(self, dist, device=None, group=None):
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device

    def _tensor(self, arr):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy())
        return t.to(self.device) if self.device is not None else t

    def counts(self, send_counts):
        import torch
        s = torch.tensor(np.asarray(send_counts, np.int64))
        r = torch.empty(self.world, dtype=torch.int64)
        if self.device is not None:
            s, r = s.to(self.device), r.to(self.device)
        self.dist.all_to_all_single(r, s, group=self.group)
        return r.cpu().numpy()

    def column(self, parts, dtype, recv_counts):
        """parts[dst] -> this rank's rows from every source, concatenated in rank order."""
        import torch
        dtype = np.dtype(dtype)
        send = np.concatenate([np.ascontiguousarray(p, dtype=dtype) for p in parts]) if parts else np.zeros(0, dtype)
        in_split = [int(len(p)) * dtype.itemsize for p in parts]
        out_split = [int(c) * dtype.itemsize for c in recv_counts]
        out = torch.empty(sum(out_split), dtype=torch.uint8)
        if self.device is not None:
            out = out.to(self.device)
        self.dist.all_to_all_single(out, self._tensor(send), out_split, in_split, group=self.group)
        return out.cpu().numpy().view(dtype)


def merge_partials(local_tables, groupby_cols, agg_list, dtypes, backend, exchange):
    """Merge this rank's finalized shard tables with every other rank's; returns the merged
    table on rank 0 (None elsewhere).  ``dtypes``: name -> dtype of the finalized columns
    (needed by ranks that hold no shard)."""
    names = list(groupby_cols) + [x[2] for x in agg_list]
    local_tables = [t for t in local_tables
                    if t is not None and not (isinstance(t, str) and t == '') and len(t[names[0]])]
    if exchange.world == 1:
        # partition / exchange / gather are the identity: one reduce of everything
        if not local_tables:
            return OrderedDict((n, np.zeros(0, dtypes[n])) for n in names)
        return backend.reduce(local_tables, groupby_cols, agg_list)
    if local_tables:
        local = backend.reduce(local_tables, groupby_cols, agg_list)
        parts = backend.partition(local, groupby_cols, exchange.world)
    else:
        parts = [OrderedDict((n, np.zeros(0, dtypes[n])) for n in names) for _ in range(exchange.world)]
    recv_counts = exchange.counts([len(p[names[0]]) for p in parts])
    mine = OrderedDict((n, exchange.column([p[n] for p in parts], dtypes[n], recv_counts)) for n in names)
    if len(mine[names[0]]):
        mine = backend.reduce(mine, groupby_cols, agg_list)
    # gather to rank 0
    n_mine = len(mine[names[0]])
    to_root = [n_mine if dst == 0 else 0 for dst in range(exchange.world)]
    recv = exchange.counts(to_root)
    gathered = OrderedDict()
    for n in names:
        parts_n = [mine[n] if dst == 0 else np.zeros(0, dtypes[n]) for dst in range(exchange.world)]
        gathered[n] = exchange.column(parts_n, dtypes[n], recv)
    return gathered if exchange.rank == 0 else None
