"""Cross-GPU merge of per-shard results for ``aggregate=True``.

The reference merges on the client: every shard's finalized table is appended and re-grouped
with ``sum`` of every column ("we can only sum now", ``bqueryd/rpc.py:164-173``).  For shards
co-located on one node this module does the same merge across GPU ranks:

  1. local:    each rank sums its own shards' tables by key (GPU groupby-sum);
  2. partition: rows are assigned to rank ``hash(key values) mod world`` (GPU kernel
               ``bqg_hash_partition``: a pure function of the key values, identical on every
               rank, so all partials of one key meet on one rank);
  3. exchange: one ``all_to_all_single`` per column, raw bytes with per-rank split sizes
               (``torch.distributed``: RCCL over xGMI on GPUs, gloo on CPU);
  4. reduce:   each rank sums the rows it received by key (GPU groupby-sum);
  5. gather:   the reduced partitions travel to rank 0 with the same byte all-to-all.

The protocol is written against a small backend interface (``partition`` / ``reduce``) so the
CPU test suite can run it under gloo with the oracle as the backend; the product backend is
``GpuBackend`` (libbqgpu), which has no CPU fallback.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np


def sum_spec(agg_list):
    """The client's merge aggregation list: ``[[x[2], 'sum', x[2]] for x in agg_list]``."""
    return [[x[2], 'sum', x[2]] for x in agg_list]


def concat_tables(tables, names=None):
    tables = [t for t in tables if t is not None and not (isinstance(t, str) and t == '')]
    if not tables:
        return None
    names = names or list(tables[0].keys())
    return OrderedDict((n, np.concatenate([np.asarray(t[n]) for t in tables])) for n in names)


class GpuBackend:
    """partition / reduce on the GPU through libbqgpu."""

    def __init__(self, device=None):
        from .engine import get_device
        self.device = device or get_device()

    def reduce(self, table, groupby_cols, agg_list, on_device=False):
        """``table``: one table or a list of tables -- host mappings or device ShardTables --
        row-concatenated on the device and summed by key.  ``on_device``: the result stays in
        HBM (a ShardTable) instead of coming back as numpy arrays."""
        from .engine import ShardTable
        parts = table if isinstance(table, (list, tuple)) else [table]
        names = list(groupby_cols) + [x[2] for x in agg_list]
        t = ShardTable.from_parts(parts, names, device=self.device)
        try:
            if on_device:
                return t.groupby_table(groupby_cols, sum_spec(agg_list))
            out, _ = t.groupby(groupby_cols, sum_spec(agg_list))
            return out
        finally:
            t.close()

    def partition_device(self, table, groupby_cols, nparts):
        """Device ShardTable -> ``nparts`` device ShardTables, rows split by the hash of their
        key values (the same function on every rank)."""
        import ctypes
        from . import _lib as L
        names = list(table.names)
        col = table.add_column('__part__', np.uint32)
        keys = np.array([table.slot(c) for c in groupby_cols], np.int32)
        counts = np.zeros(nparts, np.int64)
        self.device.check(L.lib().bqg_hash_partition(self.device.handle, table.handle, len(keys),
                                                     keys.ctypes.data, nparts, col, counts.ctypes.data))
        return [table.select_rows_table(names, where_terms=[('__part__', '==', p)]) for p in range(nparts)]

    def empty_table(self, names, dtypes):
        from .engine import ShardTable
        return ShardTable(OrderedDict((n, np.zeros(0, dtypes[n])) for n in names), device=self.device)

    def table_from_buffers(self, names, dtypes, bufs, nrows):
        """A device ShardTable whose columns are copied (device to device) from ``bufs``
        (name -> device address)."""
        from .engine import ShardTable
        t = ShardTable(OrderedDict(), device=self.device, nrows=nrows)
        for n in names:
            t.add_column(n, dtypes[n])
            t.names.append(n)
            if nrows:
                t.push_device(n, bufs[n], nrows)
        t.sync()
        return t

    def partition(self, table, groupby_cols, nparts):
        import ctypes
        from . import _lib as L
        from .engine import ShardTable
        t = ShardTable(table, device=self.device)
        try:
            col = t.add_column('__part__', np.uint32)
            keys = np.array([t.slot(c) for c in groupby_cols], np.int32)
            counts = np.zeros(nparts, np.int64)
            self.device.check(L.lib().bqg_hash_partition(self.device.handle, t.handle, len(keys),
                                                         keys.ctypes.data, nparts, col,
                                                         counts.ctypes.data))
            names = list(table.keys())
            parts = []
            for p in range(nparts):
                if counts[p] == 0:
                    parts.append(OrderedDict((n, np.asarray(table[n])[:0]) for n in names))
                else:
                    parts.append(t.select_rows(names, where_terms=[('__part__', '==', p)]))
            return parts
        finally:
            t.close()


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


class DeviceExchange(Exchange):
    """Byte all-to-all of device-resident columns: RCCL over xGMI (``torch.distributed`` with
    the nccl backend), no host copies.  Columns of ShardTables are packed into one torch
    device buffer per column with device-to-device copies."""

    def column_device(self, parts, name, dtype, recv_counts):
        """parts[dst]: ShardTables on this GPU -> (device address, torch buffer) of this rank's
        rows of column ``name`` from every source, concatenated in rank order."""
        import torch
        dtype = np.dtype(dtype)
        in_split = [int(p.nrows) * dtype.itemsize for p in parts]
        out_split = [int(c) * dtype.itemsize for c in recv_counts]
        stream = torch.cuda.current_stream(self.device)
        send = torch.empty(max(1, sum(in_split)), dtype=torch.uint8, device=self.device)
        out = torch.empty(max(1, sum(out_split)), dtype=torch.uint8, device=self.device)
        stream.synchronize()  # the fresh buffers are idle before another stream writes them
        off = 0
        for p, nb in zip(parts, in_split):
            if nb:
                p.read_device(name, send.data_ptr() + off)  # synchronous on libbqgpu's stream
            off += nb
        self.dist.all_to_all_single(out[:sum(out_split)], send[:sum(in_split)], out_split, in_split,
                                    group=self.group)
        stream.synchronize()  # received bytes are complete before libbqgpu reads them
        return out.data_ptr(), out

    def host_bytes(self, buf, nbytes):
        """The first ``nbytes`` of a buffer returned by ``column_device``, in host memory."""
        return buf[:nbytes].cpu().numpy()


def merge_partials_device(local_tables, groupby_cols, agg_list, dtypes, backend, exchange, reduced=False):
    """``merge_partials`` with every step in HBM: ``local_tables`` are this rank's finalized
    shard tables as device ShardTables (``ShardTable.groupby_table``), the reduce, partition,
    all-to-all and gather run on device buffers, and only the merged table comes back to host
    memory (rank 0; None elsewhere).  ``reduced``: ``local_tables`` is ONE table whose keys are
    already unique (a co-located groupby, ``ColocatedShards``), so the local re-group is skipped."""
    names = list(groupby_cols) + [x[2] for x in agg_list]
    local_tables = [t for t in local_tables if t is not None and t.nrows]
    reduced = reduced and len(local_tables) == 1
    if exchange.world == 1:
        if not local_tables:
            return OrderedDict((n, np.zeros(0, dtypes[n])) for n in names)
        if reduced:
            return OrderedDict((n, local_tables[0].read(n)) for n in names)
        return backend.reduce(local_tables, groupby_cols, agg_list)
    if local_tables:
        local = local_tables[0] if reduced else backend.reduce(local_tables, groupby_cols, agg_list, on_device=True)
        try:
            parts = backend.partition_device(local, groupby_cols, exchange.world)
        finally:
            if not reduced:
                local.close()
    else:
        parts = [backend.empty_table(names, dtypes) for _ in range(exchange.world)]
    recv_counts = exchange.counts([p.nrows for p in parts])
    n_recv = int(np.sum(recv_counts))
    keep = []
    bufs = OrderedDict()
    for n in names:
        ptr, buf = exchange.column_device(parts, n, dtypes[n], recv_counts)
        bufs[n] = ptr
        keep.append(buf)
    for p in parts:
        p.close()
    mine = backend.table_from_buffers(names, dtypes, bufs, n_recv)
    del keep[:]
    if n_recv:
        reduced = backend.reduce([mine], groupby_cols, agg_list, on_device=True)
        mine.close()
        mine = reduced
    # gather the disjoint reduced partitions to rank 0
    empty = backend.empty_table(names, dtypes)
    to_root = [mine.nrows if dst == 0 else 0 for dst in range(exchange.world)]
    recv = exchange.counts(to_root)
    gathered = OrderedDict()
    for n in names:
        ptr, buf = exchange.column_device([mine if dst == 0 else empty for dst in range(exchange.world)], n,
                                          dtypes[n], recv)
        nbytes = int(np.sum(recv)) * np.dtype(dtypes[n]).itemsize
        gathered[n] = exchange.host_bytes(buf, nbytes).view(np.dtype(dtypes[n])) if exchange.rank == 0 else None
    mine.close()
    empty.close()
    return gathered if exchange.rank == 0 else None


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


# aggregations whose client-side merge (a sum of the per-shard finalized values, rpc.py:170-172)
# equals the aggregation over the union of the shards' rows
DECOMPOSABLE = frozenset(['sum', 'count'])


def decomposable(agg_list):
    """True when every aggregation of ``agg_list`` (3-element specs, as ``aggregate=True``
    requires, rpc.py:171) merges by summing: then Σ over shards of the per-shard result equals
    the result over the union of the rows -- exactly for counts and integer sums (integer sums
    wrap to the input width either way), within float rounding for float sums -- and the group
    order agrees too: first appearance in the concatenation of per-shard tables, each in its
    shard's first-appearance order, is first appearance in the concatenated rows."""
    return all(isinstance(x, (list, tuple)) and len(x) == 3 and x[1] in DECOMPOSABLE for x in agg_list)


class ColocatedShards:
    """The shards one rank holds for an ``aggregate=True`` query (controller.py:494-506 fans
    out one calc per shard).  For decomposable aggregations the rank's shards
    are aggregated in ONE pass over their rows -- the shards' columns concatenated once in HBM
    (device-to-device copies, kept while the shard set is resident) -- instead of one groupby
    per shard followed by a local re-group; other aggregations (mean, std, count_distinct,
    sorted_count_distinct: their client merge sums per-shard finalized values, which is not
    the value over the union) keep the per-shard path."""

    def __init__(self, tables):
        self.tables = [t for t in tables if t is not None]
        self._union = None
        self._union_cols = ()

    def union(self, cols):
        from .engine import ShardTable
        cols = tuple(cols)
        if self._union is None or not set(cols) <= set(self._union_cols):
            if self._union is not None:
                self._union.close()
            self._union = ShardTable.from_parts(self.tables, list(cols), device=self.tables[0].dev)
            self._union_cols = cols
        return self._union

    def close(self):
        if self._union is not None:
            self._union.close()
            self._union = None

    def groupby_tables(self, groupby_cols, agg_list, where_terms=None):
        """(device result tables, reduced): one table over the union for decomposable
        aggregations, else one per shard."""
        if not self.tables:
            return [], False
        if decomposable(agg_list):
            cols = list(dict.fromkeys(list(groupby_cols) + [x[0] for x in agg_list] +
                                      [t[0] for t in (where_terms or [])]))
            u = self.union(cols)
            return [u.groupby_table(groupby_cols, agg_list, where_terms=where_terms)], True
        return [t.groupby_table(groupby_cols, agg_list, where_terms=where_terms) for t in self.tables], False

    def groupby_merged(self, groupby_cols, agg_list, dtypes, backend, exchange, where_terms=None):
        """The ``aggregate=True`` answer over every rank's shards (rank 0; None elsewhere)."""
        per, reduced = self.groupby_tables(groupby_cols, agg_list, where_terms)
        try:
            return merge_partials_device(per, groupby_cols, agg_list, dtypes, backend, exchange, reduced=reduced)
        finally:
            for p in per:
                p.close()
