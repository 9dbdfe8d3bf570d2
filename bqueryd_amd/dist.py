"""Cross-GPU merge of per-shard results for ``aggregate=True``.

The reference merges on the client: every shard's finalized table is appended and re-grouped
with ``sum`` of every column ("we can only sum now", ``bqueryd/rpc.py:164-173``).  For shards
co-located on one node the same merge runs across GPU ranks:

  1. local:     each rank sums its own shards' tables by key (GPU groupby-sum);
  2. partition: rows are assigned to rank ``hash(key values) mod world`` (``bqg_hash_partition``:
                a pure function of the key values, identical on every rank, so all partials of
                one key meet on one rank);
  3. exchange:  row counts, then the rows, between every pair of ranks;
  4. reduce:    each rank sums the rows it received by key;
  5. gather:    the reduced partitions travel to rank 0.

The product path is ``merge_partials_device`` / ``merge_group_device``: libbqgpu's ``bqg_merge``
runs all five steps on device buffers with RCCL over xGMI (``RcclComm``: one process per GPU;
``CommGroup``: a process owning several GPUs).  The protocol's host-side specification (the
same five steps over torch.distributed, run under gloo by the CPU test suite) lives with the
tests, ``tests/merge_protocol.py``.
"""
from __future__ import annotations

import ctypes
import time
from collections import OrderedDict

import numpy as np


def sum_spec(agg_list):
    """The client's merge aggregation list: ``[[x[2], 'sum', x[2]] for x in agg_list]``."""
    return [[x[2], 'sum', x[2]] for x in agg_list]


def new_unique_id():
    """An RCCL unique id (``bqg_comm_unique_id``): created once, on rank 0, and handed to every
    rank by the host layer over any side channel (bytes)."""
    from . import _lib as L
    buf = ctypes.create_string_buffer(L.UNIQUE_ID_BYTES)
    L.check(L.lib().bqg_comm_unique_id(buf), None)
    return buf.raw


class RcclComm:
    """This process's rank of an RCCL communicator over the node's GPUs (``bqg_comm_init``
    on a libbqgpu context: one process per GPU).  The merge's exchange runs inside libbqgpu on
    device buffers; torch is not involved."""

    def __init__(self, device, rank=0, nranks=1, unique_id=None):
        from . import _lib as L
        if unique_id is None:
            if nranks != 1:
                raise ValueError('every rank needs the same unique id (new_unique_id on rank 0)')
            unique_id = new_unique_id()
        self.device = device
        self.rank, self.world = int(rank), int(nranks)
        buf = ctypes.create_string_buffer(bytes(unique_id), L.UNIQUE_ID_BYTES)
        device.check(L.lib().bqg_comm_init(device.handle, self.rank, self.world, buf))

    def close(self):
        from . import _lib as L
        if self.device is not None and self.device.handle:
            L.lib().bqg_comm_destroy(self.device.handle)
        self.device = None


class CommGroup:
    """Every rank of a communicator in THIS process, one libbqgpu context (Device) per rank:
    ``transport='rccl'`` -- RCCL over xGMI, one GPU per rank (``bqg_comm_init_all``, a process
    owning the node's GPUs); ``'local'`` -- device-to-device copies (``bqg_comm_init_local``;
    contexts may share one GPU)."""

    def __init__(self, devices, transport='rccl'):
        from . import _lib as L
        self.devices = list(devices)
        self.world = len(self.devices)
        arr = (ctypes.c_void_p * self.world)(*[d.handle.value for d in self.devices])
        fn = L.lib().bqg_comm_init_all if transport == 'rccl' else L.lib().bqg_comm_init_local
        self.devices[0].check(fn(self.world, arr))
        self.transport = transport

    def close(self):
        from . import _lib as L
        for d in self.devices:
            if d.handle:
                L.lib().bqg_comm_destroy(d.handle)
        self.devices = []


MERGE_PHASES = ('local', 'counts', 'exchange', 'reduce', 'gather_counts', 'gather')


def merge_phases(device):
    """Host wall time (ms) of this context's rank in the last merge, per phase
    (``bqg_comm_last_phases``; collective steps charged to every rank of the call)."""
    from . import _lib as L
    out = (ctypes.c_double * len(MERGE_PHASES))()
    device.check(L.lib().bqg_comm_last_phases(device.handle, out, len(MERGE_PHASES)))
    return OrderedDict(zip(MERGE_PHASES, list(out)))


def merge_progress(device):
    """Where this context's rank is in its merges (``bqg_comm_progress``; safe while a merge
    runs on another thread): the phase entered last (``'idle'`` between merges) and the merges
    begun / ended -- what a watchdog reports for a rank whose collective does not return."""
    from . import _lib as L
    ph, started, done = ctypes.c_int32(-1), ctypes.c_int64(0), ctypes.c_int64(0)
    device.check(L.lib().bqg_comm_progress(device.handle, ctypes.byref(ph), ctypes.byref(started),
                                           ctypes.byref(done)))
    return {'phase': MERGE_PHASES[ph.value] if 0 <= ph.value < len(MERGE_PHASES) else 'idle',
            'merges_started': started.value, 'merges_done': done.value}


def _schema(groupby_cols, agg_list, dtypes):
    """(column names, C dtype codes) of the merge: datetime64 keys travel as their int64 ticks;
    string keys cannot merge on the device (each table's dictionary codes are its own)."""
    from . import _lib as L
    from .engine import device_dtype, is_string
    names = list(groupby_cols) + [x[2] for x in agg_list]
    for n in names:
        if is_string(dtypes[n]):
            raise NotImplementedError('device merge of a string column (%s): merge the host results' % n)
    codes = (ctypes.c_int32 * len(names))(*[L.DTYPE_CODE[device_dtype(dtypes[n])] for n in names])
    return names, codes


def _logical(cols, dtypes):
    """datetime64 / timedelta64 columns back from their ticks."""
    from .engine import is_time
    for n in list(cols):
        if is_time(dtypes[n]):
            cols[n] = np.ascontiguousarray(cols[n]).view(dtypes[n])
    return cols


def merge_partials_device(local_tables, groupby_cols, agg_list, dtypes, comm, reduced=False):
    """The client's ``aggregate=True`` merge (rpc.py:164-173) of every rank's shard results,
    in HBM over RCCL (``bqg_merge_host``): ``local_tables`` are this rank's finalized shard
    tables as device ShardTables (``ShardTable.groupby_table``), keys first.  Returns the merged
    table (host columns, zero-copy views of the library's pinned result) on rank 0, None
    elsewhere.  ``reduced``: ``local_tables`` is ONE table with unique keys
    (``ColocatedShards`` one-pass groupby): the local re-group is skipped.  Rows come grouped by
    key hash; the reference's order is the client's file-system glob order (rpc.py:151), so
    compare after sorting by the keys."""
    from . import _lib as L
    from .engine import _result_to_columns
    names, codes = _schema(groupby_cols, agg_list, dtypes)
    tabs = [t for t in local_tables if t is not None]
    arr = (ctypes.c_void_p * max(1, len(tabs)))(*[t.handle.value for t in tabs])
    out = ctypes.c_void_p()
    dev = comm.device
    dev.check(L.lib().bqg_merge_host(dev.handle, len(tabs), arr, len(groupby_cols), len(names), codes,
                                     1 if reduced else 0, ctypes.byref(out)))
    if comm.rank != 0 or not out.value:
        return None
    return _logical(_result_to_columns(dev, out, names)[0], dtypes)


class SharedResult:
    """A merged result in host memory shared by the node's rank processes
    (``bqg_merge_shared_host``): rank 0 creates the block (POSIX shared memory), the other ranks
    attach to it by name, and every rank's merge copies its partition into its slice over its
    own link -- the result is complete in rank 0's memory when its merge returns, without a
    gather to rank 0 or one large copy behind one link.  Layout (the library's): column j at
    sum over j' < j of align256(capacity x itemsize(j')), rows in rank order."""

    def __init__(self, name, capacity_rows, names, dtypes, create):
        from multiprocessing import shared_memory
        from .engine import device_dtype
        self.name, self.names, self.create = name, list(names), bool(create)
        self.dtypes = {n: np.dtype(dtypes[n]) for n in self.names}
        self.capacity = int(capacity_rows)
        self.offsets, off = [], 0
        for n in self.names:
            self.offsets.append(off)
            off += (self.capacity * np.dtype(device_dtype(self.dtypes[n])).itemsize + 255) & ~255
        self.nbytes = max(off, 1)
        if create:
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=self.nbytes)
        else:
            self.shm = shared_memory.SharedMemory(name=name)
            try:  # an attaching process must not unlink the creator's block at its exit
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, 'shared_memory')
            except Exception:
                pass
        self._bytes = np.frombuffer(self.shm.buf, np.uint8, self.nbytes)
        self.ptr = self._bytes.ctypes.data

    def columns(self, rows):
        """The merged table: views of the block's first ``rows`` rows of every column."""
        from .engine import device_dtype
        out = OrderedDict()
        for n, off in zip(self.names, self.offsets):
            dt = np.dtype(device_dtype(self.dtypes[n]))
            out[n] = self._bytes[off:off + rows * dt.itemsize].view(dt)
        return _logical(out, self.dtypes)

    def close(self):
        self._bytes = None
        try:
            self.shm.close()
        except BufferError:  # views still held by the caller: the mapping goes with the process
            return
        if self.create:
            self.shm.unlink()


def merge_partials_shared(local_tables, groupby_cols, agg_list, dtypes, comm, shared, reduced=False):
    """``merge_partials_device`` for one process per GPU with the merged rows written straight
    into ``shared`` (a ``SharedResult`` every rank maps; ``bqg_merge_shared_host``).  Returns
    the merged row count on every rank (``shared.columns(rows)`` reads them on any rank).  A
    block too small for the merge raises ValueError carrying the rows it needs (every rank alike)."""
    from . import _lib as L
    names, codes = _schema(groupby_cols, agg_list, dtypes)
    if list(names) != shared.names:
        raise ValueError('shared result columns %s, merge schema %s' % (shared.names, names))
    tabs = [t for t in local_tables if t is not None]
    arr = (ctypes.c_void_p * max(1, len(tabs)))(*[t.handle.value for t in tabs])
    rows = ctypes.c_int64(0)
    dev = comm.device
    rc = L.lib().bqg_merge_shared_host(dev.handle, len(tabs), arr, len(groupby_cols), len(names), codes,
                                       1 if reduced else 0, ctypes.c_void_p(shared.ptr), shared.capacity,
                                       ctypes.byref(rows))
    if rc == L.E_INVALID and rows.value > shared.capacity:
        raise ValueError('shared merge result too small: %d rows needed' % rows.value, rows.value)
    dev.check(rc)
    return rows.value


def merge_group_device(tables_per_rank, groupby_cols, agg_list, dtypes, group, reduced=False):
    """``merge_partials_device`` for every rank of a ``CommGroup`` from one host thread
    (``bqg_merge_group_host``): ``tables_per_rank[i]`` are rank i's device tables (on
    ``group.devices[i]``).  Every rank copies its reduced partition straight into its slice of
    one pinned host result (no gather to rank 0).  Returns the merged table (host columns)."""
    from . import _lib as L
    from .engine import _result_to_columns
    names, codes = _schema(groupby_cols, agg_list, dtypes)
    flat, counts = [], []
    for tabs in tables_per_rank:
        tabs = [t for t in tabs if t is not None]
        counts.append(len(tabs))
        flat += [t.handle.value for t in tabs]
    w = group.world
    ctxs = (ctypes.c_void_p * w)(*[d.handle.value for d in group.devices])
    ntab = (ctypes.c_int32 * w)(*counts)
    arr = (ctypes.c_void_p * max(1, len(flat)))(*flat)
    out = ctypes.c_void_p()
    t0 = time.perf_counter()
    group.devices[0].check(L.lib().bqg_merge_group_host(w, ctxs, ntab, arr, len(groupby_cols), len(names), codes,
                                                        1 if reduced else 0, ctypes.byref(out)))
    LAST_MERGE.update(merge_ms=1e3 * (time.perf_counter() - t0))
    return _logical(_result_to_columns(group.devices[0], out, names)[0], dtypes)


def merge_group_device_table(tables_per_rank, groupby_cols, agg_list, dtypes, group, reduced=False):
    """The device-result variant (``bqg_merge_group``): the merged table gathered to rank 0 as
    a device ShardTable (a later query can run on it in HBM)."""
    from . import _lib as L
    from .engine import ShardTable
    names, codes = _schema(groupby_cols, agg_list, dtypes)
    flat, counts = [], []
    for tabs in tables_per_rank:
        tabs = [t for t in tabs if t is not None]
        counts.append(len(tabs))
        flat += [t.handle.value for t in tabs]
    w = group.world
    ctxs = (ctypes.c_void_p * w)(*[d.handle.value for d in group.devices])
    ntab = (ctypes.c_int32 * w)(*counts)
    arr = (ctypes.c_void_p * max(1, len(flat)))(*flat)
    outs = (ctypes.c_void_p * w)()
    group.devices[0].check(L.lib().bqg_merge_group(w, ctxs, ntab, arr, len(groupby_cols), len(names), codes,
                                                   1 if reduced else 0, outs))
    return ShardTable._wrap(ctypes.c_void_p(outs[0]), names, [dtypes[n] for n in names], group.devices[0])


# host wall time of the last merge_group_device (profiling)
LAST_MERGE = {}


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
        self._union_key = None

    def union(self, cols):
        """The member shards' columns ``cols`` row-concatenated in HBM, kept while the members
        are unchanged (their identity and write versions) and extended, never narrowed: a query
        over new columns rebuilds the union with the old and new columns together."""
        from .engine import ShardTable
        key = tuple((id(t), t.version) for t in self.tables)
        if self._union is not None and key == self._union_key and set(cols) <= set(self._union_cols):
            return self._union
        if key == self._union_key:
            cols = tuple(dict.fromkeys(tuple(self._union_cols) + tuple(cols)))
        else:
            cols = tuple(cols)
        if self._union is not None:
            self._union.close()
        self._union = ShardTable.from_parts(self.tables, list(cols), device=self.tables[0].dev)
        self._union_cols = cols
        self._union_key = key
        return self._union

    def resident_bytes(self):
        """HBM held by the union (0 when none is built)."""
        u = self._union
        return 0 if u is None or not getattr(u, 'handle', None) else u.device_bytes()

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

    def groupby_merged(self, groupby_cols, agg_list, dtypes, comm, where_terms=None):
        """The ``aggregate=True`` answer over every rank's shards (rank 0; None elsewhere)."""
        per, reduced = self.groupby_tables(groupby_cols, agg_list, where_terms)
        try:
            return merge_partials_device(per, groupby_cols, agg_list, dtypes, comm, reduced=reduced)
        finally:
            for p in per:
                p.close()
