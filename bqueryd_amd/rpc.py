"""Gather and client-side merge of per-shard results.

* ``tar_of_tars`` restates ``ControllerNode.process_sink_results`` (bqueryd/controller.py:
  146-221): once every shard replied, the per-shard result tars are packed into one tar with
  ``arcname=filename``; empty ``''`` replies are skipped (controller.py:175-179,196).
* ``fan_out`` / ``CalcSegment`` restate the controller's scatter (controller.py:471-508) and
  its gather accounting (controller.py:146-221), with the node-level patch of
  INTEGRATION.md §4 (one message and one reply covering a GPU node's files).
* ``uncompress_groupby_to_df`` restates ``RPC.uncompress_groupby_to_df`` (bqueryd/rpc.py:
  134-179): each inner tar is opened as a ctable and appended; with ``aggregate=True`` the
  appended table is re-grouped with ``sum`` of every finalized column ("we can only sum now",
  rpc.py:170-171) -- here on the GPU; otherwise the concatenation is returned.  No shard
  results -> empty ``DataFrame()``.  Member order follows ``glob`` in the reference (file
  system order); this implementation uses sorted member names, and parity is compared after
  sorting by the group keys (the reference's order is not stable).
"""
from __future__ import annotations

import io
import tarfile
from collections import OrderedDict

import numpy as np

from . import bcolz_io
from .ctable import ctable


def tar_of_tars(results):
    """``results``: mapping filename -> tar bytes (or '' / None for an empty reply)."""
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode='w') as archive:
        for filename, data in results.items():
            if not data:
                continue
            info = tarfile.TarInfo(name=filename)
            info.size = len(data)
            archive.addfile(info, io.BytesIO(data))
    return buf.getvalue()


def _is_calc_worker(info):
    # find_free_worker skips the download / movebcolz workers (controller.py:119-121)
    return info.get('workertype') not in ('download', 'movebcolz')


def fan_out(args, kwargs, worker_map=None, files_map=None):
    """The controller's scatter of one groupby RPC (``handle_calc_message``,
    controller.py:471-508) with the node-level patch of INTEGRATION.md §4.

    Returns the outgoing messages in send order as dicts ``{'args', 'filename', 'worker_id'}``
    (the fields ``handle_out`` reads, controller.py:248-257).  ``worker_map`` /
    ``files_map`` are the controller's own maps (controller.py:322-330): a calc worker that
    registered with ``'gpu_node': True`` takes, in ONE message pinned to it by ``worker_id``,
    every file of the RPC that ``files_map`` lists for that very worker -- so the message can
    only reach a worker that holds all of its files, whoever else also holds the first one.
    Used only when the client merges by sum (``kwargs['aggregate'] is True``) and a GPU worker
    holds at least two of the files; every other file gets its own unpinned message
    (``worker_id`` None: ``find_free_worker`` by file name), exactly as in the reference."""
    args = list(args)
    if len(args) != 4:
        raise ValueError('expecting: path_list, groupby_col_list, measure_col_list, where_terms_list')
    filenames = list(args[0])
    if not filenames:
        raise ValueError('no filenames given')
    files_map = files_map or {}
    out = []
    covered = set()
    if kwargs.get('aggregate') is True and worker_map:
        for wid in sorted(worker_map):
            info = worker_map[wid]
            if not info.get('gpu_node') or not _is_calc_worker(info):
                continue
            files = [f for f in filenames if f not in covered and wid in files_map.get(f, ())]
            if len(files) < 2:
                continue
            out.append({'args': [files] + args[1:], 'filename': files[0], 'worker_id': wid})
            covered.update(files)
    out += [{'args': [f] + args[1:], 'filename': f, 'worker_id': None} for f in filenames if f not in covered]
    return out


def find_free_worker(worker_map, files_map, filename=None, needs_local=False, node_name=None, rng=None):
    """``ControllerNode.find_free_worker`` (controller.py:113-144): a random non-busy calc
    worker that has ``filename`` (a local one when ``needs_local``); None when there is none."""
    import random
    rng = rng or random
    free, local = [], []
    for wid, info in worker_map.items():
        if not _is_calc_worker(info) or info.get('busy'):
            continue
        if filename and wid not in files_map.get(filename, ()):
            continue
        free.append(wid)
        if info.get('node') == node_name:
            local.append(wid)
    if not free:
        return None
    if needs_local:
        return rng.choice(local) if local else None
    return rng.choice(free)


def route(msg, worker_map, files_map, node_name=None, rng=None):
    """The worker choice of ``handle_out`` (controller.py:248-257): a pinned ``worker_id`` is
    used as is (the reference does not re-check it), ``'__needs_local__'`` and None go through
    ``find_free_worker`` by the message's ``filename``."""
    wid = msg.get('worker_id')
    if wid == '__needs_local__':
        return find_free_worker(worker_map, files_map, msg.get('filename'), True, node_name, rng)
    if wid is None:
        return find_free_worker(worker_map, files_map, msg.get('filename'), rng=rng)
    return wid


class CalcSegment:
    """The gather state of one scattered RPC (``rpc_segment``, controller.py:489-491) and the
    accounting of ``process_sink_results`` (controller.py:146-221): the reply to the client
    goes out once every file name has a result (controller.py:186).  A node-level reply (its
    ``args[0]`` a list of files) stores its tar under the first file and
    completes the others with ``None`` entries, which the tar of tars skips
    (controller.py:195-197); ``''`` replies (the factorization-check early-out) are skipped
    the same way (controller.py:175-179)."""

    def __init__(self, filenames):
        self.filenames = OrderedDict((f, None) for f in filenames)
        self.results = OrderedDict()

    def add_reply(self, args, data):
        """One worker reply (its message's args and ``data``); True when the RPC is complete."""
        names = list(args[0]) if isinstance(args[0], (list, tuple)) else [args[0]]
        if not names:
            raise ValueError('a reply without a file name')
        for f in names:
            if f not in self.filenames:
                raise KeyError('reply for %r, which this RPC did not ask for' % (f,))
        self.results[names[0]] = data if data else None
        for other in names[1:]:
            self.results[other] = None
        return self.complete

    @property
    def complete(self):
        return len(self.results) == len(self.filenames)

    def tar(self):
        """The reply's tar of tars (controller.py:192-209); only once complete."""
        if not self.complete:
            raise RuntimeError('%d of %d files have no result yet' % (len(self.filenames) - len(self.results),
                                                                      len(self.filenames)))
        return tar_of_tars(self.results)


def read_shard_results(result_tar):
    """-> list of OrderedDict tables, one per non-empty shard reply, in member-name order.

    The reference untars every inner tar into a temporary directory and opens it as a
    ctable (rpc.py:137-162); here the inner tars are read in memory (same files, no disk
    round trip): the ctable directory is the first top-level entry of each inner tar."""
    tables = []
    with tarfile.open(fileobj=io.BytesIO(result_tar), mode='r') as outer:
        members = sorted(outer.getmembers(), key=lambda m: m.name)
        for m in members:
            inner = outer.extractfile(m).read()
            with tarfile.open(fileobj=io.BytesIO(inner), mode='r') as t:
                files = [x for x in t.getmembers() if x.isfile()]
                if not files:
                    continue
                top = sorted(set(x.name.split('/', 1)[0] for x in files))[0]
                data = {x.name.split('/', 1)[1]: t.extractfile(x).read() for x in files
                        if x.name.startswith(top + '/')}
            tables.append(bcolz_io.read_ctable_files(data))
    return tables


def merge_tables(tables, groupby_col_list, agg_list, aggregate=False, device=None):
    """Append per-shard tables; ``aggregate``: GPU re-group with sum of the finalized columns."""
    if not tables:
        return None
    names = list(tables[0].keys())
    cat = OrderedDict((n, np.concatenate([t[n] for t in tables])) for n in names)
    if not aggregate:
        return cat
    new_agg_list = [[x[2], 'sum', x[2]] for x in agg_list]
    ct = ctable(columns=cat, device=device)
    try:
        return ct.groupby(groupby_col_list, new_agg_list).columns
    finally:
        ct.close()


def uncompress_groupby_to_df(result_tar, groupby_col_list, agg_list, where_terms_list, aggregate=False,
                             device=None):
    import pandas as pd
    merged = merge_tables(read_shard_results(result_tar), groupby_col_list, agg_list, aggregate, device)
    if merged is None:
        return pd.DataFrame()
    return pd.DataFrame(merged)
