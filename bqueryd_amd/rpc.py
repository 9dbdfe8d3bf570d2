"""Gather and client-side merge of per-shard results.

* ``tar_of_tars`` restates ``ControllerNode.process_sink_results`` (bqueryd/controller.py:
  146-221): once every shard replied, the per-shard result tars are packed into one tar with
  ``arcname=filename``; empty ``''`` replies are skipped (controller.py:175-179,196).
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
