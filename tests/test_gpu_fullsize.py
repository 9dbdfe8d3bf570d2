"""Full-size (BASELINE.json configs) parity on non-dyadic data: libbqgpu vs the C restatement
of bquery's per-shard groupby (oracle/cbquery.c).

* C2: 100 M rows, cent-rounded ("raw") fares -- float64 sum and bquery's row-order Knuth mean
  at 1e-12 relative (north_star), counts bit-exact.
* C3: 100 M rows, ~1 M groups (partitioned path), raw and dyadic data; keys, first-appearance
  group order and counts bit-exact, sums 1e-12 (bit-exact on dyadic data).
* C4: 200 M rows, random and (pu_location_id, passenger_count)-sorted row order;
  count_distinct and sorted_count_distinct bit-exact.
* C5: one rank's 10 shards x 12.5 M rows in one pass + the RCCL merge (world 1) against the
  reference client's merge of bquery's per-shard results.

The oracle sums every group strictly in row order (bquery's ``out[g] += v``,
bqueryd/worker.py:313 -> ctable.groupby); the GPU sums in a different order, so the float64
comparisons measure the reference's own rounding noise (~sqrt(n) ulp) as much as ours.
"""
import os

import numpy as np
import pytest

from bqueryd_amd import synth
from bqueryd_amd.engine import ShardTable
from tests.helpers import assert_tables_equal

pytestmark = pytest.mark.gpu


def _rel_err(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300))) if len(ref) else 0.0


def _gpu_groupby(cols, cfg):
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(cfg['groupby'], cfg['aggs'], where_terms=cfg['where'])
        mode = t.dev.last_timing()['mode']
    finally:
        t.close()
    return got, mode


def _float_cols(cfg, got):
    return [a[2] for a in cfg['aggs'] if got[a[2]].dtype.kind == 'f']


def test_c2_full_size_raw(oracle_c):
    cfg = synth.CONFIGS['c2']
    cols = synth.taxi_shard(cfg['rows'], config_id=2, variant='raw', columns=synth.query_columns(cfg))
    got, mode = _gpu_groupby(cols, cfg)
    ref = oracle_c.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where'])
    errs = {c: _rel_err(got[c], ref[c]) for c in _float_cols(cfg, got)}
    print('C2 raw: mode %d, max relative error %s' % (mode, errs))
    for c, e in errs.items():
        assert e <= 1e-12, (c, e)
    assert_tables_equal(got, ref, rtol=1e-12)


@pytest.mark.parametrize('variant', ['raw', 'exact'])
def test_c3_full_size(variant, oracle_c):
    cfg = synth.CONFIGS['c3']
    cols = synth.taxi_shard(cfg['rows'], config_id=3, variant=variant, columns=synth.query_columns(cfg))
    got, mode = _gpu_groupby(cols, cfg)
    ref = oracle_c.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where'])
    errs = {c: _rel_err(got[c], ref[c]) for c in _float_cols(cfg, got)}
    print('C3 %s: mode %d, %d groups, max relative error %s' % (variant, mode, len(ref['n']), errs))
    assert mode == 4  # the partitioned path
    assert len(ref['n']) > 900_000
    exact = {'fare_sum'} if variant == 'exact' else set()
    assert_tables_equal(got, ref, rtol=1e-12, exact_cols=exact)


@pytest.mark.parametrize('order', ['random', 'sorted'])
def test_c4_full_size(order, oracle_c):
    cfg = synth.CONFIGS['c4']
    sort_by = ['pu_location_id', 'passenger_count'] if order == 'sorted' else None
    cols = synth.taxi_shard(cfg['rows'], config_id=4, columns=synth.query_columns(cfg), sort_by=sort_by)
    got, mode = _gpu_groupby(cols, cfg)
    ref = oracle_c.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where'])
    print('C4 %s: mode %d, %d groups, scd total %d' % (order, mode, len(ref['pc_scd']), int(ref['pc_scd'].sum())))
    assert mode == 5  # the fused distinct pass
    assert_tables_equal(got, ref)


def test_float32_sum_realistic_groups(oracle_c):
    """float32 sums on cent-rounded data with 10^5 - 10^6 rows per group.

    bquery accumulates a float32 sum in float32 in row order (the oracle's restatement); at
    these group sizes that running sum drifts from the true sum by 2e-6 - 2e-4 relative
    (stagnation: an addend below half an ulp of the running sum is lost), and no parallel
    reduction can reproduce the drift.  libbqgpu defines a float32 sum as the float64 sum of
    the values rounded once to float32.  Checked here: bit-exact against that
    definition (float64 sums of cent values are exact to well below a float32 ulp), within the
    oracle's own drift of its row-order value, and the count / mean columns against the
    oracle at the usual tolerances."""
    rng = np.random.default_rng(31)
    n = 4_000_000
    cols = {'g': rng.integers(0, 8, n).astype(np.int32),
            'f': np.round(np.clip(rng.lognormal(2.3, 0.6, n), 2.5, 500.0), 2).astype(np.float32)}
    aggs = [['f', 'sum', 'fs'], ['f', 'mean', 'fm'], ['f', 'count', 'n']]
    t = ShardTable(cols)
    try:
        got, _ = t.groupby(['g'], aggs)
    finally:
        t.close()
    ref = oracle_c.groupby(cols, ['g'], aggs)
    np.testing.assert_array_equal(got['g'], ref['g'])
    np.testing.assert_array_equal(got['n'], ref['n'])
    np.testing.assert_allclose(got['fm'], ref['fm'], rtol=1e-12, atol=0)
    # float32 values of magnitude < 512 are multiples of 2^-20 or coarser, so float64 sums of
    # up to ~10^6 of them are exact in any order: one rounding to float32 is the definition
    label = np.empty(int(ref['g'].max()) + 1, np.int64)
    label[ref['g']] = np.arange(len(ref['g']))
    exact = np.bincount(label[cols['g']], weights=cols['f'].astype(np.float64), minlength=len(ref['g']))
    np.testing.assert_array_equal(got['fs'], exact.astype(np.float32))
    drift = np.abs(ref['fs'].astype(np.float64) - exact) / exact
    print('float32 row-order drift of the reference restatement: max %.2e' % drift.max())
    assert got['fs'].dtype == np.float32
    np.testing.assert_allclose(got['fs'], ref['fs'], rtol=max(1e-6, 2 * float(drift.max())), atol=0)


@pytest.mark.parametrize('variant', ['raw', 'exact'])
def test_c5_full_size(variant, oracle_c):
    """C5 at one rank's full share: 10 shards x 12.5 M rows (the C5 generator's shards 0-9),
    aggregated in one pass over their union (sum / count: ColocatedShards) and merged over a
    one-rank RCCL communicator (bqg_merge) -- against bquery's per-shard results merged by the
    reference client (rpc.py:164-173, aggregate=True): ~1 M groups in first-appearance order,
    counts bit-exact, sums 1e-12 (bit-exact on dyadic data)."""
    from collections import OrderedDict

    from bqueryd_amd import dist as bdist
    from oracle import bquery_oracle as bo
    cfg = synth.CONFIGS['c5']
    shard_rows = cfg['rows'] // cfg['shards']
    shards = [synth.taxi_shard(shard_rows, config_id=5, n_shards=cfg['shards'], shard=i, variant=variant,
                               columns=synth.query_columns(cfg)) for i in range(10)]
    tables = [ShardTable(s) for s in shards]
    colo = bdist.ColocatedShards(tables)
    try:
        per, reduced = colo.groupby_tables(cfg['groupby'], cfg['aggs'])
        assert reduced
        dtypes = OrderedDict((k, per[0].dtypes[k]) for k in per[0].names)
        for p in per:
            p.close()
        comm = bdist.RcclComm(tables[0].dev)
        try:
            got = colo.groupby_merged(cfg['groupby'], cfg['aggs'], dtypes, comm)
        finally:
            comm.close()
    finally:
        colo.close()
        for t in tables:
            t.close()
    ref = bo.client_merge([oracle_c.handle_work(s, cfg['groupby'], cfg['aggs'], cfg['where']) for s in shards],
                          cfg['groupby'], cfg['aggs'], aggregate=True)
    errs = {c: _rel_err(got[c], ref[c]) for c in _float_cols(cfg, got)}
    print('C5 %s: %d groups, max relative error %s' % (variant, len(ref['n']), errs))
    assert len(ref['n']) > 900_000
    exact = {'fare_sum'} if variant == 'exact' else set()
    assert_tables_equal(got, ref, rtol=1e-12, exact_cols=exact)


def _c5_shard_and_result(i, variant, oracle_c):
    """C5 generator shard i and bquery's per-shard result for it (the C restatement)."""
    cfg = synth.CONFIGS['c5']
    s = synth.taxi_shard(cfg['rows'] // cfg['shards'], config_id=5, n_shards=cfg['shards'], shard=i,
                         variant=variant, columns=synth.query_columns(cfg))
    return s, oracle_c.handle_work(s, cfg['groupby'], cfg['aggs'], cfg['where'])


@pytest.mark.parametrize('variant', ['raw', 'exact'])
def test_c5_full_shape_eight_ranks(variant, oracle_c):
    """C5 at its stated workload: 80 shards x 12.5 M rows = 1 B rows over 8 ranks (10 shards
    each, one libbqgpu context per rank, all on this box's one GPU), every rank's shards
    aggregated in one pass over their union, then the 8-rank merge (bqg_merge_group: pack
    kernel, count all-gather, per-column exchange, reduce, gather) over the in-process
    transport -- the code path RCCL runs, with device copies as the wire.  Against the
    reference client's merge (rpc.py:164-173, aggregate=True: concatenate the 80 per-shard
    bquery results, group by the keys, sum) of the C restatement's per-shard results; the
    client merge's groupby is the C restatement's too (the numpy one takes minutes on 80 M
    rows, and the two agree bit for bit on every golden case).  Rows compared after sorting by
    the keys (the merged order is by key hash; the client's is glob order, rpc.py:151):
    keys and counts bit-exact, sums within 1e-12 (bit-exact on dyadic data)."""
    from collections import OrderedDict
    from concurrent.futures import ThreadPoolExecutor

    from bqueryd_amd import dist as bdist
    from bqueryd_amd.engine import Device
    from tests.helpers import sort_by_keys
    cfg = synth.CONFIGS['c5']
    world = 8
    per_rank = cfg['shards'] // world
    devs = [Device(0) for _ in range(world)]
    tables = [[] for _ in range(world)]
    results = []
    # shard generation and the per-shard oracle on host threads (numpy's generators and the C
    # restatement release the GIL); each shard lands in its rank's context and is dropped
    with ThreadPoolExecutor(min(16, os.cpu_count() or 4)) as ex:
        for i, (s, r) in enumerate(ex.map(lambda i: _c5_shard_and_result(i, variant, oracle_c), range(cfg['shards']))):
            tables[i // per_rank].append(ShardTable(s, device=devs[i // per_rank]))
            results.append(r)
            del s
    colos = [bdist.ColocatedShards(t) for t in tables]
    per = []
    group = None
    try:
        for c in colos:
            p, reduced = c.groupby_tables(cfg['groupby'], cfg['aggs'])
            assert reduced
            per.append(p)
        dtypes = OrderedDict((k, per[0][0].dtypes[k]) for k in per[0][0].names)
        group = bdist.CommGroup(devs, transport='local')
        got = bdist.merge_group_device(per, cfg['groupby'], cfg['aggs'], dtypes, group, reduced=True)
    finally:
        if group is not None:
            group.close()
        for tabs in per:
            for p in tabs:
                p.close()
        for c in colos:
            c.close()
        for ts in tables:
            for t in ts:
                t.close()
    names = list(results[0].keys())
    cat = OrderedDict((n, np.concatenate([r[n] for r in results])) for n in names)
    del results
    ref = oracle_c.groupby(cat, cfg['groupby'], bdist.sum_spec(cfg['aggs']))
    got, ref = sort_by_keys(got, cfg['groupby']), sort_by_keys(ref, cfg['groupby'])
    errs = {c: _rel_err(got[c], ref[c]) for c in _float_cols(cfg, got)}
    print('C5 8 ranks %s: %d groups, %d rows, max relative error %s' % (variant, len(ref['n']), int(ref['n'].sum()), errs))
    assert int(ref['n'].sum()) == cfg['rows']
    assert len(ref['n']) > 990_000
    for c, e in errs.items():
        assert e <= 1e-12, (c, e)
    exact = {'fare_sum'} if variant == 'exact' else set()
    assert_tables_equal(got, ref, rtol=1e-12, exact_cols=exact)
