"""Deterministic synthetic NYC-taxi-shaped shards.

Seeds: ``SeedSequence(0xB0C0 + config_id).spawn(n_shards)[i]``, spawned once more into one
PCG64 stream per column (COLUMNS order), so any subset of the columns is drawn alone and is
the same data as in the full shard.
Float value columns come in two variants:
* ``exact`` -- quantised to multiples of 2**-6, so every partial sum is exact in float64 and
  GPU/CPU sums agree bit for bit in any order;
* ``raw`` -- rounded to cents (tolerance tests);
* ``wide`` -- fare_amount with refunds and outliers (cents spanning ~2 M codes: the 8-byte
  partition entries instead of the packed 4-byte ones); other columns as ``raw``.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

PAYMENT_W = np.array([0.55, 0.30, 0.06, 0.04, 0.02, 0.01, 0.006, 0.002, 0.001, 0.001])
PASSENGER_W = np.array([0.002, 0.70, 0.14, 0.04, 0.02, 0.05, 0.045, 0.001, 0.001, 0.001])

COLUMNS = ('payment_type', 'vendor_id', 'pu_location_id', 'pickup_location', 'passenger_count',
           'fare_amount', 'trip_distance', 'store_and_fwd_flag', 'vendor_name', 'pickup_datetime')
# the taxi frame's non-numeric columns (tests/test_simple_rpc.py:22-26 builds its shards from the
# full CSV with parse_dates): a one-byte flag ('N' / 'Y', a few empty), a unicode vendor name
# and the pickup time (datetime64[ns], January 2016)
STRING_COLUMNS = ('store_and_fwd_flag', 'vendor_name')


def _choice(rng, weights, n, offset=0):
    cdf = np.cumsum(weights / weights.sum())
    cdf[-1] = 1.0
    u = rng.random(n)
    return (np.searchsorted(cdf, u, side='right') + offset).astype(np.int32)


def shard_rng(config_id, n_shards, i):
    ss = np.random.SeedSequence(0xB0C0 + int(config_id)).spawn(int(n_shards))[int(i)]
    return np.random.Generator(np.random.PCG64(ss))


def _column_rngs(config_id, n_shards, i):
    """One child stream per column (fixed COLUMNS order): a subset of the columns is the same
    data as the full shard, and only the requested columns are drawn."""
    ss = np.random.SeedSequence(0xB0C0 + int(config_id)).spawn(int(n_shards))[int(i)]
    return {c: np.random.Generator(np.random.PCG64(s)) for c, s in zip(COLUMNS, ss.spawn(len(COLUMNS)))}


def _draw(name, rng, n, variant):
    if name == 'payment_type':
        return _choice(rng, PAYMENT_W, n)
    if name == 'vendor_id':
        return np.where(rng.random(n) < 0.47, 1, 2).astype(np.int32)
    if name == 'pu_location_id':
        return _choice(rng, 1.0 / np.arange(1, 266, dtype=np.float64) ** 1.1, n, offset=1)
    if name == 'pickup_location':
        return rng.integers(0, 500000, n, dtype=np.int32)
    if name == 'passenger_count':
        return _choice(rng, PASSENGER_W, n)
    if name == 'store_and_fwd_flag':
        return np.array([b'N', b'Y', b''], dtype='S1')[_choice(rng, np.array([0.989, 0.01, 0.001]), n)]
    if name == 'vendor_name':
        return np.array(['CMT', 'VTS', 'DDS', 'VeriFone'], dtype='U8')[_choice(rng, np.array([0.45, 0.5, 0.03, 0.02]), n)]
    if name == 'pickup_datetime':
        t0 = np.datetime64('2016-01-01T00:00:00', 'ns').astype(np.int64)
        ticks = np.sort(rng.integers(0, 31 * 86400, n)).astype(np.int64) * 1_000_000_000
        return (t0 + ticks).view('M8[ns]')
    if name == 'fare_amount':
        if variant == 'wide':
            # a real fare column's tails: refunds (negative) and outliers in the thousands, in
            # cents -- ~2 M distinct codes, too wide for the packed 16-bit partition entries
            v = rng.lognormal(2.3, 0.6, n)
            v = np.where(rng.random(n) < 0.01, v * rng.uniform(-5.0, 400.0, n), v)
            return np.round(np.clip(v, -1000.0, 10000.0), 2)
        v = np.clip(rng.lognormal(2.3, 0.6, n), 2.5, 500.0)
    else:  # trip_distance
        v = np.clip(rng.lognormal(0.6, 0.8, n), 0.0, 100.0)
    if variant == 'exact':
        return np.round(v * 64.0) / 64.0
    return np.round(v, 2)


def _stable_order(keys):
    """Row order sorting by ``keys`` (first key most significant), stable.  Small-range
    integer keys combine into one narrow code (numpy's stable sort is a radix sort there)."""
    code = np.zeros(len(keys[0]), np.int64)
    span = 1
    for k in reversed(keys):
        lo, hi = int(k.min()), int(k.max())
        code += (k.astype(np.int64) - lo) * span
        span *= hi - lo + 1
    if span <= 1 << 16:
        code = code.astype(np.uint16)
    elif span <= 1 << 32:
        code = code.astype(np.uint32)
    return np.argsort(code, kind='stable')


def taxi_shard(nrows, config_id=0, n_shards=1, shard=0, variant='exact', columns=COLUMNS,
               sort_by=None):
    """One shard as an OrderedDict of numpy columns."""
    rngs = _column_rngs(config_id, n_shards, shard)
    n = int(nrows)
    need = list(dict.fromkeys(list(columns) + list(sort_by or [])))
    full = {c: _draw(c, rngs[c], n, variant) for c in need}
    if sort_by:
        order = _stable_order([full[c] for c in sort_by])
        full = {k: v[order] for k, v in full.items()}
    out = OrderedDict()
    for c in columns:
        out[c] = full[c]
    return out


# BASELINE.json configs -- (rows, shards, query)
CONFIGS = {
    'c1': dict(rows=10_000_000, shards=10, groupby=['payment_type'],
               aggs=[['fare_amount', 'sum', 'fare_amount']], where=[], aggregate=True),
    'c2': dict(rows=100_000_000, shards=1, groupby=['payment_type'],
               aggs=[['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'mean', 'fare_mean'],
                     ['fare_amount', 'count', 'fare_cnt']],
               where=[('passenger_count', '>=', 2)], aggregate=True),
    'c3': dict(rows=100_000_000, shards=1, groupby=['pickup_location', 'vendor_id'],
               aggs=[['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']],
               where=[], aggregate=True),
    'c4': dict(rows=200_000_000, shards=1, groupby=['pu_location_id'],
               aggs=[['passenger_count', 'count_distinct', 'pc_cd'],
                     ['passenger_count', 'sorted_count_distinct', 'pc_scd']],
               where=[], aggregate=True),
    'c5': dict(rows=1_000_000_000, shards=80, groupby=['pickup_location', 'vendor_id'],
               aggs=[['fare_amount', 'sum', 'fare_sum'], ['fare_amount', 'count', 'n']],
               where=[], aggregate=True),
}
CONFIG_ID = {'c1': 1, 'c2': 2, 'c3': 3, 'c4': 4, 'c5': 5}


def query_columns(cfg):
    cols = list(cfg['groupby'])
    for a in cfg['aggs']:
        c = a[0] if isinstance(a, list) else a
        if c not in cols:
            cols.append(c)
    for t in cfg['where']:
        if t[0] not in cols:
            cols.append(t[0])
    return cols
