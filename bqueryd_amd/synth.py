"""Deterministic synthetic NYC-taxi-shaped shards.

Seeds: ``numpy.random.Generator(PCG64(SeedSequence(0xB0C0 + config_id).spawn(n_shards)[i]))``.
Float value columns come in two variants:
* ``exact`` -- quantised to multiples of 2**-6, so every partial sum is exact in float64 and
  GPU/CPU sums agree bit for bit in any order;
* ``raw`` -- rounded to cents (tolerance tests).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

PAYMENT_W = np.array([0.55, 0.30, 0.06, 0.04, 0.02, 0.01, 0.006, 0.002, 0.001, 0.001])
PASSENGER_W = np.array([0.002, 0.70, 0.14, 0.04, 0.02, 0.05, 0.045, 0.001, 0.001, 0.001])

COLUMNS = ('payment_type', 'vendor_id', 'pu_location_id', 'pickup_location', 'passenger_count',
           'fare_amount', 'trip_distance')


def _choice(rng, weights, n, offset=0):
    cdf = np.cumsum(weights / weights.sum())
    cdf[-1] = 1.0
    u = rng.random(n)
    return (np.searchsorted(cdf, u, side='right') + offset).astype(np.int32)


def shard_rng(config_id, n_shards, i):
    ss = np.random.SeedSequence(0xB0C0 + int(config_id)).spawn(int(n_shards))[int(i)]
    return np.random.Generator(np.random.PCG64(ss))


def taxi_shard(nrows, config_id=0, n_shards=1, shard=0, variant='exact', columns=COLUMNS,
               sort_by=None):
    """One shard as an OrderedDict of numpy columns."""
    rng = shard_rng(config_id, n_shards, shard)
    n = int(nrows)
    out = OrderedDict()
    # draw every column (fixed order) so a subset is the same data as the full shard
    payment = _choice(rng, PAYMENT_W, n)
    vendor = np.where(rng.random(n) < 0.47, 1, 2).astype(np.int32)
    zipf_w = 1.0 / np.arange(1, 266, dtype=np.float64) ** 1.1
    pu = _choice(rng, zipf_w, n, offset=1)
    pickup = rng.integers(0, 500000, n, dtype=np.int32)
    pcount = _choice(rng, PASSENGER_W, n)
    fare = np.clip(rng.lognormal(2.3, 0.6, n), 2.5, 500.0)
    dist = np.clip(rng.lognormal(0.6, 0.8, n), 0.0, 100.0)
    if variant == 'exact':
        fare = np.round(fare * 64.0) / 64.0
        dist = np.round(dist * 64.0) / 64.0
    else:
        fare = np.round(fare, 2)
        dist = np.round(dist, 2)
    full = {'payment_type': payment, 'vendor_id': vendor, 'pu_location_id': pu,
            'pickup_location': pickup, 'passenger_count': pcount, 'fare_amount': fare,
            'trip_distance': dist}
    if sort_by:
        order = np.lexsort(tuple(full[c] for c in reversed(sort_by)))
        full = {k: v[order] for k, v in full.items()}
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
