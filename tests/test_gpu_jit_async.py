"""Run-time compilation off the query path (option jit_async, bqg_jit_wait):
on a cold JIT cache a query shape runs the precompiled generic kernel at once while a
background host thread compiles its specialised kernel; the next query of the shape runs the
specialised kernel, and both give the same bits (reference: one message is one query,
bqueryd/worker.py:313 -- there is no warm-up query to hide a compile behind)."""
import glob
import os
import time
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd.engine import ShardTable
from tests.helpers import assert_tables_equal

pytestmark = pytest.mark.gpu


def _cols(mode, n, rng):
    # a query shape no other test compiles (uint16 key, int16 terms, uint32 / float32 sums), so
    # this process's memory cache cannot hold it either
    k = rng.integers(0, 9 if mode == 'private' else 300_000, n)
    return OrderedDict(k=k.astype(np.uint16 if mode == 'private' else np.int32),
                       t=rng.integers(-300, 300, n).astype(np.int16),
                       u=rng.integers(0, 1 << 20, n).astype(np.uint32),
                       f=(np.round(rng.normal(size=n) * 64) / 64).astype(np.float32),
                       d=rng.integers(-10**6, 10**6, n) / 100.0)


@pytest.mark.parametrize('mode', ['private', 'partitioned'])
def test_cold_shape_runs_generic_then_specialised(mode, oracle_c, engine_options, monkeypatch, tmp_path):
    monkeypatch.setenv('BQGPU_JIT_CACHE', str(tmp_path))
    engine_options(jit=1, jit_min_rows=0, jit_async=1)
    rng = np.random.default_rng(7 if mode == 'private' else 8)
    n = 400_007
    cols = _cols(mode, n, rng)
    aggs = [['u', 'sum', 'us'], ['f', 'mean', 'fm'], ['d', 'sum', 'ds'], ['u', 'count', 'n']]
    if mode == 'partitioned':
        aggs = [['d', 'sum', 'ds'], ['u', 'count', 'n']]
    terms = [('t', 'nin', [-7, 0, 11, 13, 250]), ('t', '>', -290)]
    t = ShardTable(cols)
    try:
        t0 = time.perf_counter()
        first, _ = t.groupby(['k'], aggs, where_terms=terms)
        first_s = time.perf_counter() - t0
        info1 = t.dev.last_timing()
        assert info1['mode'] == {'private': 0, 'partitioned': 4}[mode], info1
        assert not info1['specialized'], 'a cold shape must not wait for its compile'
        w = t.dev.jit_wait(300)
        assert w['idle'] and w['compiled'] >= 1, w
        assert glob.glob(os.path.join(str(tmp_path), '*.hsaco')), 'the background compile writes the disk cache'
        second, _ = t.groupby(['k'], aggs, where_terms=terms)
        info2 = t.dev.last_timing()
        assert info2['specialized'], info2
    finally:
        t.close()
    # no compile on the query path: far below a hiprtc compile (seconds)
    assert first_s < 1.0, first_s
    ref = oracle_c.groupby(cols, ['k'], aggs, oracle_c.where_terms(cols, terms))
    assert_tables_equal(first, ref)
    for c in first:  # generic and specialised kernels: the same bits
        assert first[c].tobytes() == second[c].tobytes(), c


def test_jit_wait_without_pending_compiles(gpu_device):
    w = gpu_device.jit_wait(0)
    assert w['idle'] and w['compiled'] >= 0 and w['failed'] >= 0
