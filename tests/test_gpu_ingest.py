"""GPU: cold-path ingest (bqg_table_load_carray) -- bcolz carrays decoded on host threads or
on the GPU straight into HBM, compared byte for byte with the numpy columns they were written from."""
import os
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import _lib, bcolz_io, synth
from bqueryd_amd.ctable import ctable
from bqueryd_amd.engine import ShardTable
from oracle import bquery_oracle as bo
from tests.helpers import assert_tables_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('decode', ['host', 'device'])
@pytest.mark.parametrize('cname', ['lz4', 'blosclz', 'zstd', 'zlib'])
@pytest.mark.parametrize('dtype,n,chunklen', [('int32', 100_003, 4096), ('float64', 77_777, 1000),
                                              ('int8', 5, 2), ('uint64', 65_536, 65_536),
                                              ('bool', 12_345, 777), ('int16', 1, 1024)])
def test_load_carray_roundtrip(tmp_path, cname, dtype, n, chunklen, decode):
    rng = np.random.default_rng(n)
    if dtype == 'bool':
        a = rng.random(n) < 0.3
    elif dtype.startswith('float'):
        a = rng.normal(size=n).astype(dtype)
    else:
        info = np.iinfo(dtype)
        a = rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True)
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=chunklen, cname=cname)
    t = ShardTable(OrderedDict(), nrows=n)
    try:
        t.add_column('x', a.dtype)
        t.load_carray('x', d, bcolz_io.CArrayMeta(d).chunklen, nthreads=3, decode=decode)
        t.sync()
        got = t.read('x')
    finally:
        t.close()
    np.testing.assert_array_equal(got, a)


@pytest.mark.parametrize('decode', ['host', 'device'])
def test_load_carray_errors(tmp_path, decode):
    a = np.arange(10_000, dtype=np.int32)
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=1000)
    t = ShardTable(OrderedDict(), nrows=len(a))
    try:
        t.add_column('x', np.int32)
        with open(os.path.join(d, 'data', '__3.blp'), 'r+b') as f:
            f.write(b'nope')  # bad bloscpack magic
        with pytest.raises(_lib.BqgError, match='bloscpack'):
            t.load_carray('x', d, 1000, decode=decode)
        os.remove(os.path.join(d, 'data', '__3.blp'))
        with pytest.raises(_lib.BqgError, match='cannot open'):
            t.load_carray('x', d, 1000, decode=decode)
    finally:
        t.close()


def test_ctable_cold_open_matches_oracle(tmp_path):
    """bquery.ctable(rootdir) -> where_terms -> groupby with every column ingested natively."""
    cfg = synth.CONFIGS['c2']
    cols = synth.taxi_shard(300_000, config_id=2, columns=synth.query_columns(cfg))
    root = str(tmp_path / 'shard.bcolzs')
    bcolz_io.write_ctable(root, cols, chunklen=32_768)
    ct = ctable(rootdir=root, mode='r', auto_cache=True)
    try:
        bool_arr = ct.where_terms(cfg['where'], cache=True)
        got = ct.groupby(cfg['groupby'], cfg['aggs'], bool_arr=bool_arr).columns
        assert not ct._host, 'columns must not be decoded through the host path'
    finally:
        ct.close()
    ref = bo.handle_work(cols, cfg['groupby'], cfg['aggs'], cfg['where'])
    assert_tables_equal(got, ref)
