"""GPU: on-GPU blosc1 decode of bcolz carrays (bqg_table_load_carray_ex, decode='device').

The frames are written by the system c-blosc 1.x (bcolz_io.compress_chunk -> libblosc, the
library bcolz itself links); the device decoder's column must equal, byte for byte, the numpy
array the frames were made from -- the same check as the host path's (test_gpu_ingest.py) --
and the report must say which chunks ran where.  Codecs the kernels do not decode (zstd,
zlib) must come back through host libblosc, and corrupt streams must fail the call.
"""
import os
import struct
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import _lib, bcolz_io
from bqueryd_amd.engine import ShardTable

pytestmark = pytest.mark.gpu


def _array(dtype, n, seed, kind='random'):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if kind == 'runs':  # sorted, long runs: long LZ matches
        return np.sort(rng.integers(0, 50, n)).astype(dt)
    if kind == 'cents':  # taxi-like fares: shuffled high bytes compress, low bytes do not
        return np.round(np.clip(rng.lognormal(2.3, 0.6, n), 2.5, 500.0), 2).astype(dt)
    if dt.kind == 'b':
        return rng.random(n) < 0.3
    if dt.kind == 'f':
        return rng.normal(size=n).astype(dt)
    info = np.iinfo(dt)
    lo, hi = (0, min(1000, info.max // 4)) if kind == 'small' else (info.min, info.max)
    return rng.integers(lo, hi, n, dtype=dt, endpoint=True)


def _load(d, a, decode='device', nthreads=3):
    t = ShardTable(OrderedDict(), nrows=len(a))
    try:
        t.add_column('x', a.dtype)
        rep = t.load_carray('x', d, bcolz_io.CArrayMeta(d).chunklen, nthreads=nthreads, decode=decode)
        t.sync()
        got = t.read('x')
    finally:
        t.close()
    return got, rep


CASES = [('int32', 100_003, 4096, 'small'), ('float64', 77_777, 1000, 'random'), ('int8', 5, 2, 'random'),
         ('uint64', 65_536, 65_536, 'random'), ('bool', 12_345, 777, 'random'), ('int16', 1, 1024, 'random'),
         ('int64', 300_001, 131_072, 'runs'), ('float64', 250_000, 131_072, 'cents'),
         ('float32', 200_000, 50_000, 'cents'), ('uint16', 99_999, 33_333, 'small')]


@pytest.mark.parametrize('cname', ['lz4', 'blosclz', 'lz4hc'])
@pytest.mark.parametrize('shuffle', [1, 0])
@pytest.mark.parametrize('dtype,n,chunklen,kind', CASES)
def test_device_decode_matches(tmp_path, cname, shuffle, dtype, n, chunklen, kind):
    a = _array(dtype, n, n + shuffle, kind)
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=chunklen, cname=cname, shuffle=shuffle)
    got, rep = _load(d, a)
    np.testing.assert_array_equal(got, a)
    assert rep['decoder'] == _lib.DECODE_DEVICE
    assert rep['host_chunks'] == 0
    assert rep['chunks'] == -(-n // chunklen)
    assert rep['bytes'] == a.nbytes


@pytest.mark.parametrize('clevel', [1, 9])
def test_device_decode_clevels(tmp_path, clevel):
    a = _array('int64', 500_000, clevel, 'runs')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=200_000, clevel=clevel, cname='blosclz')
    got, _ = _load(d, a)
    np.testing.assert_array_equal(got, a)


def test_memcpyed_frames(tmp_path):
    """Incompressible bytes: blosc stores the frame as it is (flags bit 1)."""
    a = np.random.default_rng(5).integers(0, 256, 300_000, dtype=np.uint8)
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=70_000, cname='lz4', shuffle=0, clevel=9)
    with open(os.path.join(d, 'data', '__0.blp'), 'rb') as f:
        flags = f.read()[16 + 2]
    assert flags & 0x2, 'expected a memcpyed frame (flags %#x)' % flags
    got, rep = _load(d, a)
    np.testing.assert_array_equal(got, a)
    assert rep['host_chunks'] == 0


def test_unimplemented_flag_bit_goes_to_host(tmp_path):
    """A frame with header flag bit 0x8 set (reserved in c-blosc 1.x, the delta filter in later
    blosc) is not decoded on the device, where the filter would be silently skipped: it goes
    to host libblosc, which refuses it (1.21 here), so the call fails instead of returning
    wrong column data."""
    a = _array('int32', 50_000, 9, 'small')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=8192, cname='lz4')
    path = os.path.join(d, 'data', '__2.blp')
    with open(path, 'r+b') as f:
        f.seek(16 + 2)
        flags = f.read(1)[0]
        f.seek(16 + 2)
        f.write(bytes([flags | 0x8]))
    with pytest.raises(RuntimeError):
        _load(d, a)


@pytest.mark.parametrize('cname', ['zstd', 'zlib'])
def test_other_codecs_fall_back_to_host(tmp_path, cname):
    a = _array('int32', 50_000, 3, 'small')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=8192, cname=cname)
    got, rep = _load(d, a)
    np.testing.assert_array_equal(got, a)
    assert rep['decoder'] == _lib.DECODE_DEVICE
    assert rep['host_chunks'] == rep['chunks'] == 7


def test_mixed_codecs_in_one_carray(tmp_path):
    """Chunk files written with different codecs (a carray appended to under other cparams)."""
    a = _array('float64', 40_000, 4, 'cents')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=10_000, cname='lz4')
    other = bcolz_io.carray_files(a, chunklen=10_000, cname='zstd')
    for rel, data in other:
        if rel in ('data/__1.blp', 'data/__3.blp'):
            with open(os.path.join(d, rel), 'wb') as f:
                f.write(data)
    got, rep = _load(d, a)
    np.testing.assert_array_equal(got, a)
    assert rep['host_chunks'] == 2


def test_device_and_host_decoders_agree_multibatch(tmp_path):
    """More chunks than one 512 MiB batch: both staging slots and the batch loop run."""
    n = 80_000_000
    a = _array('int64', n, 9, 'small')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=1 << 20, cname='lz4')
    got, rep = _load(d, a, nthreads=8)
    np.testing.assert_array_equal(got, a)
    assert rep['chunks'] == -(-n // (1 << 20)) and rep['host_chunks'] == 0
    got_h, rep_h = _load(d, a, decode='host', nthreads=8)
    assert rep_h['decoder'] == _lib.DECODE_HOST
    np.testing.assert_array_equal(got_h, got)


def _first_split(frame):
    """(offset of the first split's int32 size in the frame, its size) of a non-memcpyed frame."""
    bstart = struct.unpack_from('<i', frame, 16)[0]
    return bstart, struct.unpack_from('<i', frame, bstart)[0]


@pytest.mark.parametrize('cname', ['lz4', 'blosclz'])
def test_corrupt_stream_fails(tmp_path, cname):
    a = _array('int64', 100_000, 1, 'runs')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=50_000, cname=cname)
    path = os.path.join(d, 'data', '__1.blp')
    with open(path, 'rb') as f:
        data = bytearray(f.read())
    off, csize = _first_split(bytes(data[16:]))
    assert 0 < csize < 100_000
    # a stream of 0xFF bytes: LZ4 literal lengths / BloscLZ matches that overrun the output
    data[16 + off + 4:16 + off + 4 + csize] = b'\xff' * csize
    with open(path, 'wb') as f:
        f.write(bytes(data))
    with pytest.raises(_lib.BqgError, match='corrupt'):
        _load(d, a)


def test_bad_split_size_fails(tmp_path):
    a = _array('int32', 30_000, 2, 'small')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=10_000, cname='lz4')
    path = os.path.join(d, 'data', '__2.blp')
    with open(path, 'rb') as f:
        data = bytearray(f.read())
    off, _ = _first_split(bytes(data[16:]))
    struct.pack_into('<i', data, 16 + off, 1 << 30)
    with open(path, 'wb') as f:
        f.write(bytes(data))
    with pytest.raises(_lib.BqgError, match='out of the frame'):
        _load(d, a)


def test_missing_chunk_and_magic(tmp_path):
    a = np.arange(10_000, dtype=np.int32)
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=1000)
    with open(os.path.join(d, 'data', '__3.blp'), 'r+b') as f:
        f.write(b'nope')
    with pytest.raises(_lib.BqgError, match='bloscpack'):
        _load(d, a)
    os.remove(os.path.join(d, 'data', '__3.blp'))
    with pytest.raises(_lib.BqgError, match='cannot open'):
        _load(d, a)


@pytest.mark.parametrize('decode', ['device', 'host'])
def test_load_carrays_several_columns(tmp_path, decode):
    """One call for several columns: batches span columns on the device path; every column
    and its report must come out as if loaded alone."""
    n = 3_000_000
    cols = OrderedDict([('a', _array('int32', n, 1, 'small')), ('b', _array('float64', n, 2, 'cents')),
                        ('c', _array('int8', n, 3, 'small')), ('d', _array('uint16', n, 4, 'runs'))])
    cnames = {'a': 'lz4', 'b': 'blosclz', 'c': 'zstd', 'd': 'lz4'}
    chunklens = {'a': 262_144, 'b': 100_000, 'c': 1 << 20, 'd': 77_777}
    t = ShardTable(OrderedDict(), nrows=n)
    try:
        specs = []
        for k, a in cols.items():
            d = str(tmp_path / k)
            bcolz_io.write_carray(d, a, chunklen=chunklens[k], cname=cnames[k])
            t.add_column(k, a.dtype)
            specs.append((k, d, chunklens[k]))
        reps = t.load_carrays(specs, nthreads=4, decode=decode)
        t.sync()
        for (k, a), rep in zip(cols.items(), reps):
            np.testing.assert_array_equal(t.read(k), a)
            assert rep['chunks'] == -(-n // chunklens[k]) and rep['bytes'] == a.nbytes
            if decode == 'device':
                assert rep['host_chunks'] == (rep['chunks'] if cnames[k] == 'zstd' else 0), (k, rep)
    finally:
        t.close()


def test_load_carrays_rejects_duplicates(tmp_path):
    a = np.arange(1000, dtype=np.int32)
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=100)
    t = ShardTable(OrderedDict(), nrows=len(a))
    try:
        t.add_column('x', a.dtype)
        with pytest.raises(_lib.BqgError, match='twice'):
            t.load_carrays([('x', d, 100), ('x', d, 100)], decode='device')
    finally:
        t.close()


@pytest.mark.parametrize('cname', ['lz4', 'blosclz'])
@pytest.mark.parametrize('period', [3_000, 20_000, 40_000, 60_000])
def test_far_matches(tmp_path, cname, period):
    """A random block repeated at distances past the LDS history (LZ4 / BloscLZ far offsets,
    BloscLZ's 16-bit distance escape beyond 8191): the matches read the output back from
    global memory."""
    rng = np.random.default_rng(period)
    block = rng.integers(0, 256, period, dtype=np.uint8)
    a = np.tile(block, 1_200_000 // period + 1)[:1_200_000]
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=1_200_000, cname=cname, shuffle=0, clevel=9)
    with open(os.path.join(d, 'data', '__0.blp'), 'rb') as f:
        flags = f.read()[16 + 2]
    got, rep = _load(d, a)
    np.testing.assert_array_equal(got, a)
    assert rep['host_chunks'] == 0, 'flags %#x' % flags


def test_long_literal_runs_and_short_matches(tmp_path):
    """Incompressible stretches (literal runs longer than a group sequence) between short
    repeats, in one stream."""
    rng = np.random.default_rng(77)
    parts = []
    for i in range(400):
        parts.append(rng.integers(0, 256, int(rng.integers(1, 700)), dtype=np.uint8))
        parts.append(np.full(int(rng.integers(4, 300)), i % 7, dtype=np.uint8))
    a = np.concatenate(parts)
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=len(a), cname='lz4', shuffle=0)
    got, _ = _load(d, a)
    np.testing.assert_array_equal(got, a)


@pytest.mark.parametrize('cname', ['lz4', 'blosclz'])
def test_fuzzed_streams_never_fault(tmp_path, cname):
    """Random byte flips inside the compressed streams (headers and block tables left intact):
    every load either decodes or fails with BqgError; the kernels never read or write outside
    their buffers (a fault would end the process)."""
    a = _array('int32', 400_000, 11, 'small')
    d = str(tmp_path / 'col')
    bcolz_io.write_carray(d, a, chunklen=100_000, cname=cname)
    path = os.path.join(d, 'data', '__1.blp')
    with open(path, 'rb') as f:
        orig = f.read()
    frame = orig[16:]
    first, _ = _first_split(frame)
    rng = np.random.default_rng(5)
    outcomes = {'ok': 0, 'error': 0}
    for trial in range(24):
        data = bytearray(orig)
        for _ in range(int(rng.integers(1, 40))):
            pos = 16 + first + 4 + int(rng.integers(0, len(frame) - first - 4))
            data[pos] = int(rng.integers(0, 256))
        with open(path, 'wb') as f:
            f.write(bytes(data))
        try:
            _load(d, a)
            outcomes['ok'] += 1
        except _lib.BqgError:
            outcomes['error'] += 1
    assert sum(outcomes.values()) == 24
    with open(path, 'wb') as f:
        f.write(orig)
    got, _ = _load(d, a)
    np.testing.assert_array_equal(got, a)
