"""CPU: the blosc1 frame layout the on-GPU decoder's planner assumes (ingest.hip plan_chunk).

c-blosc is not vendored (only its shared library is installed), so the layout rule --
block start table, `typesize` splits per full block when typesize <= 16, blocksize /
typesize >= 128 and flags bit 4 is clear, else one; each split an int32 size + stream -- is
pinned here against frames the system libblosc writes: walking the splits by that rule must
land exactly on the next block's start (and the last block on cbytes) for every codec, type
size, shuffle mode and compression level bcolz can use.
"""
import struct

import numpy as np
import pytest

from bqueryd_amd import bcolz_io


def walk(frame):
    flags, ts = frame[2], frame[3]
    nbytes, bs, cbytes = struct.unpack_from('<iii', frame, 4)
    if flags & 0x2:
        assert cbytes == 16 + nbytes
        return 'memcpyed'
    nblocks = -(-nbytes // bs)
    left = nbytes % bs
    starts = [struct.unpack_from('<i', frame, 16 + 4 * b)[0] for b in range(nblocks)]
    for b in range(nblocks):
        partial = b == nblocks - 1 and left
        nsplits = ts if (not flags & 0x10 and ts <= 16 and bs // ts >= 128 and not partial) else 1
        p = starts[b]
        for _ in range(nsplits):
            csize = struct.unpack_from('<i', frame, p)[0]
            assert 0 <= csize
            p += 4 + csize
        assert p == (starts[b + 1] if b + 1 < nblocks else cbytes)
    return flags >> 5


@pytest.mark.parametrize('cname,code', [('blosclz', 0), ('lz4', 1), ('lz4hc', 1), ('zlib', 3), ('zstd', 4)])
def test_split_rule_tiles_every_frame(cname, code):
    rng = np.random.default_rng(7)
    for dt in ['?', 'i1', 'i2', 'i4', 'i8', 'f4', 'f8', 'u8']:
        for n in [1, 5, 1000, 77_777]:
            for clevel in [1, 5, 9]:
                for shuffle in [0, 1]:
                    a = rng.integers(0, 100, n).astype(dt)
                    got = walk(bcolz_io.compress_chunk(a, clevel, shuffle, cname))
                    assert got in (code, 'memcpyed')


def test_incompressible_is_memcpyed():
    a = np.random.default_rng(1).integers(0, 256, 100_000, dtype=np.uint8)
    assert walk(bcolz_io.compress_chunk(a, 9, 0, 'lz4')) == 'memcpyed'
