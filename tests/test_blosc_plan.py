"""The bcolz chunk-file parser of the on-GPU decode (``bqueryd_amd/csrc/blosc_plan.h``,
``plan_chunk``) built on the host with ``-fsanitize=address,undefined`` (SURVEY §5 "race
detection / sanitizers").  It turns file bytes -- the chunks bqueryd's worker
opens at ``bqueryd/worker.py:291`` -- into the stream tasks the GPU decoder follows, so a
malformed file must be rejected, never read out of bounds or turned into a task that writes
outside its chunk.  ``tests/blosc_plan_check.cpp`` plans synthetic frames of every layout, every
truncation and random corruptions of them, garbage files, and frames the system libblosc wrote
(every codec the device decodes, shuffle on / off, memcpyed)."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from bqueryd_amd import bcolz_io

HERE = os.path.dirname(os.path.abspath(__file__))


def test_chunk_parser_under_asan_ubsan(tmp_path):
    cxx = shutil.which('g++')
    if cxx is None:
        pytest.skip('g++ not available')
    frames = []
    rng = np.random.default_rng(5)
    try:
        for i, (cname, dt, n, shuffle) in enumerate([('lz4', 'i4', 50_000, 1), ('blosclz', 'f8', 20_000, 1),
                                                     ('lz4', 'i8', 1000, 0), ('blosclz', 'u1', 70_000, 0),
                                                     ('lz4', 'u1', 9_000, 0), ('zstd', 'i2', 5_000, 1)]):
            a = (rng.integers(0, 1 << 20, n) if i != 4 else rng.integers(0, 256, n)).astype(dt)
            frame = bcolz_io.compress_chunk(a, 5, shuffle, cname)
            path = tmp_path / ('chunk%d.blp' % i)
            path.write_bytes(b'blpk' + bytes([3, 0, 0, 0]) + struct.pack('<q', 1) + bytes(frame))
            frames.append(str(path))
    except (OSError, RuntimeError) as e:  # no system libblosc: the synthetic frames still run
        frames = []
        print('libblosc frames skipped:', e)
    exe = str(tmp_path / 'blosc_plan_check')
    subprocess.check_call([cxx, '-O1', '-std=c++17', '-Wall', '-Werror', '-fsanitize=address,undefined',
                           '-fno-sanitize-recover=undefined', os.path.join(HERE, 'blosc_plan_check.cpp'), '-o', exe])
    out = subprocess.run([exe] + frames, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == 'OK', out.stdout + out.stderr[-3000:]
