#!/usr/bin/env python3
"""Blosc frames of the C2 shard's columns for tools/micro/blosc_micro.hip: <col>.lz4 and
<col>.blz (one chunk each, raw blosc1 frames, LZ4 / BloscLZ) and <col>.<ext>.expect (the decoded, still byte-shuffled block bytes the
decode kernel must produce before the un-shuffle)."""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from bqueryd_amd import bcolz_io, synth  # noqa: E402


def main():
    out_dir = os.path.join(HERE, 'frames')
    os.makedirs(out_dir, exist_ok=True)
    cfg = synth.CONFIGS['c2']
    cols = synth.taxi_shard(1_000_000, config_id=2, columns=synth.query_columns(cfg))
    for name, a in cols.items():
        x = np.ascontiguousarray(a[:(1 << 20) // a.itemsize])
        for cname, ext in (('lz4', '.lz4'), ('blosclz', '.blz')):
            f = bcolz_io.compress_chunk(x, 5, 1, cname)
            ts = f[3]
            nbytes, bs, _ = struct.unpack_from('<iii', f, 4)
            raw = x.view(np.uint8)
            exp = bytearray()
            for b0 in range(0, nbytes, bs):
                blk = raw[b0:b0 + bs]
                n = len(blk) // ts
                exp += blk[:n * ts].reshape(n, ts).T.tobytes() + blk[n * ts:].tobytes()
            with open(os.path.join(out_dir, name + ext), 'wb') as fh:
                fh.write(f)
            with open(os.path.join(out_dir, name + ext + '.expect'), 'wb') as fh:
                fh.write(bytes(exp))


if __name__ == '__main__':
    main()
