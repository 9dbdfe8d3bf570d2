"""C4 fused-distinct-pass variants in one process (BQGPU_JIT_DEFS read per query by libbqgpu),
timed with the library's HIP events."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bqueryd_amd import synth  # noqa: E402
from bqueryd_amd.engine import Device, ShardTable  # noqa: E402

cfg = synth.CONFIGS['c4']
cols = synth.taxi_shard(cfg['rows'], config_id=4, columns=synth.query_columns(cfg))
dev = Device(0)
t = ShardTable(cols, device=dev)
dev.enable_timing(True)
print('loaded', flush=True)
ref = None
for defs in ('', 'BQ_SCD_PEEL=1', 'BQ_SCD_PEEL=2', 'BQ_SCD_PEEL=3', ''):
    if defs:
        os.environ['BQGPU_JIT_DEFS'] = defs
    else:
        os.environ.pop('BQGPU_JIT_DEFS', None)
    ks = []
    for i in range(8):
        out, _ = t.groupby(cfg['groupby'], cfg['aggs'], where_terms=cfg['where'])
        ks.append(dev.last_timing()['scan_ms'])
    if ref is None:
        ref = out
    same = all(np.array_equal(np.asarray(ref[k]), np.asarray(out[k])) for k in ref)
    print('%-16s scan_ms median %.4f min %.4f identical=%s' % (defs or 'default', np.median(ks[2:]), min(ks[2:]), same),
          flush=True)
