"""C3 launch-shape sweep in one process: scatter threads x workgroups per CU (env knobs read per
query by libbqgpu), timing the partitioned kernels with the library's HIP events."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bqueryd_amd import synth  # noqa: E402
from bqueryd_amd.engine import Device, ShardTable  # noqa: E402

cfg = synth.CONFIGS['c3']
cols = synth.taxi_shard(100_000_000, config_id=3, columns=synth.query_columns(cfg))
dev = Device(0)
t = ShardTable(cols, device=dev)
dev.enable_timing(True)
print('loaded', flush=True)
for threads, per_cu, chunks in (('1024', '2', '1'), ('1024', '1', '2'), ('1024', '2', '2'), ('512', '2', '2'),
                                ('512', '4', '2'), ('1024', '2', '1')):
    os.environ['BQGPU_PART_THREADS'] = threads
    os.environ['BQGPU_PART_PER_CU'] = per_cu
    os.environ['BQGPU_PART_CHUNKS'] = chunks
    ks = []
    for i in range(8):
        t.groupby(cfg['groupby'], cfg['aggs'], where_terms=cfg['where'])
        ks.append(dev.last_timing()['scan_ms'])
    print('threads=%s per_cu=%s chunks=%s scan_ms median %.4f min %.4f' % (threads, per_cu, chunks, np.median(ks[2:]), min(ks[2:])),
          flush=True)
