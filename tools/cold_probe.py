"""Where a cold first query's time goes (round 6): a fresh process and context, the C2 shard,
then the first queries with the run-time compile cache empty.  Prints one JSON object."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ['BQGPU_JIT_CACHE'] = tempfile.mkdtemp(prefix='bqgpu-cold-probe-')

from bqueryd_amd import synth  # noqa: E402
from bqueryd_amd.engine import Device, ShardTable  # noqa: E402

out = {}
t0 = time.perf_counter()
dev = Device(0)
out['context_ms'] = 1e3 * (time.perf_counter() - t0)
dev.set_option('compact', 0)
config = sys.argv[1] if len(sys.argv) > 1 else 'c2'
cfg = synth.CONFIGS[config]
rows = int(sys.argv[2]) if len(sys.argv) > 2 else cfg['rows']
cols = synth.taxi_shard(rows, config_id=synth.CONFIG_ID[config], columns=synth.query_columns(cfg))
t0 = time.perf_counter()
table = ShardTable(cols, device=dev)
dev.synchronize()
out['table_ms'] = 1e3 * (time.perf_counter() - t0)


def q(aggs, where):
    dev.enable_timing(True)
    dev.synchronize()
    t = time.perf_counter()
    table.groupby(cfg['groupby'], aggs, where_terms=where)
    dev.synchronize()
    wall = 1e3 * (time.perf_counter() - t)
    tm = dev.last_timing()
    dev.enable_timing(False)
    return {'wall_ms': wall, 'device_ms': tm['total_ms'], 'scan_ms': tm['scan_ms'], 'spec': tm['specialized']}


out['first'] = q(cfg['aggs'], cfg['where'])
out['second'] = q(cfg['aggs'], cfg['where'])
out['third'] = q(cfg['aggs'], cfg['where'])
# another shape on the same table: what is per shape, not per process
if config == 'c2':
    out['other_shape_first'] = q([['fare_amount', 'sum', 's']], [('passenger_count', '>', 3)])
    out['other_shape_second'] = q([['fare_amount', 'sum', 's']], [('passenger_count', '>', 3)])
out['jit_wait'] = dev.jit_wait(600)
out['after_compile'] = q(cfg['aggs'], cfg['where'])
print(json.dumps(out))
