"""bqueryd_amd -- MI355X-native engine for bqueryd's per-shard groupby calc path.

Drop-in for the block of ``WorkerNode.handle_work`` that calls bquery
(``bqueryd/worker.py:291-323``): columns of a shard live in HBM (``ShardTable``), and
where-terms, key factorisation, hash aggregation and emit run as hand-written gfx950 kernels
in ``libbqgpu.so`` (C ABI: ``include/bqgpu.h``).
"""
from .engine import Device, ShardTable, device_count, get_device  # noqa: F401

__version__ = '0.1.0'
