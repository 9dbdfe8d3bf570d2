"""The cross-rank merge on the GPU: RCCL (nccl backend) exchange + libbqgpu partition/reduce,
run in a torch.distributed.run child process (one rank per visible GPU, at most 2)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_merge_matches_client_merge():
    from bqueryd_amd.engine import device_count
    n = max(1, min(2, device_count()))
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(ROOT, 'tools', 'dist_check.py')]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert 'ok=True' in p.stdout


def test_rccl_merge_two_ranks_on_one_gpu():
    """The RCCL branch at world 2 on a one-GPU box: both ranks on GPU 0, each claiming a host
    of its own (NCCL_HOSTID) so that RCCL connects them over its socket transport -- the
    grouped send / recv and all-gather calls of the merge, and the message schedule both sides
    derive, executed by RCCL itself against the reference client merge (rpc.py:164-173)."""
    env = dict(os.environ, BQGPU_DIST_ONE_GPU='1')
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(ROOT, 'tools', 'dist_check.py')]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert 'dist_check world=2' in p.stdout and 'ok=True' in p.stdout, p.stdout[-2000:]
