"""The co-located merge's point-to-point schedules on the host (no GPU, no RCCL).

``bqueryd_amd/csrc/merge_schedule.h`` builds the message lists comm.hip posts as grouped
ncclSend / ncclRecv in the payload exchange and the gather to rank 0.  The RCCL branch has not
run at world > 1 on hardware (no multi-GPU box in this build's pool), so this test compiles the
same header with g++ and checks, for 400 random count matrices of 1-9 ranks and 1-6 columns,
that every (sender, receiver) pair's lists agree message for message in posting order with
equal byte counts -- RCCL's matching rule -- and that delivering them puts every element where
the receiver expects it (tests/merge_schedule_check.cpp)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_exchange_and_gather_schedules_match(tmp_path):
    cxx = shutil.which('g++')
    if cxx is None:
        pytest.skip('g++ not available')
    exe = str(tmp_path / 'merge_schedule_check')
    subprocess.check_call([cxx, '-O1', '-std=c++17', '-Wall', '-Werror', '-fsanitize=address,undefined',
                           os.path.join(HERE, 'merge_schedule_check.cpp'), '-o', exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == 'OK', out.stdout + out.stderr
