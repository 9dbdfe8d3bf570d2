import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs libbqgpu kernels)')
    config.addinivalue_line('markers', 'slow: full-size (BASELINE) parity runs')


@pytest.fixture(scope='session')
def oracle_c():
    from oracle import cbquery
    cbquery.build()
    return cbquery


@pytest.fixture(scope='session')
def gpu_device():
    from bqueryd_amd.engine import get_device
    return get_device()


@pytest.fixture
def engine_options():
    """Set engine options (include/bqgpu.h, bqg_set_option) on the process's default context
    for one test; the defaults are restored afterwards."""
    from bqueryd_amd.engine import get_device
    dev = get_device()

    def set_options(**kw):
        # a test that asks for the specialised kernels wants them on its first query: compile
        # synchronously (the background path has its own test)
        if ('jit' in kw or 'jit_min_rows' in kw) and 'jit_async' not in kw:
            kw['jit_async'] = 0
        for k, v in kw.items():
            dev.set_option(k, v)
    yield set_options
    dev.reset_options()
