"""The run-time specialiser compiles on the host (hiprtc, no GPU needed)."""
import ctypes

import pytest

from bqueryd_amd import _lib

C2_SPEC = (b"#define BQ_NC 3\n#define BQ_SPEC p.ncols=3;"
           b"p.cols[0].dtype=10;p.cols[0].lg=3;p.cols[1].dtype=3;p.cols[1].lg=2;p.cols[2].dtype=3;p.cols[2].lg=2;"
           b"p.nterms=1;p.terms[0].col=2;p.terms[0].op=6;p.terms[0].is_float=0;"
           b"p.nkeys=1;p.keys[0].col=1;p.keys[0].is_float=0;p.keys[0].stride=1ull;"
           b"p.nsum=1;p.sum_is_float[0]=1;p.sum_conv[0]=0;p.sum_centered[0]=0;p.mask_col=-1;p.hash=0;\n")


def test_specialised_scan_compiles():
    f = _lib.lib().bqg_internal_jit_compile_check
    f.argtypes = [ctypes.c_char_p]
    f.restype = ctypes.c_int
    rc = f(C2_SPEC)
    if rc == 1:
        pytest.skip('hiprtc not loadable here')
    assert rc == 0
