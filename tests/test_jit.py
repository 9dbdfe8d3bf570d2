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


C4_SPEC = (b"#define BQ_NC 2\n#define BQ_SPEC p.ncols=2;"
           b"p.cols[0].dtype=3;p.cols[0].lg=2;p.cols[1].dtype=3;p.cols[1].lg=2;"
           b"p.nterms=0;p.nkeys=1;p.keys[0].col=0;p.keys[0].is_float=0;p.keys[0].stride=1ull;"
           b"p.nsum=0;p.mask_col=-1;p.hash=0;\n"
           b"#define BQ_SCD_CD 1\n#define BQ_SCD_VC 1\n#define BQ_SCD_CC 1\n#define BQ_SCD_P16 1\n")


@pytest.mark.parametrize('extra', [b'', b'#define BQ_PART_K 4\n#define BQ_PART_NARROW 1\n#define BQ_PART_PACK 1\n',
                                   b'#define BQ_PART_K 2\n#define BQ_PART_NARROW 1\n#define BQ_PART_PACK 0\n'])
def test_specialised_distinct_and_partition_kernels_compile(extra):
    """Every JIT entry point (the fused distinct pass in both loops, the partition scatter with
    packed / narrow entries and 16384-row tiles) compiles for a C4-shaped query."""
    f = _lib.lib().bqg_internal_jit_compile_check
    f.argtypes = [ctypes.c_char_p]
    f.restype = ctypes.c_int
    rc = f(C4_SPEC + extra)
    if rc == 1:
        pytest.skip('hiprtc not loadable here')
    assert rc == 0
