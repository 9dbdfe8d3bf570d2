"""ctypes binding of libbqgpu (include/bqgpu.h).

The library is built in-tree (``bqueryd_amd/libbqgpu.so``) by ``__graft_entry__.build()`` /
``make -C bqueryd_amd/csrc``.  There is no fallback: if the shared object is missing or the
HIP runtime cannot create a device context, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libbqgpu.so')

# enum bqg_dtype
DTYPES = [np.dtype(np.bool_), np.dtype(np.int8), np.dtype(np.int16), np.dtype(np.int32),
          np.dtype(np.int64), np.dtype(np.uint8), np.dtype(np.uint16), np.dtype(np.uint32),
          np.dtype(np.uint64), np.dtype(np.float32), np.dtype(np.float64)]
DTYPE_CODE = {dt: i for i, dt in enumerate(DTYPES)}
BOOL = 0

# enum bqg_agg_op
AGG_CODE = {'sum': 0, 'count': 1, 'count_distinct': 2, 'sorted_count_distinct': 3, 'mean': 4,
            'std': 5}
# enum bqg_term_op
T_FALSE, T_TRUE, T_EQ, T_NE, T_IN, T_NIN, T_GT, T_GE, T_LT, T_LE = -1, 0, 1, 2, 3, 4, 5, 6, 7, 8

E_INVALID, E_UNSUPPORTED, E_HIP, E_OOM, E_STATE = -1, -2, -3, -4, -5
UNIQUE_ID_BYTES = 128
ABI_VERSION = 10
OPTIONS = ('jit', 'jit_min_rows', 'partition', 'part_wbits', 'part_k', 'part_threads', 'part_per_cu',
           'part_splits', 'part_narrow', 'fused_scd', 'scd_compact', 'scd_pack16', 'priv_ahead',
           'private_per_cu', 'small_emit', 'hash_slots', 'distinct_slots', 'part_pack', 'scd_runs', 'part_win', 'compact', 'part_first',
           'fx_sums', 'mem_cap_mb', 'part_ring', 'jit_async', 'warm', 'slot_emit')


class Term(ctypes.Structure):
    _fields_ = [('col', ctypes.c_int32), ('op', ctypes.c_int32), ('nvals', ctypes.c_int64),
                ('ivals', ctypes.c_void_p), ('fvals', ctypes.c_void_p)]


class Agg(ctypes.Structure):
    _fields_ = [('col', ctypes.c_int32), ('op', ctypes.c_int32)]


class Query(ctypes.Structure):
    _fields_ = [('n_keys', ctypes.c_int32), ('key_cols', ctypes.c_void_p),
                ('n_terms', ctypes.c_int32), ('terms', ctypes.c_void_p),
                ('mask_col', ctypes.c_int32),
                ('n_aggs', ctypes.c_int32), ('aggs', ctypes.c_void_p)]


class ResultView(ctypes.Structure):
    _fields_ = [('n_rows', ctypes.c_int64), ('n_cols', ctypes.c_int32),
                ('dtypes', ctypes.POINTER(ctypes.c_int32)),
                ('cols', ctypes.POINTER(ctypes.c_void_p)), ('filtered', ctypes.c_int32)]


class Timing(ctypes.Structure):
    _fields_ = [('scan_ms', ctypes.c_double), ('scan_launches', ctypes.c_int32),
                ('total_ms', ctypes.c_double), ('rows', ctypes.c_int64),
                ('bytes', ctypes.c_int64), ('mode', ctypes.c_int32), ('specialized', ctypes.c_int32),
                ('narrow', ctypes.c_int32), ('regrows', ctypes.c_int32),
                ('bytes_read', ctypes.c_int64), ('compact_ms', ctypes.c_double),
                ('scan_ms_sum', ctypes.c_double), ('timed_queries', ctypes.c_int64),
                ('copy_ms', ctypes.c_double)]


# enum bqg_decode
DECODE_AUTO, DECODE_HOST, DECODE_DEVICE = 0, 1, 2
DECODE_CODE = {'auto': DECODE_AUTO, 'host': DECODE_HOST, 'device': DECODE_DEVICE}


class IngestStats(ctypes.Structure):
    _fields_ = [('chunks', ctypes.c_int64), ('compressed_bytes', ctypes.c_int64), ('bytes', ctypes.c_int64),
                ('device_splits', ctypes.c_int64), ('host_chunks', ctypes.c_int64), ('decoder', ctypes.c_int32)]


class BqgError(RuntimeError):
    pass


class BqgUnsupported(NotImplementedError):
    pass


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_PROTOS = {
    'bqg_abi_version': ([], ctypes.c_int),
    'bqg_device_count': ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    'bqg_create': ([ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_destroy': ([_P], ctypes.c_int),
    'bqg_last_error': ([_P], ctypes.c_char_p),
    'bqg_set_stream': ([_P, _P], ctypes.c_int),
    'bqg_synchronize': ([_P], ctypes.c_int),
    'bqg_enable_timing': ([_P, ctypes.c_int], ctypes.c_int),
    'bqg_last_timing': ([_P, ctypes.POINTER(Timing)], ctypes.c_int),
    'bqg_set_option': ([_P, ctypes.c_char_p, _I64], ctypes.c_int),
    'bqg_get_option': ([_P, ctypes.c_char_p, ctypes.POINTER(_I64)], ctypes.c_int),
    'bqg_reset_options': ([_P], ctypes.c_int),
    'bqg_alloc_pinned': ([_P, ctypes.c_size_t, ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_free_pinned': ([_P, _P], ctypes.c_int),
    'bqg_table_create': ([_P, _I64, _I32, _P, ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_table_destroy': ([_P], ctypes.c_int),
    'bqg_table_add_column': ([_P, _I32, ctypes.POINTER(_I32)], ctypes.c_int),
    'bqg_push_chunk': ([_P, _I32, _P, _I64, _I64], ctypes.c_int),
    'bqg_table_load_carray': ([_P, _I32, ctypes.c_char_p, _I64, _I32], ctypes.c_int),
    'bqg_table_load_carray_ex': ([_P, _I32, ctypes.c_char_p, _I64, _I32, _I32, _P], ctypes.c_int),
    'bqg_table_load_carrays': ([_P, _I32, _P, _P, _P, _I32, _I32, _P], ctypes.c_int),
    'bqg_table_sync': ([_P], ctypes.c_int),
    'bqg_table_column_ptr': ([_P, _I32, ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_table_stats': ([_P, _I32, ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                         ctypes.POINTER(_I32)], ctypes.c_int),
    'bqg_table_read': ([_P, _I32, _P, _I64, _I64], ctypes.c_int),
    'bqg_where': ([_P, _P, _I32, _P, _I32, ctypes.POINTER(_I64)], ctypes.c_int),
    'bqg_expand_subgroups': ([_P, _P, _I32, _I32, _I32], ctypes.c_int),
    'bqg_groupby': ([_P, _P, ctypes.POINTER(Query), ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_select_rows': ([_P, _P, ctypes.POINTER(Query), _I32, _P, ctypes.POINTER(_P)],
                        ctypes.c_int),
    'bqg_groupby_table': ([_P, _P, ctypes.POINTER(Query), ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_select_rows_table': ([_P, _P, ctypes.POINTER(Query), _I32, _P, ctypes.POINTER(_P)],
                              ctypes.c_int),
    'bqg_table_nrows': ([_P, ctypes.POINTER(_I64)], ctypes.c_int),
    'bqg_table_device_bytes': ([_P, ctypes.POINTER(_I64)], ctypes.c_int),
    'bqg_table_build_compact': ([_P, _I32, _P, ctypes.POINTER(_I32)], ctypes.c_int),
    'bqg_table_drop_compact': ([_P], ctypes.c_int),
    'bqg_table_ncols': ([_P, ctypes.POINTER(_I32)], ctypes.c_int),
    'bqg_table_dtype': ([_P, _I32, ctypes.POINTER(_I32)], ctypes.c_int),
    'bqg_comm_unique_id': ([_P], ctypes.c_int),
    'bqg_comm_init': ([_P, _I32, _I32, _P], ctypes.c_int),
    'bqg_comm_init_all': ([_I32, _P], ctypes.c_int),
    'bqg_comm_init_local': ([_I32, _P], ctypes.c_int),
    'bqg_comm_destroy': ([_P], ctypes.c_int),
    'bqg_comm_info': ([_P, ctypes.POINTER(_I32), ctypes.POINTER(_I32)], ctypes.c_int),
    'bqg_comm_last_phases': ([_P, ctypes.POINTER(ctypes.c_double), _I32], ctypes.c_int),
    'bqg_jit_wait': ([_P, ctypes.c_double, ctypes.POINTER(_I32), ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
                     ctypes.c_int),
    'bqg_comm_progress': ([_P, ctypes.POINTER(_I32), ctypes.POINTER(_I64), ctypes.POINTER(_I64)], ctypes.c_int),
    'bqg_merge': ([_P, _I32, _P, _I32, _I32, _P, _I32, ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_merge_group': ([_I32, _P, _P, _P, _I32, _I32, _P, _I32, _P], ctypes.c_int),
    'bqg_merge_host': ([_P, _I32, _P, _I32, _I32, _P, _I32, ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_merge_shared_host': ([_P, _I32, _P, _I32, _I32, _P, _I32, _P, _I64, ctypes.POINTER(_I64)], ctypes.c_int),
    'bqg_merge_group_host': ([_I32, _P, _P, _P, _I32, _I32, _P, _I32, ctypes.POINTER(_P)], ctypes.c_int),
    'bqg_result_view_get': ([_P, ctypes.POINTER(ResultView)], ctypes.c_int),
    'bqg_hash_partition': ([_P, _P, _I32, _P, _I32, _I32, _P], ctypes.c_int),
    'bqg_result_free': ([_P], ctypes.c_int),
    'bqg_factorize': ([_P, _P, _I32, _P, _P, _I64, ctypes.POINTER(_I64)], ctypes.c_int),
    'bqg_encode_bytes': ([_P, _P, _I32, _P, _I32, _P, _I64, ctypes.POINTER(_I64)], ctypes.c_int),
}

_lib = None


def lib():
    """Load libbqgpu.so (raises OSError when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError('libbqgpu.so is not built (%s); run __graft_entry__.build() or '
                          'make -C bqueryd_amd/csrc' % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _PROTOS.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        if L.bqg_abi_version() != ABI_VERSION:
            raise OSError('%s has ABI %d, this binding expects %d (rebuild it)' % (LIB_PATH, L.bqg_abi_version(),
                                                                                   ABI_VERSION))
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc == 0:
        return
    msg = lib().bqg_last_error(ctx)
    msg = msg.decode('utf-8', 'replace') if msg else 'error %d' % rc
    if rc == E_UNSUPPORTED:
        raise BqgUnsupported(msg)
    if rc == E_INVALID:
        raise BqgError(msg)
    raise BqgError(msg)
