"""ctypes binding of libbrickrec.so (the C-ABI declared in include/brickrec.h).

The library is built in-tree (``make -C brickbrain-rec-engine_amd/csrc`` or
``__graft_entry__.build()``) and loaded from this directory.  There is no fallback: if the
library is missing or a call fails, a :class:`BrickrecError` is raised.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BRICKREC_LIB", os.path.join(HERE, "libbrickrec.so"))

BB_F32, BB_BF16, BB_F64 = 0, 1, 2
BB_HOST, BB_DEVICE = 0, 1
BB_MODE_SEMANTIC, BB_MODE_SIMILAR, BB_MODE_CF, BB_MODE_HYBRID = 0, 1, 2, 3
BB_Q_OUT_KEYS = 1
BB_Q_NULL_STREAM = 2
BB_OPT_STREAM, BB_OPT_STREAM_MIN_ITEMS, BB_OPT_WORKSPACE_BYTES, BB_OPT_STREAM_REFINE, BB_OPT_RR_LISTS = 1, 2, 3, 4, 5
BB_OPT_SMALL_BATCH, BB_OPT_PREFILTER = 6, 7
ABI_VERSION = 2   # include/brickrec.h BB_ABI_VERSION (2: bb_query.mask_count)
BB_OK, BB_E_ARG, BB_E_HIP, BB_E_STATE, BB_E_NOMEM, BB_E_HOSTSYNC = 0, -1, -2, -3, -4, -5

# every entry point include/brickrec.h declares (checked by tests/test_abi.py)
EXPORTS = ("bb_create", "bb_upload_items", "bb_upload_cf", "bb_upload_attrs", "bb_eval_mask",
           "bb_search", "bb_key_lens", "bb_finalize", "bb_set_profiling", "bb_get_profile", "bb_set_option",
           "bb_info", "bb_get_rows", "bb_create_view", "bb_destroy", "bb_last_error", "bb_abi_version",
           "bb_plan_create", "bb_plan_launch", "bb_plan_destroy", "bb_check_dual_scan_args")


class BrickrecError(RuntimeError):
    """A libbrickrec call failed (or the library is missing)."""


class bb_desc(C.Structure):
    _fields_ = [("device", C.c_int32), ("dtype", C.c_int32), ("id_offset", C.c_int64),
                ("workspace_bytes", C.c_int64)]


class bb_predicate(C.Structure):
    _fields_ = [("parts_min", C.c_int32), ("parts_max", C.c_int32), ("year_min", C.c_int32),
                ("year_max", C.c_int32), ("theme_mode", C.c_int32), ("n_theme_bits", C.c_int32),
                ("theme_bits", C.c_void_p), ("excluded_items", C.c_void_p),
                ("n_excluded", C.c_int64)]


class bb_query(C.Structure):
    _fields_ = [("mode", C.c_int32), ("flags", C.c_int32), ("B", C.c_int32), ("k", C.c_int32),
                ("k_side", C.c_int32), ("where", C.c_int32),
                ("q_rows", C.c_void_p), ("q_dtype", C.c_int32),
                ("q_items", C.c_void_p),
                ("q_cf", C.c_void_p), ("q_cf_dtype", C.c_int32),
                ("mask_bits", C.c_void_p), ("excl_bits", C.c_void_p),
                ("w_content", C.c_double), ("w_cf", C.c_double),
                ("stream", C.c_void_p), ("mask_count", C.c_int64)]


class bb_result(C.Structure):
    _fields_ = [("scores", C.c_void_p), ("ids", C.c_void_p), ("counts", C.c_void_p),
                ("where", C.c_int32), ("keys", C.c_void_p), ("max_keys", C.c_void_p)]


class bb_profile(C.Structure):
    _fields_ = [("ms", C.c_double * 8), ("launches", C.c_int64 * 8),
                ("names", C.c_char_p * 8), ("n", C.c_int32)]


_lock = threading.Lock()
_lib = None


def load() -> C.CDLL:
    """Load libbrickrec.so once; raise BrickrecError if it is not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise BrickrecError(
                f"libbrickrec.so not found at {LIB_PATH}; build it with "
                "`make -C brickbrain-rec-engine_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = C.CDLL(LIB_PATH)
        P = C.c_void_p
        sig = {
            "bb_create": ([C.POINTER(bb_desc), C.POINTER(P)], C.c_int),
            "bb_upload_items": ([P, P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P], C.c_int),
            "bb_upload_cf": ([P, P, C.c_int32, C.c_int32, P], C.c_int),
            "bb_upload_attrs": ([P, P, P, P], C.c_int),
            "bb_eval_mask": ([P, C.POINTER(bb_predicate), P, C.c_int32], C.c_int),
            "bb_search": ([P, C.POINTER(bb_query), C.POINTER(bb_result)], C.c_int),
            "bb_key_lens": ([C.POINTER(bb_query), C.POINTER(C.c_int32), C.POINTER(C.c_int32)], C.c_int),
            "bb_finalize": ([P, C.POINTER(bb_query), P, P, C.c_int32, C.POINTER(bb_result)], C.c_int),
            "bb_set_profiling": ([P, C.c_int32], C.c_int),
            "bb_get_profile": ([P, C.POINTER(bb_profile)], C.c_int),
            "bb_set_option": ([P, C.c_int32, C.c_int64], C.c_int),
            "bb_info": ([P, C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                         C.POINTER(C.c_int32)], C.c_int),
            "bb_get_rows": ([P, P, C.c_int32, P, C.c_int32], C.c_int),
            "bb_create_view": ([P, C.POINTER(P)], C.c_int),
            "bb_destroy": ([P], C.c_int),
            "bb_plan_create": ([P, C.POINTER(bb_query), C.POINTER(bb_result), C.POINTER(P)], C.c_int),
            "bb_plan_launch": ([P], C.c_int),
            "bb_plan_destroy": ([P], C.c_int),
            "bb_check_dual_scan_args": ([C.c_int64], C.c_int),
            "bb_last_error": ([], C.c_char_p),
            "bb_abi_version": ([], C.c_int),
        }
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.bb_abi_version() != ABI_VERSION:
            raise BrickrecError(f"libbrickrec ABI {lib.bb_abi_version()} != {ABI_VERSION}")
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().bb_last_error().decode(errors="replace")
        raise BrickrecError(f"{what} failed ({rc}): {msg}")
