"""ctypes binding of libstc.so (the C ABI in include/stc.h).

This is the Python stand-in for the JNI shim a Spark deployment would use:
every call crosses the same C boundary.  There is deliberately NO fallback: if the HIP library
is missing or no GPU is visible, the product path raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# STC_LIB selects an alternative build of the same library (e.g. the in-kernel stamp diagnostic
# build tools/stamp_estep.py uses); default: the in-tree libstc.so
LIB_PATH = os.environ.get("STC_LIB") or os.path.join(_HERE, "libstc.so")

STC_OK, STC_ERR_INVALID_ARG, STC_ERR_HIP, STC_ERR_RCCL, STC_ERR_OOM, STC_ERR_STATE = range(6)
STC_HASH_STANDARD, STC_HASH_SPARK24 = 0, 1
STC_F32, STC_F64, STC_MIXED = 0, 1, 2  # (STC_MIXED: an LDA dtype; its corpus CSR is STC_F64)


def corpus_dtype(lda_dtype):
    """the CSR value dtype an LDA handle of `lda_dtype` reads (STC_MIXED: fp64)"""
    return STC_F64 if lda_dtype == STC_MIXED else lda_dtype
STC_LAYOUT_VK, STC_LAYOUT_KV = 0, 1
STC_TRANSPORT_NONE, STC_TRANSPORT_IN_PROCESS, STC_TRANSPORT_RCCL = 0, 1, 2

_i32, _i64, _u64, _dbl, _int = C.c_int32, C.c_int64, C.c_uint64, C.c_double, C.c_int
_p = C.c_void_p
_pi32 = C.POINTER(C.c_int32)
_pi64 = C.POINTER(C.c_int64)
_pdbl = C.POINTER(C.c_double)
_pu8 = C.POINTER(C.c_uint8)


class LdaConfig(C.Structure):
    _fields_ = [
        ("k", _i32),
        ("vocab_size", _i64),
        ("doc_concentration", _pdbl),
        ("doc_concentration_len", _i32),
        ("topic_concentration", _dbl),
        ("tau0", _dbl),
        ("kappa", _dbl),
        ("mini_batch_fraction", _dbl),
        ("gamma_shape", _dbl),
        ("optimize_doc_concentration", _i32),
        ("sample_with_replacement", _i32),
        ("seed", _u64),
        ("dtype", _i32),
        ("max_inner_iter", _i32),
        ("mixed_resolve_iters", _i32),
    ]


class StepStats(C.Structure):
    _fields_ = [
        ("batch_docs", _i64),
        ("nonempty_docs", _i64),
        ("batch_entries", _i64),
        ("inner_iters", _i64),
        ("inner_iters_max", _i32),
        ("cap_hits", _i32),
        ("rho", _dbl),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


# name -> (restype, argtypes); every symbol include/stc.h declares
SIGNATURES = {
    "stc_last_error": (C.c_char_p, []),
    "stc_abi_version": (_int, []),
    "stc_device_count": (_int, [_pi32]),
    "stc_init": (_int, [_int, C.POINTER(_p)]),
    "stc_destroy": (_int, [_p]),
    "stc_synchronize": (_int, [_p]),
    "stc_comm_unique_id": (_int, [_pu8]),
    "stc_comm_init": (_int, [_p, _pu8, _int, _int]),
    "stc_comm_allreduce_f64": (_int, [_p, _pdbl, _i64]),
    "stc_dcsr_upload": (_int, [_p, _i64, _i64, _pi64, _pi32, _pdbl, _int, C.POINTER(_p)]),
    "stc_dcsr_shape": (_int, [_p, _pi64, _pi64, _pi64]),
    "stc_dcsr_download": (_int, [_p, _p, _pi64, _pi32, _pdbl]),
    "stc_dcsr_free": (_int, [_p]),
    "stc_hashing_tf_dev": (_int, [_p, _pu8, _i64, _pi64, _i64, _pi64, _i64, _i32, _int, _int, _int,
                                  C.POINTER(_p)]),
    "stc_hashing_tf": (_int, [_p, _pu8, _i64, _pi64, _i64, _pi64, _i64, _i32, _int, _int, _pi64,
                              _pi32, _pdbl]),
    "stc_hash_tokens": (_int, [_p, _pu8, _i64, _pi64, _i64, _i32, _int, _pi32]),
    "stc_tokens_upload": (_int, [_p, _pu8, _i64, _pi64, _i64, _pi64, _i64, C.POINTER(_p)]),
    "stc_tokens_free": (_int, [_p]),
    "stc_hashing_tf_tokens": (_int, [_p, _p, _i32, _int, _int, _int, C.POINTER(_p)]),
    "stc_tokenize": (_int, [_p, _pu8, _i64, _pi64, _i64, _pu8, _i64, _pi64, _pi64, _pi64, _pi64]),
    "stc_tokenize_hashing_tf_dev": (_int, [_p, _pu8, _i64, _pi64, _i64, _i32, _int, _int, _int,
                                           C.POINTER(_p)]),
    "stc_idf_fit": (_int, [_p, _p, _i64, _pdbl, _pi64, _pi64]),
    "stc_idf_transform": (_int, [_p, _p, _pdbl, _dbl]),
    "stc_idf_fit_dev": (_int, [_p, _p, _i64, C.POINTER(_p)]),
    "stc_idf_get": (_int, [_p, _p, _pdbl, _pi64, _pi64]),
    "stc_idf_transform_dev": (_int, [_p, _p, _p, C.c_double]),
    "stc_didf_shape": (_int, [_p, _pi64, _pi64]),
    "stc_didf_free": (_int, [_p]),
    "stc_lda_config_default": (None, [C.POINTER(LdaConfig)]),
    "stc_lda_create": (_int, [_p, C.POINTER(LdaConfig), C.POINTER(_p)]),
    "stc_lda_destroy": (_int, [_p]),
    "stc_lda_set_corpus": (_int, [_p, _p, _i64]),
    "stc_lda_init_random": (_int, [_p, _u64]),
    "stc_lda_set_topics": (_int, [_p, _pdbl, _int]),
    "stc_lda_get_topics": (_int, [_p, _pdbl, _int]),
    "stc_lda_set_alpha": (_int, [_p, _pdbl]),
    "stc_lda_get_alpha": (_int, [_p, _pdbl]),
    "stc_lda_get_eta": (_int, [_p, _pdbl]),
    "stc_lda_get_iteration": (_int, [_p, _pi64]),
    "stc_lda_shape": (_int, [_p, _pi32, _pi64]),
    "stc_lda_step": (_int, [_p, _pi64, _i64, _pdbl, C.POINTER(StepStats)]),
    "stc_lda_next": (_int, [_p, C.POINTER(StepStats)]),
    "stc_lda_estep": (_int, [_p, _pi64, _i64, _pdbl, _pdbl, _pdbl, _pi32]),
    "stc_lda_bound": (_int, [_p, _p, _u64, _i64, _pdbl, _pdbl, _pdbl, _pdbl, _pdbl]),
    "stc_lda_topic_distribution": (_int, [_p, _p, _u64, _i64, _pdbl, _pdbl]),
    "stc_lda_describe": (_int, [_p, _i32, _pi32, _pdbl]),
    "stc_lda_enable_timing": (_int, [_p, _int]),
    "stc_lda_phase_times": (_int, [_p, _pdbl, _pi64]),
    "stc_lda_counters": (_int, [_p, _pi64]),
    "stc_lda_kernel_counts": (_int, [_p, _pi64]),
    "stc_group_create": (_int, [_pi32, _int, C.POINTER(LdaConfig), C.POINTER(_p)]),
    "stc_group_destroy": (_int, [_p]),
    "stc_group_size": (_int, [_p, _pi32]),
    "stc_group_transport": (_int, [_p, _pi32]),
    "stc_group_member": (_int, [_p, _int, C.POINTER(_p)]),
    "stc_group_set_corpus": (_int, [_p, _i64, _i64, _pi64, _pi32, _pdbl]),
    "stc_group_init_random": (_int, [_p, _u64]),
    "stc_group_set_topics": (_int, [_p, _pdbl, _int]),
    "stc_group_get_topics": (_int, [_p, _pdbl, _int]),
    "stc_group_get_alpha": (_int, [_p, _pdbl]),
    "stc_group_get_iteration": (_int, [_p, _pi64]),
    "stc_group_synchronize": (_int, [_p]),
    "stc_group_release_corpus": (_int, [_p]),
    "stc_group_next": (_int, [_p, C.POINTER(StepStats)]),
    "stc_group_step": (_int, [_p, _pi64, _i64, _pdbl, C.POINTER(StepStats)]),
    "stc_group_describe": (_int, [_p, _i32, _pi32, _pdbl]),
    "stc_group_bound": (_int, [_p, _i64, _i64, _pi64, _pi32, _pdbl, _u64, _i64, _pdbl, _pdbl, _pdbl, _pdbl, _pdbl]),
    "stc_group_topic_distribution": (_int, [_p, _i64, _i64, _pi64, _pi32, _pdbl, _u64, _i64, _pdbl, _pdbl]),
}


class StcError(RuntimeError):
    """A non-zero status from libstc (message = stc_last_error())."""

    def __init__(self, code, msg):
        super().__init__(f"[stc status {code}] {msg}")
        self.code = code


class StcIllegalArgument(StcError, ValueError):
    """STC_ERR_INVALID_ARG — the JNI shim raises IllegalArgumentException for this code."""


_lib = None


def load():
    """Load libstc.so (raises if it was not built: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != STC_OK:
        msg = load().stc_last_error().decode("utf-8", "replace")
        if rc == STC_ERR_INVALID_ARG:
            raise StcIllegalArgument(rc, msg)
        raise StcError(rc, msg)


def ptr(a, ctype):
    """Pointer to a contiguous numpy array (None → NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(ctype))


def as_i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def as_i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def as_f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)
