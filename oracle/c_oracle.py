"""ctypes wrapper of oracle/_build/liblda_oracle.so — CPU ORACLE (checker / cpu_baseline only)."""
import ctypes as C
import os

import numpy as np

_LIB = None
PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "liblda_oracle.so")


def lib():
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(PATH)
        _LIB.oracle_estep.restype = C.c_int64
        _LIB.oracle_estep.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        _LIB.oracle_max_threads.restype = C.c_int
        _LIB.oracle_minibatch.restype = C.c_int64
        _LIB.oracle_minibatch.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_double, C.c_double,
                                          C.c_double, C.c_int, C.c_int]
    return _LIB


def minibatch(indptr, indices, values, doc_ids, gamma0, lam_kv, alpha, eta, rho, scale, optimize_alpha=True,
              n_threads=0):
    """One submitMiniBatch + updateLambda (+ updateAlpha) in Spark's structure (per-thread dense k×V
    stats summed like treeReduce).  lam_kv (k×V, float64, C order) and alpha are updated IN PLACE.
    Returns Σ inner iterations (−1 when the batch had no non-empty document)."""
    indptr = np.ascontiguousarray(indptr, np.int64)
    indices = np.ascontiguousarray(indices, np.int32)
    values = np.ascontiguousarray(values, np.float64)
    ids = np.ascontiguousarray(doc_ids, np.int64)
    g0 = np.ascontiguousarray(gamma0, np.float64)
    assert lam_kv.dtype == np.float64 and lam_kv.flags["C_CONTIGUOUS"]
    assert alpha.dtype == np.float64 and alpha.flags["C_CONTIGUOUS"]
    k, V = lam_kv.shape
    return int(lib().oracle_minibatch(ids.size, indptr.ctypes.data, indices.ctypes.data, values.ctypes.data,
                                      ids.ctypes.data, g0.ctypes.data, k, V, lam_kv.ctypes.data,
                                      alpha.ctypes.data, float(eta), float(rho), float(scale),
                                      int(bool(optimize_alpha)), int(n_threads)))


def available():
    return os.path.exists(PATH)


def estep(indptr, indices, values, doc_ids, exp_elog_beta, alpha, gamma0, n_threads=0, max_iter=0):
    """variationalTopicInference for each doc_ids[i] (fp64, Spark's unscaled form). Returns
    (gamma n×k, iters n, Σ iters)."""
    indptr = np.ascontiguousarray(indptr, np.int64)
    indices = np.ascontiguousarray(indices, np.int32)
    values = np.ascontiguousarray(values, np.float64)
    ids = np.ascontiguousarray(doc_ids, np.int64)
    eeb = np.ascontiguousarray(exp_elog_beta, np.float64)
    alpha = np.ascontiguousarray(alpha, np.float64)
    g0 = np.ascontiguousarray(gamma0, np.float64)
    k = eeb.shape[1]
    out = np.zeros((ids.size, k))
    its = np.zeros(ids.size, np.int32)
    tot = lib().oracle_estep(ids.size, indptr.ctypes.data, indices.ctypes.data, values.ctypes.data,
                             ids.ctypes.data, eeb.ctypes.data, k, alpha.ctypes.data, g0.ctypes.data,
                             out.ctypes.data, its.ctypes.data, int(n_threads), int(max_iter))
    return out, its, int(tot)


def max_threads():
    return lib().oracle_max_threads()
