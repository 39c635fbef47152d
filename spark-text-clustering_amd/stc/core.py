"""Device context + CSR containers over the C ABI.

``CsrMatrix`` is the host-side stand-in for the ``RDD[(Long, Vector)]`` / DataFrame ``features``
column the reference passes around (rows = documents, Spark ``SparseVector`` semantics: sorted
unique indices per row).  ``DeviceCsr`` is a device-resident copy owned by libstc.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class CsrMatrix:
    """Rows of sparse vectors: indptr int64[n+1], indices int32[nnz], values float64[nnz]."""

    def __init__(self, indptr, indices, values, num_cols):
        self.indptr = L.as_i64(indptr)
        self.indices = L.as_i32(indices)
        self.values = L.as_f64(values)
        self.num_cols = int(num_cols)
        if self.indptr.ndim != 1 or self.indptr.size < 1 or self.indptr[0] != 0:
            raise ValueError("indptr must be 1-D and start at 0")
        if self.indices.size != self.indptr[-1] or self.values.size != self.indptr[-1]:
            raise ValueError("indices/values must have indptr[-1] entries")

    @property
    def num_rows(self):
        return self.indptr.size - 1

    @property
    def nnz(self):
        return int(self.indptr[-1])

    @property
    def shape(self):
        return (self.num_rows, self.num_cols)

    def row(self, i):
        s, e = self.indptr[i], self.indptr[i + 1]
        return self.indices[s:e], self.values[s:e]

    def rows(self, ids):
        """Sub-matrix of the given rows (in order)."""
        ids = np.asarray(ids, np.int64)
        lens = self.indptr[ids + 1] - self.indptr[ids]
        indptr = np.zeros(ids.size + 1, np.int64)
        np.cumsum(lens, out=indptr[1:])
        sel = np.concatenate([np.arange(self.indptr[i], self.indptr[i + 1]) for i in ids]) \
            if ids.size else np.zeros(0, np.int64)
        return CsrMatrix(indptr, self.indices[sel], self.values[sel], self.num_cols)

    @staticmethod
    def from_rows(rows, num_cols):
        """rows: iterable of (indices, values)."""
        indptr = [0]
        idx, val = [], []
        for ids, vs in rows:
            idx.append(np.asarray(ids, np.int32))
            val.append(np.asarray(vs, np.float64))
            indptr.append(indptr[-1] + len(ids))
        cat = (lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt))
        return CsrMatrix(np.asarray(indptr, np.int64), cat(idx, np.int32), cat(val, np.float64), num_cols)

    def copy(self):
        return CsrMatrix(self.indptr.copy(), self.indices.copy(), self.values.copy(), self.num_cols)


class Context:
    """One GPU (stc_ctx).  ``Context.get(device)`` returns the process-wide context."""

    _instances = {}

    def __init__(self, device=0):
        self.lib = L.load()
        h = C.c_void_p()
        L.check(self.lib.stc_init(int(device), C.byref(h)))
        self.handle = h
        self.device = int(device)
        self.n_ranks = 1
        self.rank = 0

    @classmethod
    def get(cls, device=0):
        if device not in cls._instances:
            cls._instances[device] = Context(device)
        return cls._instances[device]

    @staticmethod
    def device_count():
        n = C.c_int32()
        L.check(L.load().stc_device_count(C.byref(n)))
        return n.value

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        L.check(L.load().stc_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes, n_ranks: int, rank: int):
        """Join the RCCL communicator (one process per GPU)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        L.check(self.lib.stc_comm_init(self.handle, buf, int(n_ranks), int(rank)))
        self.n_ranks, self.rank = int(n_ranks), int(rank)

    def allreduce(self, x):
        a = L.as_f64(np.atleast_1d(x)).copy()
        L.check(self.lib.stc_comm_allreduce_f64(self.handle, L.ptr(a, C.c_double), a.size))
        return a

    def synchronize(self):
        L.check(self.lib.stc_synchronize(self.handle))

    def close(self):
        if self.handle:
            self.lib.stc_destroy(self.handle)
            self.handle = None


class DeviceCsr:
    """A CSR matrix resident in HBM (stc_dcsr)."""

    def __init__(self, ctx: Context, handle):
        self.ctx = ctx
        self.handle = handle
        r, c, n = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(ctx.lib.stc_dcsr_shape(handle, C.byref(r), C.byref(c), C.byref(n)))
        self.num_rows, self.num_cols, self.nnz = r.value, c.value, n.value

    @staticmethod
    def upload(ctx: Context, m: CsrMatrix, dtype=L.STC_F64):
        h = C.c_void_p()
        L.check(ctx.lib.stc_dcsr_upload(ctx.handle, m.num_rows, m.num_cols, L.ptr(m.indptr, C.c_int64),
                                        L.ptr(m.indices, C.c_int32), L.ptr(m.values, C.c_double),
                                        int(dtype), C.byref(h)))
        return DeviceCsr(ctx, h)

    def download(self) -> CsrMatrix:
        indptr = np.zeros(self.num_rows + 1, np.int64)
        idx = np.zeros(self.nnz, np.int32)
        val = np.zeros(self.nnz, np.float64)
        L.check(self.ctx.lib.stc_dcsr_download(self.ctx.handle, self.handle, L.ptr(indptr, C.c_int64),
                                               L.ptr(idx, C.c_int32), L.ptr(val, C.c_double)))
        return CsrMatrix(indptr, idx, val, self.num_cols)

    def free(self):
        if self.handle:
            self.ctx.lib.stc_dcsr_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
