"""HashingTF / IDF / IDFModel with the Spark ML surface, backed by the HIP kernels K1–K5.

Mirrors ``org.apache.spark.ml.feature.{HashingTF, IDF, IDFModel}`` ([U] spark 2.4.3, build.sbt:10)
and the mllib ``IDF(minDocFreq)`` the reference calls at LDAClustering.scala:177.  Parameter names,
defaults and validation follow Spark (numFeatures = 2^18, binary = false, minDocFreq = 0).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .core import Context, CsrMatrix, DeviceCsr

_VARIANTS = {"murmur3": L.STC_HASH_STANDARD, "standard": L.STC_HASH_STANDARD,
             "spark24": L.STC_HASH_SPARK24, "murmur3-spark24": L.STC_HASH_SPARK24}


def encode_tokens(docs):
    """list[list[str|bytes]] → (utf8 uint8 blob, tok_off int64[n_tok+1], doc_off int64[n_docs+1])."""
    parts, tok_len, doc_len = [], [], []
    for toks in docs:
        doc_len.append(len(toks))
        for t in toks:
            b = t.encode("utf-8") if isinstance(t, str) else bytes(t)
            parts.append(b)
            tok_len.append(len(b))
    blob = np.frombuffer(b"".join(parts), np.uint8) if parts else np.zeros(0, np.uint8)
    tok_off = np.zeros(len(tok_len) + 1, np.int64)
    np.cumsum(tok_len, out=tok_off[1:])
    doc_off = np.zeros(len(doc_len) + 1, np.int64)
    np.cumsum(doc_len, out=doc_off[1:])
    return np.ascontiguousarray(blob), tok_off, doc_off


def encode_texts(texts):
    """list[str|bytes] → (utf8 uint8 blob, text_off int64[n_docs+1]) — one string per document."""
    parts = [t.encode("utf-8") if isinstance(t, str) else bytes(t) for t in texts]
    blob = np.frombuffer(b"".join(parts), np.uint8) if parts else np.zeros(0, np.uint8)
    off = np.zeros(len(parts) + 1, np.int64)
    np.cumsum([len(p) for p in parts], out=off[1:])
    return np.ascontiguousarray(blob), off


class DeviceTokens:
    """Token input resident on the GPU (stc_dtok): the (utf8, tok_off, doc_off) triple uploaded once."""

    def __init__(self, ctx: Context, blob, tok_off, doc_off):
        blob = np.ascontiguousarray(blob, np.uint8)
        tok_off = L.as_i64(tok_off)
        doc_off = L.as_i64(doc_off)
        h = C.c_void_p()
        L.check(ctx.lib.stc_tokens_upload(ctx.handle, L.ptr(blob, C.c_uint8), blob.size, L.ptr(tok_off, C.c_int64),
                                          tok_off.size - 1, L.ptr(doc_off, C.c_int64), doc_off.size - 1,
                                          C.byref(h)))
        self.ctx, self.handle = ctx, h
        self.n_bytes, self.n_tok, self.n_docs = blob.size, tok_off.size - 1, doc_off.size - 1

    def free(self):
        if self.handle:
            self.ctx.lib.stc_tokens_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Tokenizer:
    """Lower-cases each document and splits it on Java whitespace, on the GPU (kernel K0).

    Mirrors ``org.apache.spark.ml.feature.Tokenizer`` ([U] spark 2.4.3, build.sbt:10):
    ``text.toLowerCase.split("\\s")`` — interior empty tokens kept, trailing ones dropped, a
    document without whitespace is one token.  Lower-casing covers ASCII and Latin-1; text with
    characters that need other case tables raises ``ValueError`` (STC_ERR_INVALID_ARG).
    """

    def __init__(self, inputCol=None, outputCol=None, ctx: Context | None = None):
        self.inputCol, self.outputCol = inputCol, outputCol
        self._ctx = ctx

    @property
    def ctx(self):
        return self._ctx or Context.get()

    def encode(self, texts):
        """Tokens of every doc in HashingTF's input layout: (utf8 blob, tok_off, doc_off)."""
        text, off = encode_texts(texts)
        n_docs = off.size - 1
        blob = np.zeros(max(text.size + text.size // 2, 1), np.uint8)  # lower-casing may grow text by half (İ → "i̇")
        tok_off = np.zeros(text.size + n_docs + 1, np.int64)
        doc_off = np.zeros(n_docs + 1, np.int64)
        nb, nt = C.c_int64(), C.c_int64()
        L.check(self.ctx.lib.stc_tokenize(self.ctx.handle, L.ptr(text, C.c_uint8), text.size,
                                          L.ptr(off, C.c_int64), n_docs, L.ptr(blob, C.c_uint8), blob.size,
                                          C.byref(nb), L.ptr(tok_off, C.c_int64), C.byref(nt),
                                          L.ptr(doc_off, C.c_int64)))
        return blob[:nb.value].copy(), tok_off[:nt.value + 1].copy(), doc_off

    def transform(self, texts):
        """list[str] → list[list[str]] (the tokens of each document)."""
        blob, tok_off, doc_off = self.encode(texts)
        raw = blob.tobytes()
        toks = [raw[tok_off[t]:tok_off[t + 1]].decode("utf-8") for t in range(tok_off.size - 1)]
        return [toks[doc_off[d]:doc_off[d + 1]] for d in range(doc_off.size - 1)]


class HashingTF:
    """Maps a sequence of terms to their term frequencies using the hashing trick.

    numFeatures (default 2^18) buckets; bucket = nonNegativeMod(murmur3_x86_32(utf8(term), 42),
    numFeatures).  The default ``hashAlgorithm="murmur3-spark24"`` is what the pinned Spark 2.4.3
    (TextClustering/build.sbt:10) computes: ``Murmur3_x86_32.hashUnsafeBytes`` mixes each of the
    len % 4 tail bytes, sign-extended, as its own block, so a drop-in for the reference's pipeline
    lands every term in the same bucket.  ``"murmur3"`` selects the standard MurmurHash3_x86_32 tail
    (Spark 3.x ``hashUnsafeBytes2``); the two agree whenever the UTF-8 length is a multiple of 4.
    """

    def __init__(self, numFeatures=1 << 18, binary=False, hashAlgorithm="murmur3-spark24",
                 inputCol=None, outputCol=None, ctx: Context | None = None):
        self.setNumFeatures(numFeatures)
        self.setBinary(binary)
        if hashAlgorithm not in _VARIANTS:
            raise ValueError(f"HashingTF does not support hash function: {hashAlgorithm}")
        self.hashAlgorithm = hashAlgorithm
        self.inputCol, self.outputCol = inputCol, outputCol
        self._ctx = ctx

    @property
    def ctx(self):
        return self._ctx or Context.get()

    def setNumFeatures(self, n):
        if int(n) <= 0:
            raise ValueError(f"numFeatures must be > 0 but got {n}")
        self.numFeatures = int(n)
        return self

    def getNumFeatures(self):
        return self.numFeatures

    def setBinary(self, b):
        self.binary = bool(b)
        return self

    def getBinary(self):
        return self.binary

    def indexOf(self, term) -> int:
        """Bucket index of one term (mllib HashingTF.indexOf)."""
        return int(self.indices_of([term])[0])

    def indices_of(self, terms):
        blob, tok_off, _ = encode_tokens([list(terms)])
        out = np.zeros(len(terms), np.int32)
        L.check(self.ctx.lib.stc_hash_tokens(self.ctx.handle, L.ptr(blob, C.c_uint8), blob.size,
                                             L.ptr(tok_off, C.c_int64), len(terms), self.numFeatures,
                                             _VARIANTS[self.hashAlgorithm], L.ptr(out, C.c_int32)))
        return out

    def transform_device(self, docs, value_dtype=L.STC_F64, encoded=None) -> DeviceCsr:
        """Term frequencies of every doc, left resident in HBM (for IDF/LDA on the same GPU)."""
        blob, tok_off, doc_off = encoded if encoded is not None else encode_tokens(docs)
        h = C.c_void_p()
        L.check(self.ctx.lib.stc_hashing_tf_dev(
            self.ctx.handle, L.ptr(blob, C.c_uint8), blob.size, L.ptr(tok_off, C.c_int64),
            tok_off.size - 1, L.ptr(doc_off, C.c_int64), doc_off.size - 1, self.numFeatures,
            int(self.binary), _VARIANTS[self.hashAlgorithm], int(value_dtype), C.byref(h)))
        return DeviceCsr(self.ctx, h)

    def transform_tokens_device(self, tokens: "DeviceTokens", value_dtype=L.STC_F64) -> DeviceCsr:
        """Term frequencies of tokens already resident on the GPU (no host → device copy)."""
        h = C.c_void_p()
        L.check(self.ctx.lib.stc_hashing_tf_tokens(self.ctx.handle, tokens.handle, self.numFeatures, int(self.binary),
                                                   _VARIANTS[self.hashAlgorithm], int(value_dtype), C.byref(h)))
        return DeviceCsr(self.ctx, h)

    def transform_text_device(self, texts, value_dtype=L.STC_F64) -> DeviceCsr:
        """Tokenizer → HashingTF fused on the GPU: raw document strings in, term frequencies left
        resident in HBM (no host round trip between the stages)."""
        text, off = encode_texts(texts)
        h = C.c_void_p()
        L.check(self.ctx.lib.stc_tokenize_hashing_tf_dev(
            self.ctx.handle, L.ptr(text, C.c_uint8), text.size, L.ptr(off, C.c_int64), off.size - 1,
            self.numFeatures, int(self.binary), _VARIANTS[self.hashAlgorithm], int(value_dtype),
            C.byref(h)))
        return DeviceCsr(self.ctx, h)

    def transform(self, docs, encoded=None) -> CsrMatrix:
        d = self.transform_device(docs, L.STC_F64, encoded)
        try:
            return d.download()
        finally:
            d.free()


class IDFModel:
    """Fitted IDF: ``idf`` (float64[numFeatures]), ``docFreq`` (int64), ``numDocs``.  A model fitted on the
    device (IDF.fit_device) stays there (stc_didf): transform_device uses it in place and the host arrays
    are copied out only when read."""

    def __init__(self, idf=None, docFreq=None, numDocs=None, ctx: Context | None = None, _dev=None, _cols=0):
        self._idf = None if idf is None else np.asarray(idf, np.float64)
        self._df = None if docFreq is None else np.asarray(docFreq, np.int64)
        self._m = None if numDocs is None else int(numDocs)
        self._ctx = ctx
        self._dev, self._cols = _dev, int(_cols)
        # freeing the device model needs only the library, never a context (a __del__ at
        # interpreter shutdown must not create or initialise one)
        self._lib = L.load() if _dev is not None else None
        if _dev is not None:
            cols = C.c_int64()
            L.check(self._lib.stc_didf_shape(_dev, C.byref(cols), None))
            self._cols = cols.value

    @property
    def ctx(self):
        return self._ctx or Context.get()

    def _fetch(self):
        idf = np.zeros(self._cols, np.float64)
        df = np.zeros(self._cols, np.int64)
        m = C.c_int64()
        L.check(self.ctx.lib.stc_idf_get(self.ctx.handle, self._dev, L.ptr(idf, C.c_double), L.ptr(df, C.c_int64),
                                         C.byref(m)))
        self._idf, self._df, self._m = idf, df, m.value

    @property
    def idf(self):
        if self._idf is None:
            self._fetch()
        return self._idf

    @property
    def docFreq(self):
        if self._df is None:
            self._fetch()
        return self._df

    @property
    def numDocs(self):
        if self._m is None:
            self._fetch()
        return self._m

    def transform_device(self, tf: DeviceCsr, zero_floor=0.0) -> DeviceCsr:
        """In place on a device CSR.  zero_floor=1e-4 reproduces LDAClustering.scala:184-187."""
        if self._dev is not None:
            if tf.num_cols != self._cols:
                raise ValueError(f"vector size {tf.num_cols} does not match IDF size {self._cols}")
            L.check(self.ctx.lib.stc_idf_transform_dev(self.ctx.handle, tf.handle, self._dev, float(zero_floor)))
            return tf
        idf = L.as_f64(self.idf)
        if tf.num_cols != idf.size:
            raise ValueError(f"vector size {tf.num_cols} does not match IDF size {idf.size}")
        L.check(self.ctx.lib.stc_idf_transform(self.ctx.handle, tf.handle, L.ptr(idf, C.c_double),
                                               float(zero_floor)))
        return tf

    def transform(self, tf: CsrMatrix, zero_floor=0.0) -> CsrMatrix:
        d = DeviceCsr.upload(self.ctx, tf, L.STC_F64)
        try:
            return self.transform_device(d, zero_floor).download()
        finally:
            d.free()

    def free(self):
        """releases the device copy (the host arrays are fetched first, so the model stays usable)"""
        if self._dev is not None:
            if self._idf is None:
                self._fetch()
            self._lib.stc_didf_free(self._dev)
            self._dev = None

    def __del__(self):
        try:
            if self._dev is not None:
                self._lib.stc_didf_free(self._dev)
                self._dev = None
        except Exception:
            pass


class IDF:
    """Compute the Inverse Document Frequency of a collection of term-frequency vectors."""

    def __init__(self, minDocFreq=0, inputCol=None, outputCol=None, ctx: Context | None = None):
        self.setMinDocFreq(minDocFreq)
        self.inputCol, self.outputCol = inputCol, outputCol
        self._ctx = ctx

    @property
    def ctx(self):
        return self._ctx or Context.get()

    def setMinDocFreq(self, v):
        if int(v) < 0:
            raise ValueError(f"minDocFreq must be >= 0 but got {v}")
        self.minDocFreq = int(v)
        return self

    def getMinDocFreq(self):
        return self.minDocFreq

    def fit_device(self, tf: DeviceCsr) -> IDFModel:
        """IDF.fit on a device CSR; the model stays on the device (stc_idf_fit_dev)"""
        h = C.c_void_p()
        L.check(self.ctx.lib.stc_idf_fit_dev(self.ctx.handle, tf.handle, self.minDocFreq, C.byref(h)))
        return IDFModel(ctx=self._ctx, _dev=h, _cols=tf.num_cols)

    def fit(self, tf: CsrMatrix) -> IDFModel:
        d = DeviceCsr.upload(self.ctx, tf, L.STC_F64)
        try:
            idf = np.zeros(tf.num_cols, np.float64)
            df = np.zeros(tf.num_cols, np.int64)
            m = C.c_int64()
            L.check(self.ctx.lib.stc_idf_fit(self.ctx.handle, d.handle, self.minDocFreq,
                                             L.ptr(idf, C.c_double), L.ptr(df, C.c_int64), C.byref(m)))
            return IDFModel(idf, df, m.value, self._ctx)
        finally:
            d.free()
