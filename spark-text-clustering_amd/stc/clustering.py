"""Online-variational-Bayes LDA with the Spark ML / mllib surface, backed by libstc (K6–K12).

* ``LDA`` / ``LDAModel`` mirror ``org.apache.spark.ml.clustering.{LDA, LocalLDAModel}``
  ([U] spark 2.4.3): k=10, maxIter=20, optimizer="online", learningOffset=1024,
  learningDecay=0.51, subsamplingRate=0.05, optimizeDocConcentration=true, seed = the class-name
  hash; model methods topicsMatrix, describeTopics, logLikelihood, logPerplexity, transform.
* ``OnlineLDAOptimizer`` + ``MllibLDA`` mirror the RDD API the reference drives at
  LDAClustering.scala:37-61 (``new LDA().setOptimizer(new OnlineLDAOptimizer()
  .setMiniBatchFraction(0.05 + 1.0 / N)).setK(..).setMaxIterations(..)...run(corpus)``).

Only the online optimizer exists here; ``"em"`` (the reference's default, Params.scala:9) is out of
scope and raises like an unknown optimizer does in LDAClustering.scala:44-45.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib as L
from .core import Context, CsrMatrix, DeviceCsr


def _java_string_hash(s: str) -> int:
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


ML_LDA_DEFAULT_SEED = _java_string_hash("org.apache.spark.ml.clustering.LDA")
_DTYPES = {"f32": L.STC_F32, "float32": L.STC_F32, "f64": L.STC_F64, "float64": L.STC_F64, "mixed": L.STC_MIXED}


def _lda_config(lib, k, vocab_size, doc_concentration, topic_concentration, tau0, kappa, mini_batch_fraction,
                gamma_shape, optimize_doc_concentration, sample_with_replacement, seed, dtype, max_inner_iter,
                mixed_resolve_iters=0):
    """stc_lda_config from the Spark-ML parameters (returns the config and the α buffer it points to)."""
    cfg = L.LdaConfig()
    lib.stc_lda_config_default(C.byref(cfg))
    cfg.k = int(k)
    cfg.vocab_size = int(vocab_size)
    alpha_buf = None
    if doc_concentration is not None:
        alpha_buf = L.as_f64(np.atleast_1d(doc_concentration))
        cfg.doc_concentration = L.ptr(alpha_buf, C.c_double)
        cfg.doc_concentration_len = alpha_buf.size
    cfg.topic_concentration = float(-1.0 if topic_concentration is None else topic_concentration)
    cfg.tau0 = float(tau0)
    cfg.kappa = float(kappa)
    cfg.mini_batch_fraction = float(mini_batch_fraction)
    cfg.gamma_shape = float(gamma_shape)
    cfg.optimize_doc_concentration = int(bool(optimize_doc_concentration))
    cfg.sample_with_replacement = int(bool(sample_with_replacement))
    cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    cfg.dtype = _DTYPES[dtype] if isinstance(dtype, str) else int(dtype)
    cfg.max_inner_iter = int(max_inner_iter)
    cfg.mixed_resolve_iters = int(mixed_resolve_iters)  # dtype "mixed": the fp64 re-solve threshold (0: 500)
    return cfg, alpha_buf


def _phase_times(lib, h):
    """stc_lda_phase_times of one handle: mean device ms per step of each phase"""
    ms = np.zeros(5, np.float64)
    steps = C.c_int64()
    L.check(lib.stc_lda_phase_times(h, L.ptr(ms, C.c_double), C.byref(steps)))
    return {"sample": ms[0], "estep": ms[1], "sstats": ms[2], "allreduce": ms[3], "mstep": ms[4],
            "steps": steps.value}


# stc.h enum stc_kernel_count: the E-step kernel families stc_lda_kernel_counts counts launches of
KERNEL_FAMILIES = ("k_estep_rows64", "k_estep_rows64_long", "k_estep_grid", "k_estep_wide", "k_estep_wide_mc",
                   "k_estep_wide_tc", "k_estep_tgrid64", "team_fallback", "k_estep", "mixed_resolves", "mixed_docs")


def _counters(lib, h):
    """stc_lda_counters + stc_lda_kernel_counts of one handle (cumulative since creation)"""
    out = np.zeros(4, np.int64)
    L.check(lib.stc_lda_counters(h, L.ptr(out, C.c_int64)))
    kc = np.zeros(12, np.int64)
    L.check(lib.stc_lda_kernel_counts(h, L.ptr(kc, C.c_int64)))
    return {"docs": int(out[0]), "entries": int(out[1]), "inner_iters": int(out[2]), "cap_hits": int(out[3]),
            "kernels": {f: int(kc[i]) for i, f in enumerate(KERNEL_FAMILIES)}}


class LdaHandle:
    """Owns one stc_lda (optimizer state + LocalLDAModel parameters on the GPU)."""

    def __init__(self, ctx: Context, k, vocab_size, doc_concentration=None, topic_concentration=-1.0,
                 tau0=1024.0, kappa=0.51, mini_batch_fraction=0.05, gamma_shape=100.0,
                 optimize_doc_concentration=True, sample_with_replacement=True, seed=0,
                 dtype="f64", max_inner_iter=0, mixed_resolve_iters=0):
        self.ctx = ctx
        cfg, self._alpha_buf = _lda_config(ctx.lib, k, vocab_size, doc_concentration, topic_concentration, tau0,
                                           kappa, mini_batch_fraction, gamma_shape, optimize_doc_concentration,
                                           sample_with_replacement, seed, dtype, max_inner_iter, mixed_resolve_iters)
        h = C.c_void_p()
        L.check(ctx.lib.stc_lda_create(ctx.handle, C.byref(cfg), C.byref(h)))
        self.handle = h
        self.k, self.vocab_size, self.dtype = cfg.k, cfg.vocab_size, cfg.dtype
        self.seed = cfg.seed
        self.gamma_shape = cfg.gamma_shape
        self._corpus = None

    # ---- state
    def set_corpus(self, corpus: DeviceCsr, corpus_size_total=None):
        total = corpus.num_rows if corpus_size_total is None else int(corpus_size_total)
        L.check(self.ctx.lib.stc_lda_set_corpus(self.handle, corpus.handle, total))
        self._corpus = corpus  # keep alive

    def init_random(self, seed):
        L.check(self.ctx.lib.stc_lda_init_random(self.handle, int(seed) & 0xFFFFFFFFFFFFFFFF))

    def set_topics(self, topics, layout=L.STC_LAYOUT_VK):
        t = L.as_f64(topics)
        L.check(self.ctx.lib.stc_lda_set_topics(self.handle, L.ptr(t, C.c_double), layout))

    def topics(self, layout=L.STC_LAYOUT_VK):
        shape = (self.vocab_size, self.k) if layout == L.STC_LAYOUT_VK else (self.k, self.vocab_size)
        out = np.zeros(shape, np.float64)
        L.check(self.ctx.lib.stc_lda_get_topics(self.handle, L.ptr(out, C.c_double), layout))
        return out

    def alpha(self):
        out = np.zeros(self.k, np.float64)
        L.check(self.ctx.lib.stc_lda_get_alpha(self.handle, L.ptr(out, C.c_double)))
        return out

    def set_alpha(self, a):
        a = L.as_f64(np.broadcast_to(np.asarray(a, np.float64), (self.k,)))
        L.check(self.ctx.lib.stc_lda_set_alpha(self.handle, L.ptr(a, C.c_double)))

    def eta(self):
        x = C.c_double()
        L.check(self.ctx.lib.stc_lda_get_eta(self.handle, C.byref(x)))
        return x.value

    def iteration(self):
        x = C.c_int64()
        L.check(self.ctx.lib.stc_lda_get_iteration(self.handle, C.byref(x)))
        return x.value

    # ---- optimizer
    def step(self, batch_ids, gamma0=None, stats=True):
        ids = L.as_i64(batch_ids)
        g0 = None if gamma0 is None else L.as_f64(gamma0)
        st = L.StepStats() if stats else None
        L.check(self.ctx.lib.stc_lda_step(self.handle, L.ptr(ids, C.c_int64), ids.size,
                                          L.ptr(g0, C.c_double), C.byref(st) if stats else None))
        return st.as_dict() if stats else None

    def next(self, stats=True):
        st = L.StepStats() if stats else None
        L.check(self.ctx.lib.stc_lda_next(self.handle, C.byref(st) if stats else None))
        return st.as_dict() if stats else None

    def estep(self, batch_ids, gamma0=None, want_stat=False):
        ids = L.as_i64(batch_ids)
        g0 = None if gamma0 is None else L.as_f64(gamma0)
        gamma = np.zeros((ids.size, self.k), np.float64)
        iters = np.zeros(ids.size, np.int32)
        stat = np.zeros((self.vocab_size, self.k), np.float64) if want_stat else None
        L.check(self.ctx.lib.stc_lda_estep(self.handle, L.ptr(ids, C.c_int64), ids.size, L.ptr(g0, C.c_double),
                                           L.ptr(gamma, C.c_double), L.ptr(stat, C.c_double),
                                           L.ptr(iters, C.c_int32)))
        return gamma, stat, iters

    # ---- LocalLDAModel
    def bound(self, docs: DeviceCsr, gamma_seed=0, doc_id_base=0, gamma0=None):
        g0 = None if gamma0 is None else L.as_f64(gamma0)
        b, cp, tp, tok = C.c_double(), C.c_double(), C.c_double(), C.c_double()
        L.check(self.ctx.lib.stc_lda_bound(self.handle, docs.handle, int(gamma_seed) & 0xFFFFFFFFFFFFFFFF,
                                           int(doc_id_base), L.ptr(g0, C.c_double), C.byref(b), C.byref(cp),
                                           C.byref(tp), C.byref(tok)))
        return {"bound": b.value, "corpus_part": cp.value, "topics_part": tp.value, "token_count": tok.value}

    def topic_distribution(self, docs: DeviceCsr, gamma_seed=0, doc_id_base=0, gamma0=None):
        g0 = None if gamma0 is None else L.as_f64(gamma0)
        out = np.zeros((docs.num_rows, self.k), np.float64)
        L.check(self.ctx.lib.stc_lda_topic_distribution(self.handle, docs.handle,
                                                        int(gamma_seed) & 0xFFFFFFFFFFFFFFFF, int(doc_id_base),
                                                        L.ptr(g0, C.c_double), L.ptr(out, C.c_double)))
        return out

    def describe(self, max_terms=10):
        n = min(int(max_terms), self.vocab_size)
        idx = np.zeros((self.k, n), np.int32)
        w = np.zeros((self.k, n), np.float64)
        L.check(self.ctx.lib.stc_lda_describe(self.handle, int(max_terms), L.ptr(idx, C.c_int32),
                                              L.ptr(w, C.c_double)))
        return idx, w

    # ---- instrumentation
    def enable_timing(self, on=True):
        L.check(self.ctx.lib.stc_lda_enable_timing(self.handle, int(bool(on))))

    def phase_times(self):
        return _phase_times(self.ctx.lib, self.handle)

    def counters(self):
        return _counters(self.ctx.lib, self.handle)

    def close(self):
        if self.handle:
            self.ctx.lib.stc_lda_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LdaGroup:
    """Owns one stc_group: the LDA over several devices from ONE process (stc_group_create; the JVM
    drop-in's multi-GPU form).  The corpus is given on the host and sharded by the library; document ids
    are global.  ``devices`` repeating one device runs the multi-GPU decomposition on that device."""

    def __init__(self, devices, k, vocab_size, doc_concentration=None, topic_concentration=-1.0, tau0=1024.0,
                 kappa=0.51, mini_batch_fraction=0.05, gamma_shape=100.0, optimize_doc_concentration=True,
                 sample_with_replacement=True, seed=0, dtype="f64", max_inner_iter=0, mixed_resolve_iters=0):
        self.lib = L.load()
        cfg, self._alpha_buf = _lda_config(self.lib, k, vocab_size, doc_concentration, topic_concentration, tau0,
                                           kappa, mini_batch_fraction, gamma_shape, optimize_doc_concentration,
                                           sample_with_replacement, seed, dtype, max_inner_iter, mixed_resolve_iters)
        devs = np.ascontiguousarray(np.asarray(devices, np.int32))
        h = C.c_void_p()
        L.check(self.lib.stc_group_create(L.ptr(devs, C.c_int32), devs.size, C.byref(cfg), C.byref(h)))
        self.handle = h
        self.devices = devs.tolist()
        self.k, self.vocab_size = cfg.k, cfg.vocab_size

    @staticmethod
    def _csr(m: CsrMatrix):
        return (L.as_i64(m.indptr), np.ascontiguousarray(m.indices, np.int32), L.as_f64(m.values))

    def set_corpus(self, corpus: CsrMatrix):
        ip, ix, v = self._csr(corpus)
        L.check(self.lib.stc_group_set_corpus(self.handle, corpus.num_rows, corpus.num_cols, L.ptr(ip, C.c_int64),
                                              L.ptr(ix, C.c_int32), L.ptr(v, C.c_double)))

    def init_random(self, seed):
        L.check(self.lib.stc_group_init_random(self.handle, int(seed) & 0xFFFFFFFFFFFFFFFF))

    def set_topics(self, topics, layout=L.STC_LAYOUT_VK):
        t = L.as_f64(topics)
        L.check(self.lib.stc_group_set_topics(self.handle, L.ptr(t, C.c_double), layout))

    def topics(self, layout=L.STC_LAYOUT_VK):
        shape = (self.vocab_size, self.k) if layout == L.STC_LAYOUT_VK else (self.k, self.vocab_size)
        out = np.zeros(shape, np.float64)
        L.check(self.lib.stc_group_get_topics(self.handle, L.ptr(out, C.c_double), layout))
        return out

    def alpha(self):
        out = np.zeros(self.k, np.float64)
        L.check(self.lib.stc_group_get_alpha(self.handle, L.ptr(out, C.c_double)))
        return out

    def iteration(self):
        x = C.c_int64()
        L.check(self.lib.stc_group_get_iteration(self.handle, C.byref(x)))
        return x.value

    def release_corpus(self):
        """frees the training corpus shards (inference needs none; stc_group_release_corpus)"""
        L.check(self.lib.stc_group_release_corpus(self.handle))

    def synchronize(self):
        """waits for every member's queued work (stc_group_synchronize)"""
        L.check(self.lib.stc_group_synchronize(self.handle))

    def members(self):
        """the member stc_lda handles, for counters and timing only (stc_group_member)"""
        out = []
        for i in range(len(self.devices)):
            h = C.c_void_p()
            L.check(self.lib.stc_group_member(self.handle, i, C.byref(h)))
            out.append(h)
        return out

    def enable_timing(self, on=True):
        for h in self.members():
            L.check(self.lib.stc_lda_enable_timing(h, int(bool(on))))

    def phase_times(self):
        """per member: mean device ms per step of each phase"""
        return [_phase_times(self.lib, h) for h in self.members()]

    def counters(self):
        """per member: cumulative docs / entries / inner iterations / cap hits"""
        return [_counters(self.lib, h) for h in self.members()]

    def transport(self):
        """how the members' collectives travel: "none" (one member), "in-process" (one device repeated) or
        "rccl" (ncclCommInitAll over distinct devices — one included under STC_GROUP_RCCL=1)"""
        t = C.c_int32()
        L.check(self.lib.stc_group_transport(self.handle, C.byref(t)))
        return {L.STC_TRANSPORT_NONE: "none", L.STC_TRANSPORT_IN_PROCESS: "in-process",
                L.STC_TRANSPORT_RCCL: "rccl"}[t.value]

    def step(self, batch_ids, gamma0=None, stats=True):
        ids = L.as_i64(batch_ids)
        g0 = None if gamma0 is None else L.as_f64(gamma0)
        st = L.StepStats() if stats else None
        L.check(self.lib.stc_group_step(self.handle, L.ptr(ids, C.c_int64), ids.size, L.ptr(g0, C.c_double),
                                        C.byref(st) if stats else None))
        return st.as_dict() if stats else None

    def next(self, stats=True):
        st = L.StepStats() if stats else None
        L.check(self.lib.stc_group_next(self.handle, C.byref(st) if stats else None))
        return st.as_dict() if stats else None

    def describe(self, max_terms=10):
        n = min(int(max_terms), self.vocab_size)
        idx = np.zeros((self.k, n), np.int32)
        w = np.zeros((self.k, n), np.float64)
        L.check(self.lib.stc_group_describe(self.handle, int(max_terms), L.ptr(idx, C.c_int32), L.ptr(w, C.c_double)))
        return idx, w

    def bound(self, docs: CsrMatrix, gamma_seed=0, doc_id_base=0, gamma0=None):
        ip, ix, v = self._csr(docs)
        g0 = None if gamma0 is None else L.as_f64(gamma0)
        b, cp, tp, tok = C.c_double(), C.c_double(), C.c_double(), C.c_double()
        L.check(self.lib.stc_group_bound(self.handle, docs.num_rows, docs.num_cols, L.ptr(ip, C.c_int64),
                                         L.ptr(ix, C.c_int32), L.ptr(v, C.c_double),
                                         int(gamma_seed) & 0xFFFFFFFFFFFFFFFF, int(doc_id_base),
                                         L.ptr(g0, C.c_double), C.byref(b), C.byref(cp), C.byref(tp), C.byref(tok)))
        return {"bound": b.value, "corpus_part": cp.value, "topics_part": tp.value, "token_count": tok.value}

    def topic_distribution(self, docs: CsrMatrix, gamma_seed=0, doc_id_base=0, gamma0=None):
        ip, ix, v = self._csr(docs)
        g0 = None if gamma0 is None else L.as_f64(gamma0)
        out = np.zeros((docs.num_rows, self.k), np.float64)
        L.check(self.lib.stc_group_topic_distribution(self.handle, docs.num_rows, docs.num_cols, L.ptr(ip, C.c_int64),
                                                      L.ptr(ix, C.c_int32), L.ptr(v, C.c_double),
                                                      int(gamma_seed) & 0xFFFFFFFFFFFFFFFF, int(doc_id_base),
                                                      L.ptr(g0, C.c_double), L.ptr(out, C.c_double)))
        return out

    def close(self):
        if self.handle:
            self.lib.stc_group_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _as_device(ctx, data, dtype):
    if isinstance(data, DeviceCsr):
        return data, False
    return DeviceCsr.upload(ctx, data, L.corpus_dtype(dtype)), True


class LDAModel:
    """LocalLDAModel: topicsMatrix (V×k = λᵀ), docConcentration α, topicConcentration η."""

    def __init__(self, handle: LdaHandle, gamma_seed=None):
        self._h = handle
        self.k = handle.k
        self.vocabSize = handle.vocab_size
        self.gammaSeed = handle.seed if gamma_seed is None else gamma_seed

    @staticmethod
    def from_topics(topics_matrix, doc_concentration, topic_concentration, gamma_shape=100.0,
                    seed=0, dtype="f64", ctx: Context | None = None):
        """Build a LocalLDAModel from an existing V×k topicsMatrix (e.g. DistributedLDAModel.toLocal)."""
        tm = np.asarray(topics_matrix, np.float64)
        ctx = ctx or Context.get()
        h = LdaHandle(ctx, tm.shape[1], tm.shape[0], doc_concentration=doc_concentration,
                      topic_concentration=topic_concentration, gamma_shape=gamma_shape, seed=seed,
                      dtype=dtype)
        h.set_topics(tm)
        return LDAModel(h)

    def isDistributed(self):
        return False

    def topicsMatrix(self):
        return self._h.topics(L.STC_LAYOUT_VK)

    def estimatedDocConcentration(self):
        return self._h.alpha()

    def getTopicConcentration(self):
        return self._h.eta()

    def describeTopics(self, maxTermsPerTopic=10):
        """[(topic, termIndices, termWeights)] like the ml DataFrame rows."""
        idx, w = self._h.describe(maxTermsPerTopic)
        return [(t, idx[t].astype(np.int64), w[t]) for t in range(self.k)]

    def logLikelihood(self, dataset, gamma0=None):
        d, own = _as_device(self._h.ctx, dataset, self._h.dtype)
        try:
            return self._h.bound(d, self.gammaSeed, 0, gamma0)["bound"]
        finally:
            if own:
                d.free()

    def logPerplexity(self, dataset, gamma0=None):
        d, own = _as_device(self._h.ctx, dataset, self._h.dtype)
        try:
            b = self._h.bound(d, self.gammaSeed, 0, gamma0)
            return -b["bound"] / b["token_count"]
        finally:
            if own:
                d.free()

    def transform(self, dataset, gamma0=None):
        """topicDistribution of every row (LDALoader.scala:108); zeros for empty rows."""
        d, own = _as_device(self._h.ctx, dataset, self._h.dtype)
        try:
            return self._h.topic_distribution(d, self.gammaSeed, 0, gamma0)
        finally:
            if own:
                d.free()

    topicDistribution = transform

    # ---- persistence: [U] LocalLDAModel.save / LocalLDAModel.load (SaveLoadV1_0 layout, stc.io)
    def save(self, path, overwrite=False):
        """Write this model as a Spark mllib LocalLDAModel directory (stock Spark can load it)."""
        from . import io

        io.save_local(path, self.topicsMatrix(), self.estimatedDocConcentration(), self.getTopicConcentration(),
                      self._h.gamma_shape, overwrite=overwrite)

    @staticmethod
    def load(path, dtype="f64", seed=0, ctx: Context | None = None) -> "LDAModel":
        """Read a Spark mllib LocalLDAModel directory onto the GPU."""
        from . import io

        m = io.load_local(path)
        return LDAModel.from_topics(m["topics"], m["alpha"], m["eta"], gamma_shape=m["gamma_shape"], seed=seed,
                                    dtype=dtype, ctx=ctx)


class DistributedLDAModel:
    """[U] DistributedLDAModel as the reference loads it (LDALoader.scala:37): the saved EM graph, read
    from its parquet layout (stc.io).  What the reference then asks of it — describeTopics
    (LDALoader.scala:66) and toLocal.topicDistribution (:108) — runs on the GPU through ``toLocal``
    (topicsMatrix = the term vertices' counts n_wk)."""

    def __init__(self, data):
        self._d = data
        self.k, self.vocabSize = data["k"], data["vocab_size"]
        self.docConcentration = data["alpha"]
        self.topicConcentration = data["eta"]
        self.gammaShape = data["gamma_shape"]
        self.iterationTimes = data["iteration_times"]
        self._local = {}

    @staticmethod
    def load(path) -> "DistributedLDAModel":
        from . import io

        return DistributedLDAModel(io.load_distributed(path))

    def isDistributed(self):
        return True

    def topicsMatrix(self):
        return self._d["topics"].copy()

    def globalTopicTotals(self):
        return self._d["global_topic_totals"].copy()

    def toLocal(self, dtype="f64", seed=0, ctx: Context | None = None) -> LDAModel:
        key = (dtype, seed, id(ctx))
        if key not in self._local:
            self._local[key] = LDAModel.from_topics(self._d["topics"], self.docConcentration, self.topicConcentration,
                                                    gamma_shape=self.gammaShape, seed=seed, dtype=dtype, ctx=ctx)
        return self._local[key]

    def describeTopics(self, maxTermsPerTopic=10, ctx: Context | None = None):
        """Top terms per topic by n_wk / Σ_w n_wk (the EM model's column totals), on the GPU."""
        return self.toLocal(ctx=ctx).describeTopics(maxTermsPerTopic)


class LDA:
    """ml.clustering.LDA estimator (optimizer="online" only)."""

    def __init__(self, k=10, maxIter=20, optimizer="online", learningOffset=1024.0, learningDecay=0.51,
                 subsamplingRate=0.05, optimizeDocConcentration=True, docConcentration=None,
                 topicConcentration=None, seed=ML_LDA_DEFAULT_SEED, featuresCol="features",
                 topicDistributionCol="topicDistribution", dtype="f64", maxInnerIter=0,
                 ctx: Context | None = None):
        self.setK(k).setMaxIter(maxIter).setOptimizer(optimizer).setLearningOffset(learningOffset)
        self.setLearningDecay(learningDecay).setSubsamplingRate(subsamplingRate)
        self.optimizeDocConcentration = bool(optimizeDocConcentration)
        self.docConcentration = docConcentration
        self.topicConcentration = topicConcentration
        self.seed = int(seed)
        self.featuresCol, self.topicDistributionCol = featuresCol, topicDistributionCol
        self.dtype = dtype
        self.maxInnerIter = int(maxInnerIter)
        self._ctx = ctx
        self.iterationTimes = []

    def setK(self, k):
        if int(k) <= 1:
            raise ValueError(f"LDA k (number of clusters) must be > 1, but was set to {k}")
        self.k = int(k)
        return self

    def setMaxIter(self, n):
        if int(n) < 0:
            raise ValueError(f"maxIter must be >= 0 but got {n}")
        self.maxIter = int(n)
        return self

    def setOptimizer(self, o):
        if str(o).lower() != "online":
            raise ValueError(f"Only online is supported by this build but got {o}.")
        self.optimizer = "online"
        return self

    def setLearningOffset(self, v):
        if float(v) <= 0:
            raise ValueError(f"learningOffset must be > 0 but got {v}")
        self.learningOffset = float(v)
        return self

    def setLearningDecay(self, v):
        if float(v) <= 0:
            raise ValueError(f"learningDecay must be > 0 but got {v}")
        self.learningDecay = float(v)
        return self

    def setSubsamplingRate(self, v):
        if not (0.0 < float(v) <= 1.0):
            raise ValueError(f"subsamplingRate must be in range (0, 1] but got {v}")
        self.subsamplingRate = float(v)
        return self

    def setSeed(self, s):
        self.seed = int(s)
        return self

    def fit(self, dataset, corpus_size_total=None) -> LDAModel:
        ctx = self._ctx or Context.get()
        d, _ = _as_device(ctx, dataset, _DTYPES[self.dtype])
        total = d.num_rows
        if corpus_size_total is None and ctx.n_ranks > 1:
            total = int(ctx.allreduce([float(d.num_rows)])[0])
        elif corpus_size_total is not None:
            total = int(corpus_size_total)
        h = LdaHandle(ctx, self.k, d.num_cols, doc_concentration=self.docConcentration,
                      topic_concentration=self.topicConcentration, tau0=self.learningOffset,
                      kappa=self.learningDecay, mini_batch_fraction=self.subsamplingRate,
                      optimize_doc_concentration=self.optimizeDocConcentration, seed=self.seed,
                      dtype=self.dtype, max_inner_iter=self.maxInnerIter)
        h.set_corpus(d, total)
        h.init_random(self.seed)
        import time
        self.iterationTimes = []
        for _ in range(self.maxIter):
            t0 = time.perf_counter()
            h.next(stats=False)
            ctx.synchronize()
            self.iterationTimes.append(time.perf_counter() - t0)
        return LDAModel(h)


class OnlineLDAOptimizer:
    """mllib OnlineLDAOptimizer setters (defaults: tau0 1024, kappa 0.51, fraction 0.05,
    optimizeDocConcentration false, gammaShape 100, sampleWithReplacement true)."""

    def __init__(self):
        self.tau0, self.kappa, self.miniBatchFraction = 1024.0, 0.51, 0.05
        self.optimizeDocConcentration, self.gammaShape, self.sampleWithReplacement = False, 100.0, True

    def setTau0(self, v):
        if v <= 0:
            raise ValueError(f"LDA tau0 must be positive, but was set to {v}")
        self.tau0 = float(v)
        return self

    def setKappa(self, v):
        if v < 0:
            raise ValueError(f"Online LDA kappa must be nonnegative, but was set to {v}")
        self.kappa = float(v)
        return self

    def setMiniBatchFraction(self, v):
        if not (0.0 < v <= 1.0):
            raise ValueError(f"Online LDA miniBatchFraction must be in range (0,1], but was set to {v}")
        self.miniBatchFraction = float(v)
        return self

    def setOptimizeDocConcentration(self, b):
        self.optimizeDocConcentration = bool(b)
        return self

    def setGammaShape(self, v):
        self.gammaShape = float(v)
        return self

    def setSampleWithReplacement(self, b):
        self.sampleWithReplacement = bool(b)
        return self


class MllibLDA:
    """mllib.clustering.LDA as driven at LDAClustering.scala:37-61 (online optimizer only)."""

    def __init__(self, ctx: Context | None = None):
        self.k, self.maxIterations, self.docConcentration, self.topicConcentration = 10, 20, -1.0, -1.0
        self.seed = _java_string_hash("org.apache.spark.mllib.clustering.LDA")
        self.optimizer = OnlineLDAOptimizer()
        self.checkpointInterval = 10
        self.dtype = "f64"
        self._ctx = ctx

    def setOptimizer(self, opt):
        if isinstance(opt, str):
            if opt.lower() != "online":
                raise ValueError(f"Only em, online are supported but got {opt}." if opt.lower() != "em"
                                 else "optimizer 'em' (EMLDAOptimizer) is out of scope for this build")
            opt = OnlineLDAOptimizer()
        self.optimizer = opt
        return self

    def setK(self, k):
        if int(k) <= 1:
            raise ValueError(f"LDA k (number of clusters) must be > 1, but was set to {k}")
        self.k = int(k)
        return self

    def setMaxIterations(self, n):
        if int(n) < 0:
            raise ValueError(f"Maximum of iterations must be nonnegative, but was set to {n}")
        self.maxIterations = int(n)
        return self

    def setDocConcentration(self, a):
        self.docConcentration = a
        return self

    def setTopicConcentration(self, e):
        self.topicConcentration = float(e)
        return self

    def setCheckpointInterval(self, n):
        self.checkpointInterval = int(n)  # EM-only in Spark; accepted and ignored here
        return self

    def setSeed(self, s):
        self.seed = int(s)
        return self

    def run(self, corpus) -> LDAModel:
        o = self.optimizer
        ctx = self._ctx or Context.get()
        d, _ = _as_device(ctx, corpus, _DTYPES[self.dtype])
        total = int(ctx.allreduce([float(d.num_rows)])[0]) if ctx.n_ranks > 1 else d.num_rows
        h = LdaHandle(ctx, self.k, d.num_cols, doc_concentration=self.docConcentration,
                      topic_concentration=self.topicConcentration, tau0=o.tau0, kappa=o.kappa,
                      mini_batch_fraction=o.miniBatchFraction, gamma_shape=o.gammaShape,
                      optimize_doc_concentration=o.optimizeDocConcentration,
                      sample_with_replacement=o.sampleWithReplacement, seed=self.seed, dtype=self.dtype)
        h.set_corpus(d, total)
        h.init_random(self.seed)
        for _ in range(self.maxIterations):
            h.next(stats=False)
        return LDAModel(h)


def reference_mini_batch_fraction(corpus_size):
    """LDAClustering.scala:43: 0.05 + 1.0 / actualCorpusSize."""
    return 0.05 + 1.0 / float(corpus_size)


def rho(tau0, kappa, iteration):
    return math.pow(tau0 + iteration, -kappa)
