import sys, os, numpy as np
sys.path.insert(0, 'spark-text-clustering_amd'); sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import stc
from oracle import oracle as O
from helpers import golden_npz, golden_json
tf = golden_npz("en_idf.npz"); topics = golden_npz("en_topics.npz")["nwk"]; meta = golden_json("en_topicdist.json")
V = int(tf["vocab_size"])
corpus = stc.CsrMatrix(tf["indptr"], tf["indices"], tf["tf"].astype(np.float64), V)
exp = np.array([[float(x) for x in r] for r in meta["Result_EN_1591723228815"]])
nnz = np.diff(tf["indptr"])
ctx = stc.Context.get(0)
g0 = np.array([O.gamma_init(7, d, 5) for d in range(51)])
for dtype in ("f64", "f32"):
    model = stc.LDAModel.from_topics(topics, meta["docConcentration"], meta["topicConcentration"], seed=7, dtype=dtype, ctx=ctx)
    a = model.transform(corpus)
    b = model.transform(corpus, gamma0=g0)
    ea = np.abs(a - exp).max(1); eb = np.abs(b - exp).max(1)
    print(dtype, "rng-γ0 max err", ea.max(), "injected-γ0 max err", eb.max())
    bad = np.where(ea > 1e-5)[0]
    print(" bad docs (rng):", bad[:20], "nnz", nnz[bad[:20]])
    bad = np.where(eb > 1e-5)[0]
    print(" bad docs (inj):", bad[:20], "nnz", nnz[bad[:20]])
    print(" sample rows", a[bad[:2]] if len(bad) else None, exp[bad[:2]] if len(bad) else None)
# sub-corpus tests: single doc
for d in [0, 1, 10]:
    sub = corpus.rows([d])
    model = stc.LDAModel.from_topics(topics, meta["docConcentration"], meta["topicConcentration"], seed=7, dtype="f64", ctx=ctx)
    print("single doc", d, nnz[d], np.abs(model.transform(sub, gamma0=g0[d:d+1]) - exp[d]).max())
