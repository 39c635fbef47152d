import os, sys, time, numpy as np
sys.path.insert(0, 'spark-text-clustering_amd'); sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import stc
from oracle import oracle as O
from helpers import random_corpus
ctx = stc.Context.get(0)
for k in (16, 100):
    rng = np.random.default_rng(10 + k)
    D, V = 24, 2048
    corpus = random_corpus(rng, D, V, 1, 250)
    lam = rng.gamma(100.0, 0.01, size=(V, k)); g0 = rng.gamma(100.0, 0.01, size=(D, k))
    eeb = O.topics_exp_elog_beta(lam); alpha = np.full(k, 1.0 / k)
    res = {}
    for kern in ("wave", "wg"):
        if kern == "wg": os.environ["STC_DISABLE_WAVE"] = "1"
        else: os.environ.pop("STC_DISABLE_WAVE", None)
        h = stc.LdaHandle(ctx, k, V, dtype="f32", max_inner_iter=3000)
        d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32); h.set_corpus(d, D); h.set_topics(lam)
        t = time.time(); res[kern] = h.estep(np.arange(D), g0); print(k, kern, "time", time.time() - t, flush=True)
    for i in range(D):
        cid, cts = corpus.row(i)
        g, _, it = O.variational_topic_inference(cid, cts, eeb, alpha, g0[i])
        line = f"k={k} doc={i:2d} nnz={cid.size:3d} it_o={it:4d}"
        for kern in ("wave", "wg"):
            gg, _, its = res[kern]
            line += f" | {kern} it={its[i]:4d} rel={np.max(np.abs(gg[i]-g)/g):.2e}"
        print(line, flush=True)
