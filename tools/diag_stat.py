import os, sys, numpy as np
sys.path.insert(0, 'spark-text-clustering_amd'); sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import stc
from oracle import oracle as O
from helpers import random_corpus
ctx = stc.Context.get(0)
for k, maxnnz in ((16, 300), (16, 200), (100, 180)):
    rng = np.random.default_rng(10 + k)
    D, V = 48, 2048
    corpus = random_corpus(rng, D, V, 1, maxnnz, empty_every=13)
    lam = rng.gamma(100.0, 0.01, size=(V, k)); g0 = rng.gamma(100.0, 0.01, size=(D, k))
    eeb = O.topics_exp_elog_beta(lam); alpha = np.full(k, 1.0 / k)
    stat_o = np.zeros((V, k))
    for i in range(D):
        cid, cts = corpus.row(i)
        if cid.size == 0: continue
        g, ss, it = O.variational_topic_inference(cid, cts, eeb, alpha, g0[i]); np.add.at(stat_o, cid, ss.T)
    for kern in ("wave", "wg"):
        if kern == "wg": os.environ["STC_DISABLE_WAVE"] = "1"
        else: os.environ.pop("STC_DISABLE_WAVE", None)
        h = stc.LdaHandle(ctx, k, V, dtype="f32")
        d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32); h.set_corpus(d, D); h.set_topics(lam)
        gam, stat, its = h.estep(np.arange(D), g0, want_stat=True)
        nz = stat_o > 1e-8 * stat_o.max()
        rel = np.abs(stat - stat_o) / np.maximum(stat_o, 1e-30)
        bad = np.argwhere(nz & (rel > 1e-2))
        print(f"k={k} maxnnz={maxnnz} {kern}: max rel {rel[nz].max():.3e}, bad entries {len(bad)}, terms {np.unique(bad[:,0])[:10] if len(bad) else []}", flush=True)
        if len(bad):
            v = bad[0][0]
            docs = [i for i in range(D) if v in corpus.row(i)[0]]
            print("   term", v, "in docs", docs, "nnz", [corpus.row(i)[0].size for i in docs])
            print("   got", stat[v][:6], "\n   exp", stat_o[v][:6])
