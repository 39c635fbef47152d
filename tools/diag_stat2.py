import os, sys, numpy as np
sys.path.insert(0, 'spark-text-clustering_amd'); sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import stc
from oracle import oracle as O
from helpers import random_corpus
ctx = stc.Context.get(0)
k = 16
rng = np.random.default_rng(26)
D, V = 4, 512
corpus = random_corpus(rng, D, V, 20, 40)
lam = rng.gamma(100.0, 0.01, size=(V, k)); g0 = rng.gamma(100.0, 0.01, size=(D, k))
eeb = O.topics_exp_elog_beta(lam); alpha = np.full(k, 1.0 / k)
os.environ.pop("STC_DISABLE_WAVE", None)
h = stc.LdaHandle(ctx, k, V, dtype="f32")
d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32); h.set_corpus(d, D); h.set_topics(lam)
for i in range(D):
    cid, cts = corpus.row(i)
    g, ss, it = O.variational_topic_inference(cid, cts, eeb, alpha, g0[i])
    gam, stat, its = h.estep(np.array([i]), g0[i:i+1], want_stat=True)
    ratio = stat[cid] / ss.T    # nnz × k
    print("doc", i, "nnz", cid.size, "gamma rel", np.abs(gam[0]-g).max()/g.max(), "iters", its[0], it)
    np.set_printoptions(precision=4, linewidth=200)
    print(" ratio per topic (mean over terms):", ratio.mean(0))
    print(" ratio per term  (mean over topics):", ratio.mean(1)[:12])
    print(" sum over topics got/exp:", (stat[cid].sum(1) / ss.sum(0))[:8])
