"""CPU emulation of the E-step's precision on BASELINE configs[0] (the books through HashingTF 2^18 + IDF(2)
with the 1e-4 floor, online LDA k = 20, 10 minibatches with tests/test_gpu_config1.py's injected λ₀,
membership and γ₀): the topicsMatrix error against the fp64 oracle for
  f32     every E-step operation in fp32 (the fp32 kernel's digamma_fast, fp32 sums) — the fp32 mode
  mix     fp32 expElogβ / eθ storage, products and sums; fp64 γ, ψ, exp and stop rule (VERDICT r5's suggestion)
  mixacc  fp32 expElogβ / eθ storage; fp64 products, sums, γ, ψ
and each with the documents past T fp32 iterations re-solved in fp64 (STC_MIXED).  numpy float32 arithmetic
stands in for the kernels' (other summation orders, the same rounding unit): the input to DESIGN.md §4's
mixed-mode design.  Test infrastructure only (imports oracle/).  Output: one JSON line.

    python tools/mixed_precision_emulation.py > profiles/r06_mixed_emulation.json
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'spark-text-clustering_amd')):
    sys.path.insert(0, p)
from oracle import oracle as O
from helpers import GOLDEN, golden_npz
K, ITERS, NF = 20, 10, 1 << 18
tf = golden_npz("en_idf.npz")
vocab = open(os.path.join(GOLDEN, "en_vocab.txt"), encoding="utf-8").read().split("\n")[:-1]
bucket = np.array([O.non_negative_mod(O.murmur3_x86_32(w.encode("utf-8"), 42, O.HASH_SPARK24), NF) for w in vocab], np.int64)
ip, ix, cnt = tf["indptr"], tf["indices"], tf["tf"]
indptr, idx, val = [0], [], []
for d in range(ip.size - 1):
    b = bucket[ix[ip[d]:ip[d + 1]]]
    u, inv = np.unique(b, return_inverse=True)
    c = np.zeros(u.size); np.add.at(c, inv, cnt[ip[d]:ip[d + 1]].astype(np.float64))
    idx.append(u.astype(np.int32)); val.append(c); indptr.append(indptr[-1] + u.size)
ip_o, ix_o, vv_o = np.array(indptr), np.concatenate(idx), np.concatenate(val)
idf_o, df_o, m_o = O.idf_fit(ip_o, ix_o, vv_o, NF, 2)
vals = O.idf_transform(ix_o, vv_o, idf_o, floor=1e-4)
D = ip_o.size - 1
rows = [(ix_o[ip_o[i]:ip_o[i+1]], vals[ip_o[i]:ip_o[i+1]]) for i in range(D)]
rng = np.random.default_rng(2020)
frac = 0.05 + 1.0 / D
lam0 = rng.gamma(100.0, 0.01, size=(NF, K))
batches = []
for _ in range(ITERS):
    ids = np.flatnonzero(rng.random(D) < frac)
    if ids.size == 0: ids = rng.choice(D, size=1)
    batches.append((ids, rng.gamma(100.0, 0.01, size=(ids.size, K))))

f32 = np.float32
def dg32(x):  # the fp32 kernel's digamma_fast
    x = x.astype(f32)
    num = (f32(3)*x + f32(12))*x + f32(11)
    den = ((x + f32(6))*x + f32(11))*x + f32(6)
    r = f32(1)/x + num/den
    y = x + f32(4); iy = f32(1)/y; f = iy*iy
    t = f*(f32(-1/12) + f*(f32(1/120) + f*(f32(-1/252) + f*(f32(1/240) + f*f32(-1/132)))))
    return (np.log(y).astype(f32) - f32(0.5)*iy + t - r).astype(f32)

def estep(ids, cts, eeb, alpha, g0, mode):
    # mode: 'f64' | 'f32' (all fp32) | 'mix' (fp32 B/eθ storage+products+sums, fp64 γ/ψ/exp/stop) | 'mixacc' (fp32 storage, fp64 sums)
    k = alpha.size
    if mode == 'f64':
        return O.variational_topic_inference(ids, cts, eeb, alpha, g0)
    B = eeb[ids].astype(f32)
    c32 = cts.astype(f32)
    if mode == 'f32':
        gamma = g0.astype(f32); a32 = alpha.astype(f32)
        et = np.exp(dg32(gamma) - dg32(np.array([gamma.sum()], f32))[0]).astype(f32)
        phi = (B @ et) + f32(1e-30)
        mc = 1.0; it = 0
        while mc > 1e-3:
            last = gamma.copy()
            gamma = (et * (B.T @ (c32 / phi)) + a32).astype(f32)
            et = np.exp(dg32(gamma) - dg32(np.array([gamma.sum()], f32))[0]).astype(f32)
            phi = (B @ et) + f32(1e-30)
            mc = float(np.sum(np.abs(gamma - last))) / k; it += 1
        return gamma.astype(np.float64), np.outer(et, c32/phi).astype(np.float64), it
    gamma = np.array(g0, np.float64)
    et64 = np.exp(O.dirichlet_expectation(gamma))
    def phi_of(et64):
        et = et64.astype(f32)
        if mode == 'mix': return (B @ et).astype(np.float64) + 1e-100
        return B.astype(np.float64) @ et.astype(np.float64) + 1e-100
    def s_of(r):
        if mode == 'mix': return (B.T @ r.astype(f32)).astype(np.float64)
        return B.astype(np.float64).T @ r.astype(f32).astype(np.float64)
    phi = phi_of(et64); mc = 1.0; it = 0
    while mc > 1e-3:
        last = gamma.copy()
        gamma = et64 * s_of(cts / phi) + alpha
        et64 = np.exp(O.dirichlet_expectation(gamma))
        phi = phi_of(et64)
        mc = np.sum(np.abs(gamma - last)) / k; it += 1
    return gamma, np.outer(et64, cts/phi), it

def run(mode, resolve_above=None):
    alpha, eta = O.resolve_alpha_eta(K)
    st = O.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha, eta=eta, corpus_size=D, mini_batch_fraction=frac, optimize_doc_concentration=False)
    its = []
    for bids, g0s in batches:
        st.iteration += 1
        eeb = np.exp(O.dirichlet_expectation(st.lam)).T
        stat = np.zeros((K, NF))
        for i, g0 in zip(bids, g0s):
            ids, cts = rows[i]
            gamma, ss, it = estep(ids, cts, eeb, st.alpha, g0, mode)
            if resolve_above is not None and it > resolve_above:
                gamma, ss, it2 = estep(ids, cts, eeb, st.alpha, g0, 'f64')
            np.add.at(stat.T, ids, ss.T)
            its.append(it)
        bs = int(math.ceil(frac * D))
        O.update_lambda(st, stat * eeb.T, bs)
    return st.lam.T, its

ref, its = run('f64')
out = {"fp64_iterations_top10": sorted(its)[-10:], "documents": len(its), "topicsMatrix_rel_err": {}}
for mode, T in [('f32', None), ('mix', None), ('mixacc', None), ('mix', 1000), ('mix', 500), ('f32', 1000),
                ('f32', 500)]:
    lam, _ = run(mode, T)
    out["topicsMatrix_rel_err"][f"{mode}" + (f"+resolve>{T}" if T else "")] = float(np.max(np.abs(lam - ref) / ref))
print(json.dumps(out))
