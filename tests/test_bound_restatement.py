"""Independent pin of LocalLDAModel.logLikelihoodBound on a hand-sized case.

The bound has no artefact in the reference (no model there was trained by the online optimizer),
so the oracle's restatement is checked here against a second one written term by term from the
upstream formula with scalar loops, `math.lgamma` and scipy's digamma — nothing shared with
oracle/oracle.py except the inputs:

  corpusPart = Σ_d [ Σ_n c_n · logsumexp_k(Elogθ_dk + Elogβ_{v_n k})
                     + Σ_k (α_k − γ_dk) Elogθ_dk + Σ_k (lgamma γ_dk − lgamma α_k)
                     + lgamma Σα − lgamma Σγ_d ]
  topicsPart = Σ_{v,k} (η − λ_vk) Elogβ_vk + Σ_{v,k} (lgamma λ_vk − lgamma η)
               + Σ_k (lgamma(V·η) − lgamma Σ_v λ_vk)

with λ the V×k topicsMatrix, Elogβ_vk = ψ(λ_vk) − ψ(Σ_v λ_vk) and γ_d the E-step fixed point
([U] spark-mllib 2.4.3 LocalLDAModel.logLikelihoodBound / OnlineLDAOptimizer.variationalTopicInference).
"""
import math

import numpy as np
from scipy.special import digamma as _psi_exact


def psi(x):
    """Breeze 0.13.2 digamma, scalar: recurrence to x > 5, then the 8-term asymptotic series.  Spark
    evaluates the bound with it; it sits ≈1e-13 from the exact ψ (checked below), which is why the
    restatement uses it rather than scipy's."""
    r = 0.0
    while x <= 5.0:
        r -= 1.0 / x
        x += 1.0
    f = 1.0 / (x * x)
    t = f * (-1 / 12.0 + f * (1 / 120.0 + f * (-1 / 252.0 + f * (1 / 240.0 + f * (
        -1 / 132.0 + f * (691 / 32760.0 + f * (-1 / 12.0 + f * 3617 / 8160.0)))))))
    return r + math.log(x) - 0.5 / x + t


def test_breeze_digamma_restatement_is_digamma():
    for x in (0.05, 0.25, 1.0, 3.7, 5.0, 5.5, 40.0, 1e4):
        assert abs(psi(x) - _psi_exact(x)) <= 5e-13 * max(1.0, abs(_psi_exact(x)))


def _estep_scalar(ids, cts, lam, alpha, gamma0):
    V, k = len(lam), len(alpha)
    col = [sum(lam[v][t] for v in range(V)) for t in range(k)]
    eb = [[math.exp(psi(lam[v][t]) - psi(col[t])) for t in range(k)] for v in range(V)]
    g = list(gamma0)

    def etheta(g):
        s = psi(sum(g))
        return [math.exp(psi(x) - s) for x in g]

    et = etheta(g)
    phin = [sum(eb[v][t] * et[t] for t in range(k)) + 1e-100 for v in ids]
    while True:
        last = list(g)
        g = [et[t] * sum(eb[v][t] * c / p for v, c, p in zip(ids, cts, phin)) + alpha[t] for t in range(k)]
        et = etheta(g)
        phin = [sum(eb[v][t] * et[t] for t in range(k)) + 1e-100 for v in ids]
        if sum(abs(a - b) for a, b in zip(g, last)) / k <= 1e-3:
            return g


def _bound_scalar(docs, gamma0s, lam, alpha, eta):
    V, k = len(lam), len(alpha)
    col = [sum(lam[v][t] for v in range(V)) for t in range(k)]
    elogb = [[psi(lam[v][t]) - psi(col[t]) for t in range(k)] for v in range(V)]
    corpus = 0.0
    for (ids, cts), g0 in zip(docs, gamma0s):
        g = _estep_scalar(ids, cts, lam, alpha, g0)
        elt = [psi(x) - psi(sum(g)) for x in g]
        b = 0.0
        for v, c in zip(ids, cts):
            z = [elt[t] + elogb[v][t] for t in range(k)]
            m = max(z)
            b += c * (m + math.log(sum(math.exp(x - m) for x in z)))
        b += sum((alpha[t] - g[t]) * elt[t] for t in range(k))
        b += sum(math.lgamma(g[t]) - math.lgamma(alpha[t]) for t in range(k))
        b += math.lgamma(sum(alpha)) - math.lgamma(sum(g))
        corpus += b
    topics = 0.0
    for v in range(V):
        for t in range(k):
            topics += (eta - lam[v][t]) * elogb[v][t] + (math.lgamma(lam[v][t]) - math.lgamma(eta))
    for t in range(k):
        topics += math.lgamma(V * eta) - math.lgamma(col[t])
    return corpus + topics, corpus, topics


def test_topics_part_closed_form():
    """V = 3, k = 2: the topics part by hand, every lgamma/ψ written out."""
    from oracle import oracle as O

    lam = [[2.0, 0.5], [1.5, 3.0], [0.25, 1.0]]
    eta = 0.5
    c0, c1 = 2.0 + 1.5 + 0.25, 0.5 + 3.0 + 1.0
    eb = lambda v, t: psi(lam[v][t]) - psi((c0, c1)[t])  # noqa: E731
    hand = 0.0
    for v in range(3):
        for t in range(2):
            hand += (eta - lam[v][t]) * eb(v, t) + math.lgamma(lam[v][t]) - math.lgamma(eta)
    hand += (math.lgamma(1.5) - math.lgamma(c0)) + (math.lgamma(1.5) - math.lgamma(c1))
    _, corpus, topics = O.log_likelihood_bound([], [], np.array(lam), np.array([0.3, 0.7]), eta)
    assert corpus == 0.0
    assert abs(topics - hand) <= 1e-14 * abs(hand), (topics, hand)
    # the per-topic normaliser enters with a MINUS on lgamma Σ_v λ: a model with more mass has a
    # lower bound at equal shape, as the Dirichlet entropy term requires
    _, _, t2 = O.log_likelihood_bound([], [], np.array(lam) * 2.0, np.array([0.3, 0.7]), eta)
    assert np.isfinite(t2)


def test_bound_two_token_doc_matches_restatement():
    """One 2-token document over V = 3, k = 2: corpus and topics parts term by term."""
    from oracle import oracle as O

    lam = [[2.0, 0.5], [1.5, 3.0], [0.25, 1.0]]
    alpha = [0.3, 0.7]
    eta = 0.5
    docs = [([0, 2], [2.0, 1.0])]
    g0 = [[1.1, 0.9]]
    b_r, c_r, t_r = _bound_scalar(docs, g0, lam, alpha, eta)
    b_o, c_o, t_o = O.log_likelihood_bound([(np.array(i), np.array(c)) for i, c in docs],
                                           [np.array(g) for g in g0], np.array(lam), np.array(alpha), eta)
    assert abs(c_o - c_r) <= 1e-13 * abs(c_r), (c_o, c_r)
    assert abs(t_o - t_r) <= 1e-14 * abs(t_r), (t_o, t_r)
    assert abs(b_o - b_r) <= 1e-13 * abs(b_r), (b_o, b_r)
    lp = O.log_perplexity([(np.array(i), np.array(c)) for i, c in docs], [np.array(g) for g in g0],
                          np.array(lam), np.array(alpha), eta)
    assert abs(lp - (-b_r / 3.0)) <= 1e-13 * abs(lp)


def test_bound_random_small_corpus_matches_restatement():
    """A few random docs at V = 12, k = 3 (several E-step iterations per doc)."""
    from oracle import oracle as O

    rng = np.random.default_rng(3)
    V, k = 12, 3
    lam = rng.gamma(2.0, 1.0, size=(V, k)) + 0.1
    alpha = rng.uniform(0.1, 0.9, size=k)
    eta = 0.2
    docs = []
    for _ in range(4):
        ids = np.sort(rng.choice(V, size=int(rng.integers(1, 6)), replace=False))
        docs.append((ids, rng.integers(1, 5, ids.size).astype(np.float64)))
    g0 = [rng.gamma(100.0, 0.01, size=k) for _ in docs]
    b_r, c_r, t_r = _bound_scalar([(list(i), list(c)) for i, c in docs], [list(g) for g in g0],
                                  lam.tolist(), alpha.tolist(), eta)
    b_o, c_o, t_o = O.log_likelihood_bound(docs, g0, lam, alpha, eta)
    assert abs(c_o - c_r) <= 1e-12 * abs(c_r), (c_o, c_r)
    assert abs(t_o - t_r) <= 1e-13 * abs(t_r), (t_o, t_r)
