/*
 * lda_oracle.c — CPU ORACLE (test infrastructure + bench cpu_baseline only; never the product).
 *
 * Plain-C, fp64 restatement of [U] spark-mllib 2.4.3 OnlineLDAOptimizer.variationalTopicInference
 * (TextClustering/build.sbt:10; reached from lda.run at LDAClustering.scala:61 and from
 * toLocal.topicDistribution at LDALoader.scala:108) and Breeze 0.13.2 digamma, with the unscaled
 * expElogβ and the 1e-100 φ epsilon exactly as upstream.  OpenMP over documents, one document per
 * task like Spark's per-partition loop.  Mirrors oracle/oracle.py (which is pinned by the golden
 * fixtures); tests/test_c_oracle.py checks the two agree.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static double breeze_digamma(double x) {
  double r = 0.0;
  while (x <= 5.0) {
    r -= 1.0 / x;
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  const double t = f * (-1 / 12.0 + f * (1 / 120.0 + f * (-1 / 252.0 + f * (1 / 240.0 + f * (-1 / 132.0 +
                   f * (691 / 32760.0 + f * (-1 / 12.0 + f * 3617 / 8160.0)))))));
  return r + log(x) - 0.5 / x + t;
}

/* exp(dirichletExpectation(gamma)) for one document */
static void exp_dirichlet(const double* g, int k, double* out) {
  double s = 0.0;
  for (int t = 0; t < k; ++t) s += g[t];
  const double ps = breeze_digamma(s);
  for (int t = 0; t < k; ++t) out[t] = exp(breeze_digamma(g[t]) - ps);
}

/* variationalTopicInference for one doc; B is the gathered nnz×k block. Returns iterations. */
static int vti(int nnz, const double* cts, const double* B, const double* alpha, int k, double* gamma,
               double* eth, double* phi, double* tmp, int max_iter) {
  exp_dirichlet(gamma, k, eth);
  for (int n = 0; n < nnz; ++n) {
    double a = 0.0;
    for (int t = 0; t < k; ++t) a += B[(size_t)n * k + t] * eth[t];
    phi[n] = a + 1e-100;
  }
  double change = 1.0;
  int it = 0;
  while (change > 1e-3) {
    for (int t = 0; t < k; ++t) tmp[t] = 0.0;
    for (int n = 0; n < nnz; ++n) {
      const double w = cts[n] / phi[n];
      const double* row = B + (size_t)n * k;
      for (int t = 0; t < k; ++t) tmp[t] += row[t] * w;
    }
    change = 0.0;
    for (int t = 0; t < k; ++t) {
      const double g = eth[t] * tmp[t] + alpha[t];
      change += fabs(g - gamma[t]);
      gamma[t] = g;
    }
    change /= k;
    exp_dirichlet(gamma, k, eth);
    for (int n = 0; n < nnz; ++n) {
      double a = 0.0;
      const double* row = B + (size_t)n * k;
      for (int t = 0; t < k; ++t) a += row[t] * eth[t];
      phi[n] = a + 1e-100;
    }
    ++it;
    if (max_iter > 0 && it >= max_iter) break;
  }
  return it;
}

/*
 * E-step over `n` documents (rows doc_ids[i] of the CSR).  exp_elog_beta is V×k (Spark's
 * orientation).  gamma0/gamma_out are n×k.  Returns Σ iterations; iters_out (n) may be NULL.
 */
int64_t oracle_estep(int64_t n, const int64_t* indptr, const int32_t* indices, const double* values,
                     const int64_t* doc_ids, const double* exp_elog_beta, int k, const double* alpha,
                     const double* gamma0, double* gamma_out, int32_t* iters_out, int n_threads,
                     int max_iter) {
  int64_t total = 0;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
#pragma omp parallel reduction(+ : total)
  {
    size_t cap = 0;
    double *B = NULL, *cts = NULL, *phi = NULL;
    double* eth = (double*)malloc(sizeof(double) * k);
    double* tmp = (double*)malloc(sizeof(double) * k);
#pragma omp for schedule(dynamic, 4)
    for (int64_t i = 0; i < n; ++i) {
      const int64_t d = doc_ids ? doc_ids[i] : i;
      const int64_t s = indptr[d];
      const int nnz = (int)(indptr[d + 1] - s);
      double* g = gamma_out + (size_t)i * k;
      memcpy(g, gamma0 + (size_t)i * k, sizeof(double) * k);
      int nz = 0;
      for (int j = 0; j < nnz; ++j) nz |= values[s + j] != 0.0;
      if (!nz) {
        for (int t = 0; t < k; ++t) g[t] = 0.0;
        if (iters_out) iters_out[i] = 0;
        continue;
      }
      if ((size_t)nnz > cap) {
        cap = (size_t)nnz;
        B = (double*)realloc(B, sizeof(double) * cap * k);
        cts = (double*)realloc(cts, sizeof(double) * cap);
        phi = (double*)realloc(phi, sizeof(double) * cap);
      }
      for (int j = 0; j < nnz; ++j) {
        memcpy(B + (size_t)j * k, exp_elog_beta + (size_t)indices[s + j] * k, sizeof(double) * k);
        cts[j] = values[s + j];
      }
      const int it = vti(nnz, cts, B, alpha, k, g, eth, phi, tmp, max_iter);
      if (iters_out) iters_out[i] = it;
      total += it;
    }
    free(B);
    free(cts);
    free(phi);
    free(eth);
    free(tmp);
  }
  return total;
}

static double breeze_trigamma(double x) {
  double r = 0.0;
  while (x <= 5.0) {
    r += 1.0 / (x * x);
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  const double t = f * (1 / 6.0 + f * (-1 / 30.0 + f * (1 / 42.0 + f * (-1 / 30.0 + f * (5 / 66.0 +
                   f * (-691 / 2730.0 + f * (7 / 6.0 - f * 3617 / 510.0)))))));
  return r + 1.0 / x + f / 2.0 + t / x;
}

/*
 * One [U] OnlineLDAOptimizer.submitMiniBatch + updateLambda (+ updateAlpha), Spark's structure:
 * expElogβ from λ; per thread (≙ partition) a DENSE k×V stat, logphat and a non-empty count; the
 * E-step per member; the thread stats summed (≙ treeReduce); batchResult = stat ⊙ expElogβ;
 * λ ← (1−ρ)λ + ρ(batchResult·scale + η); α Newton step on logphat / n.  lam is k×V (Spark's internal
 * orientation) and alpha (k) are updated in place.  Returns Σ inner iterations (−1: no non-empty doc).
 */
int64_t oracle_minibatch(int64_t n, const int64_t* indptr, const int32_t* indices, const double* values,
                         const int64_t* doc_ids, const double* gamma0, int k, int64_t V, double* lam,
                         double* alpha, double eta, double rho, double scale, int optimize_alpha,
                         int n_threads) {
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
  /* expElogβ, V×k (the E-step gathers rows) */
  double* eeb = (double*)malloc(sizeof(double) * (size_t)V * k);
  double* psic = (double*)malloc(sizeof(double) * k);
  for (int t = 0; t < k; ++t) {
    double s = 0.0;
    const double* row = lam + (size_t)t * V;
    for (int64_t v = 0; v < V; ++v) s += row[v];
    psic[t] = breeze_digamma(s);
  }
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < V; ++v)
    for (int t = 0; t < k; ++t) eeb[(size_t)v * k + t] = exp(breeze_digamma(lam[(size_t)t * V + v]) - psic[t]);
  int nt = 1;
#ifdef _OPENMP
  nt = omp_get_max_threads();
#endif
  double** stats = (double**)calloc((size_t)nt, sizeof(double*));
  double* lph = (double*)calloc((size_t)nt * (k + 1), sizeof(double));
  int64_t total = 0;
#pragma omp parallel reduction(+ : total)
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    double* stat = (double*)calloc((size_t)k * V, sizeof(double));  /* k×V, like Spark's partition stat */
    stats[tid] = stat;
    double* lp = lph + (size_t)tid * (k + 1);
    size_t cap = 0;
    double *B = NULL, *cts = NULL, *phi = NULL;
    double* eth = (double*)malloc(sizeof(double) * k);
    double* tmp = (double*)malloc(sizeof(double) * k);
    double* g = (double*)malloc(sizeof(double) * k);
#pragma omp for schedule(dynamic, 4)
    for (int64_t i = 0; i < n; ++i) {
      const int64_t d = doc_ids[i];
      const int64_t s = indptr[d];
      const int nnz = (int)(indptr[d + 1] - s);
      int nz = 0;
      for (int j = 0; j < nnz; ++j) nz |= values[s + j] != 0.0;
      if (!nz) continue;
      if ((size_t)nnz > cap) {
        cap = (size_t)nnz;
        B = (double*)realloc(B, sizeof(double) * cap * k);
        cts = (double*)realloc(cts, sizeof(double) * cap);
        phi = (double*)realloc(phi, sizeof(double) * cap);
      }
      for (int j = 0; j < nnz; ++j) {
        memcpy(B + (size_t)j * k, eeb + (size_t)indices[s + j] * k, sizeof(double) * k);
        cts[j] = values[s + j];
      }
      memcpy(g, gamma0 + (size_t)i * k, sizeof(double) * k);
      total += vti(nnz, cts, B, alpha, k, g, eth, phi, tmp, 0);
      /* stat(::, ids) += eθ ⊗ (cts / φ) ; logphat += dirichletExpectation(γ) */
      for (int j = 0; j < nnz; ++j) {
        const double w = cts[j] / phi[j];
        const int64_t v = indices[s + j];
        for (int t = 0; t < k; ++t) stat[(size_t)t * V + v] += eth[t] * w;
      }
      double gs = 0.0;
      for (int t = 0; t < k; ++t) gs += g[t];
      const double pg = breeze_digamma(gs);
      for (int t = 0; t < k; ++t) lp[t] += breeze_digamma(g[t]) - pg;
      lp[k] += 1.0;
    }
    free(B);
    free(cts);
    free(phi);
    free(eth);
    free(tmp);
    free(g);
  }
  /* treeReduce(elementWiseSum) */
  double* stat = stats[0];
  for (int p = 1; p < nt; ++p) {
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < (int64_t)k * V; ++e) stat[e] += stats[p][e];
    free(stats[p]);
  }
  double* logphat = (double*)calloc((size_t)k + 1, sizeof(double));
  for (int p = 0; p < nt; ++p)
    for (int t = 0; t <= k; ++t) logphat[t] += lph[(size_t)p * (k + 1) + t];
  const double N = logphat[k];
  if (N > 0) {
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < V; ++v)
      for (int t = 0; t < k; ++t) {
        const size_t e = (size_t)t * V + v;
        lam[e] = (1.0 - rho) * lam[e] + rho * (stat[e] * eeb[(size_t)v * k + t] * scale + eta);
      }
    if (optimize_alpha) { /* updateAlpha: one Newton step, applied only if α + ρ·dα > 0 everywhere */
      double as = 0.0;
      for (int t = 0; t < k; ++t) as += alpha[t];
      const double psa = breeze_digamma(as);
      double* gr = (double*)malloc(sizeof(double) * k);
      double* q = (double*)malloc(sizeof(double) * k);
      double a1 = 0.0, a2 = 0.0;
      for (int t = 0; t < k; ++t) {
        gr[t] = N * (-(breeze_digamma(alpha[t]) - psa) + logphat[t] / N);
        q[t] = -N * breeze_trigamma(alpha[t]);
        a1 += gr[t] / q[t];
        a2 += 1.0 / q[t];
      }
      const double c = N * breeze_trigamma(as);
      const double b = a1 / (1.0 / c + a2);
      int ok = 1;
      for (int t = 0; t < k; ++t) {
        gr[t] = -(gr[t] - b) / q[t];
        ok &= (rho * gr[t] + alpha[t] > 0.0);
      }
      if (ok)
        for (int t = 0; t < k; ++t) alpha[t] += rho * gr[t];
      free(gr);
      free(q);
    }
  } else {
    total = -1;
  }
  free(stat);
  free(stats);
  free(lph);
  free(logphat);
  free(eeb);
  free(psic);
  return total;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
