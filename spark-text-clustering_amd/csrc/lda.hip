// lda.hip — online variational-Bayes LDA kernels for gfx950 (K6–K12 of SURVEY.md §7).
//
// Each kernel restates one upstream function of spark-mllib 2.4.3 (TextClustering/build.sbt:10),
// reached from lda.run(corpus) at LDAClustering.scala:61 and toLocal.topicDistribution at
// LDALoader.scala:108:
//   k_estep          [U] OnlineLDAOptimizer.variationalTopicInference (+ LocalLDAModel
//                    logLikelihoodBound corpusPart when BOUND)
//   k_sstats/k_fixup [U] submitMiniBatch `stat(::, ids) += sstats` + treeReduce (per device)
//   k_lambda_eeb     [U] submitMiniBatch `statsSum ⊙ expElogβᵀ` + updateLambda, and in the same
//                    pass the rows of exp(LDAUtils.dirichletExpectation(λ)) (+ .t)
//   k_update_alpha   [U] updateAlpha (Newton step on α)
//   k_topics_bound   [U] logLikelihoodBound topicsPart
//
// Numerics: expElogβ is stored ROW-SCALED and without its per-topic factor,
// Bp[v][t] = exp(ψ(λ_vt) − m_v) with m_v = max_t ψ(λ_vt); the E-step iterates with
// eθ' = exp(ψ(γ_t) − ψ(max γ) − ψ(Σ_v λ_vt)).  Bp·eθ' = e^{-m_v}·expElogβ·exp(ψ(γ) − ψ(max γ)), so
// both scales cancel exactly in γ ← eθ ⊙ Bᵀ(cts/(B·eθ)) + α and in batchResult = stat ⊙ expElogβ:
// the recursion is Spark's, but nothing underflows in fp32 (Spark's unscaled exp(Elogβ) reaches
// 1e-50 for rare terms).  The bound adds m_v and max E[log θ] back in fp64.
#include "lda_kernels.h"

namespace stc {
namespace lda {

template <typename T>
struct VecOf;
template <>
struct VecOf<float> {
  typedef float type __attribute__((ext_vector_type(4)));
  static constexpr int W = 4;
};
template <>
struct VecOf<double> {
  typedef double type __attribute__((ext_vector_type(2)));
  static constexpr int W = 2;
};

// Spark adds 1e-100 to φ = B·eθ (unscaled).  In the row/doc-scaled space that epsilon becomes
// ε'_n = 1e-100 / (exp(m_v)·exp(max E[log θ])) = exp(LOG_EPS − m_v − lmax): it keeps Spark's
// behaviour for terms whose unscaled expElogβ underflows (they contribute nothing in Spark).
constexpr double LOG_EPS = -230.25850929940458;  // ln(1e-100)
template <typename T>
__device__ __forceinline__ T eps_floor() { return T(1.17549435e-38); }  // FLT_MIN (f32 only)
template <>
__device__ __forceinline__ double eps_floor<double>() { return 0.0; }

template <typename T, typename VT>
__device__ __forceinline__ T hsum(VT v);
template <>
__device__ __forceinline__ float hsum<float, VecOf<float>::type>(VecOf<float>::type v) {
  return (v.x + v.y) + (v.z + v.w);
}
template <>
__device__ __forceinline__ double hsum<double, VecOf<double>::type>(VecOf<double>::type v) {
  return v.x + v.y;
}

__device__ __forceinline__ float exp_t(float x) { return __expf(x); }
__device__ __forceinline__ float psi_t(float x) { return digamma_fast(x); }
__device__ __forceinline__ double psi_t(double x) { return digamma_t<double>(x); }
__device__ __forceinline__ double exp_t(double x) { return exp(x); }
// eθ' = exp(x − ψc_t): fp64 subtracts ψc_t in the argument, fp32 multiplies by exp(−ψc_t) (EStepArgs::psic)
__device__ __forceinline__ double exp_minus_psic(double x, const double* psic, int k, int t) {
  (void)k;
  return exp(x - psic[t]);
}
__device__ __forceinline__ float exp_minus_psic(float x, const double* psic, int k, int t) {
  return __expf(x) * (float)psic[k + t];
}

// ---------------------------------------------------------------------------------------
// Block (256 threads = 4 waves) reduction of (sum, sum, max) in a fixed order: deterministic.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void block_reduce3(double& a, double& b, double& c, double* s_red) {
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_max(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_red[w * 4 + 0] = a;
    s_red[w * 4 + 1] = b;
    s_red[w * 4 + 2] = c;
  }
  __syncthreads();
  a = (s_red[0] + s_red[4]) + (s_red[8] + s_red[12]);
  b = (s_red[1] + s_red[5]) + (s_red[9] + s_red[13]);
  c = fmax(fmax(s_red[2], s_red[6]), fmax(s_red[10], s_red[14]));
  __syncthreads();
}

template <typename T>
__host__ __device__ constexpr int part_elems(int kp) {
  return (256 * VecOf<T>::W > kp) ? 256 * VecOf<T>::W : kp;
}

template <typename T>
size_t estep_lds_bytes(int kp, int lds_rows, int P) {
  size_t b = 0;
  b += 2 * (size_t)kp * sizeof(T);                 // eth, gam
  b += (size_t)part_elems<T>(kp) * sizeof(T);      // partial column sums
  b += 16 * sizeof(double);                        // reduction scratch
  b += (size_t)lds_rows * sizeof(int32_t);         // ids   (lds_rows % 4 == 0)
  b += 3 * (size_t)lds_rows * sizeof(T);           // cts, r, ln(1e-100) − m_v
  b += (size_t)lds_rows * P * sizeof(T);           // the document block B
  return b;
}

template <typename T>
int estep_lds_rows(int k, int kp, int P) {
  (void)k;
  const size_t fixed = estep_lds_bytes<T>(kp, 0, P);
  const size_t per_row = sizeof(int32_t) + 3 * sizeof(T) + (size_t)P * sizeof(T);
  if (fixed >= (size_t)kLdsBudget) return 0;
  int rows = (int)(((size_t)kLdsBudget - fixed) / per_row);
  return rows & ~3;
}

// ---------------------------------------------------------------------------------------
// K6: the E-step.  One 256-thread workgroup per document; the hardware dispatcher balances the
// data-dependent trip counts.  LDS=true keeps the gathered nnz×k block in LDS (rows padded to
// P with P/W odd ⇒ conflict-free row-per-lane ds_read_b128); LDS=false streams it from L2.
// Per inner iteration: φ_n = B_n·eθ' (row per lane), r_n = cts_n/φ_n, s = Bᵀr (column groups ×
// row subsets, partials in LDS), γ = eθ'⊙s + α, eθ' = exp(ψ(γ) − ψ(max γ)), meanΔγ ≤ 1e-3 stops.
// ---------------------------------------------------------------------------------------
template <typename T, bool STATS, bool BOUND, bool LDS>
__device__ __forceinline__ void estep_doc(const EStepArgs<T>& a, unsigned char* smem, int64_t slot,
                                          int64_t mem, int64_t row, int64_t s0, int nnz, int64_t e0) {
  using VT = typename VecOf<T>::type;
  constexpr int W = VecOf<T>::W;
  const int tid = threadIdx.x;
  const int k = a.k, kp = a.kp, ncg = kp / W, P = a.P;
  const int rows_cap = a.lds_rows;

  T* s_eth = reinterpret_cast<T*>(smem);
  T* s_gam = s_eth + kp;
  T* s_part = s_gam + kp;
  double* s_red = reinterpret_cast<double*>(s_part + part_elems<T>(kp));
  int32_t* s_ids = reinterpret_cast<int32_t*>(s_red + 16);
  T* s_cts = reinterpret_cast<T*>(s_ids + rows_cap);
  T* s_r = s_cts + rows_cap;
  T* s_lse = s_r + rows_cap;
  T* s_B = s_lse + rows_cap;

  const int32_t* ids = LDS ? s_ids : a.indices + s0;
  const T* cts = LDS ? s_cts : a.values + s0;
  T* rr = LDS ? s_r : a.r + e0;

  // -- load ids / counts (LDS) and detect an all-zero document (Spark's numNonzeros == 0)
  int nz = 0;
  for (int n = tid; n < nnz; n += kBlock) {
    const int32_t id = a.indices[s0 + n];
    const T c = a.values[s0 + n];
    if (LDS) {
      s_ids[n] = id;
      s_cts[n] = c;
      s_lse[n] = (T)(LOG_EPS - a.logscale[id]);
    }
    nz |= (c != T(0));
  }
  const bool nonempty = __syncthreads_or(nz) != 0;
  if (!nonempty) {
    for (int t = tid; t < k; t += kBlock) {
      if (a.gamma) a.gamma[mem * k + t] = T(0);
      if (STATS) a.elogth[slot * k + t] = T(0);
    }
    if (STATS)
      for (int t = tid; t < kp; t += kBlock) a.eth[slot * kp + t] = T(0);
    for (int n = tid; n < nnz; n += kBlock) {
      a.r[e0 + n] = T(0);
      if (STATS) {
        a.keys[e0 + n] = (uint32_t)a.indices[s0 + n];
        a.vals[e0 + n] = entry_val<T>(slot, e0 + n, T(0));
      }
    }
    if (tid == 0) {
      if (a.iters) a.iters[mem] = 0;
      if (a.nonempty) a.nonempty[mem] = 0;
      if (BOUND) a.bound[mem] = 0.0;
    }
    return;
  }

  // -- gather the document block B[n][:] = Bp[ids[n]][:] into LDS
  if (LDS) {
    const int total = nnz * ncg;
#pragma unroll 4
    for (int w = tid; w < total; w += kBlock) {
      const int n = w / ncg;
      const int c = w - n * ncg;
      const VT v = *reinterpret_cast<const VT*>(a.Bp + (int64_t)s_ids[n] * kp + c * W);
      *reinterpret_cast<VT*>(s_B + n * P + c * W) = v;
    }
  }

  // -- γ₀ (injected or counter RNG) and eθ'
  uint64_t stream = 0;
  if (!a.gamma0) {
    const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem)
                                         : (uint64_t)(a.doc_id_base + row);
    stream = doc_stream(a.seed, key);
  }
  double gsum = 0.0, gmax = -INFINITY, dummy = 0.0;
  for (int t = tid; t < kp; t += kBlock) {
    T g = T(0);
    if (t < k) {
      g = a.gamma0 ? a.gamma0[mem * k + t] : (T)gamma_sample(stream, t, a.gamma_shape);
      gsum += (double)g;
      gmax = fmax(gmax, (double)g);
    }
    s_gam[t] = g;
  }
  block_reduce3(gsum, dummy, gmax, s_red);
  T lmax = psi_t((T)gmax) - psi_t((T)gsum);  // max_t E[log θ_t]
  {
    const T psimax = psi_t((T)gmax);
    for (int t = tid; t < kp; t += kBlock)
      s_eth[t] = t < k ? exp_minus_psic(psi_t(s_gam[t]) - psimax, a.psic, k, t) : T(0);
  }
  __syncthreads();

  const int R = ncg >= kBlock ? 1 : kBlock / ncg;  // row subsets in the Bᵀr product
  const int nwork = R * ncg;
  int it = 0;
  bool done = false;
  double b_tok = 0.0, c_tok = 0.0;  // BOUND: Σ cts·(log φ'_n + m_v), Σ cts
  while (true) {
    // Phase A: φ_n = B_n · eθ', r_n = cts_n / φ_n
    for (int n = tid; n < nnz; n += kBlock) {
      const T* Brow = LDS ? s_B + n * P : a.Bp + (int64_t)ids[n] * kp;
      VT acc = (VT)T(0);
      for (int c = 0; c < ncg; ++c)
        acc += *reinterpret_cast<const VT*>(Brow + c * W) * *reinterpret_cast<const VT*>(s_eth + c * W);
      const T dot = hsum<T, VT>(acc);
      const T lse = LDS ? s_lse[n] : (T)(LOG_EPS - a.logscale[ids[n]]);
      const T phi = dot + fmax(exp_t(lse - lmax), eps_floor<T>());
      const T cn = cts[n];
      rr[n] = cn / phi;
      if (BOUND && (done || it >= a.max_iter) && cn != T(0)) {  // logSumExp: no epsilon
        b_tok += (double)cn * ((double)log(fmax(dot, eps_floor<T>())) + a.logscale[ids[n]]);
        c_tok += (double)cn;
      }
    }
    __syncthreads();
    if (done || it >= a.max_iter) break;

    // Phase B: partial column sums s_j[c] = Σ_{n ≡ j mod R} B[n][c]·r_n
    for (int w = tid; w < nwork; w += kBlock) {
      const int c = w % ncg;
      const int j = w / ncg;
      VT acc = (VT)T(0);
      for (int n = j; n < nnz; n += R) {
        const T* Brow = LDS ? s_B + n * P : a.Bp + (int64_t)ids[n] * kp;
        acc += *reinterpret_cast<const VT*>(Brow + c * W) * rr[n];
      }
      *reinterpret_cast<VT*>(s_part + j * kp + c * W) = acc;
    }
    __syncthreads();

    // Phase C: γ ← eθ' ⊙ s + α ; Σ|Δγ|, Σγ, max γ
    double dsum = 0.0;
    gsum = 0.0;
    gmax = -INFINITY;
    for (int t = tid; t < k; t += kBlock) {
      T s = T(0);
      for (int j = 0; j < R; ++j) s += s_part[j * kp + t];
      const T g = s_eth[t] * s + (T)a.alpha[t];
      dsum += fabs((double)g - (double)s_gam[t]);
      s_gam[t] = g;
      gsum += (double)g;
      gmax = fmax(gmax, (double)g);
    }
    block_reduce3(dsum, gsum, gmax, s_red);

    // Phase D: eθ' = exp(ψ(γ) − ψ(max γ)) ; meanGammaChange = Σ|Δγ| / k
    const T psimax = psi_t((T)gmax);
    lmax = psimax - psi_t((T)gsum);
    for (int t = tid; t < k; t += kBlock) s_eth[t] = exp_minus_psic(psi_t(s_gam[t]) - psimax, a.psic, k, t);
    ++it;
    done = dsum / (double)k <= 1e-3;
    __syncthreads();
  }

  // -- outputs
  const double psisum = digamma_t<double>(gsum);
  for (int t = tid; t < k; t += kBlock) {
    if (a.gamma) a.gamma[mem * k + t] = s_gam[t];
    if (STATS) a.elogth[slot * k + t] = (T)(digamma_t<double>((double)s_gam[t]) - psisum);
  }
  if (STATS) {
    for (int t = tid; t < kp; t += kBlock) a.eth[slot * kp + t] = s_eth[t];
    for (int n = tid; n < nnz; n += kBlock) {
      const T rv = LDS ? s_r[n] : a.r[e0 + n];  // the L2 path wrote r before the block barrier
      if (LDS) a.r[e0 + n] = rv;
      a.keys[e0 + n] = (uint32_t)ids[n];
      a.vals[e0 + n] = entry_val<T>(slot, e0 + n, rv);
    }
  }
  if (tid == 0) {
    if (a.iters) a.iters[mem] = it;
    if (a.nonempty) a.nonempty[mem] = 1;
  }
  if (BOUND) {
    // E[log p(doc|θ,β)] = Σ_n cts_n (log φ'_n + m_v + max E[log θ]);  E[log p(θ|α) − log q(θ|γ)]
    const double elog_max = digamma_t<double>(gmax) - psisum;
    double topic = 0.0, asum = 0.0, dummy2 = -INFINITY;
    for (int t = tid; t < k; t += kBlock) {
      const double g = (double)s_gam[t], al = a.alpha[t];
      const double el = digamma_t<double>(g) - psisum;
      topic += (al - g) * el + (lgamma(g) - lgamma(al));
      asum += al;
    }
    double tok = b_tok + c_tok * elog_max;
    block_reduce3(tok, topic, dummy2, s_red);
    double as2 = asum, z = 0.0, dz = -INFINITY;
    block_reduce3(as2, z, dz, s_red);
    if (tid == 0) a.bound[mem] = tok + topic + (lgamma(as2) - lgamma(gsum));
  }
}

template <typename T, bool STATS, bool BOUND>
__global__ __launch_bounds__(kBlock) void k_estep(EStepArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if ((int64_t)blockIdx.x >= a.n) return;
  const int64_t slot = a.slot0 + blockIdx.x;
  const int64_t mem = a.orig ? (int64_t)a.orig[slot] : slot;
  const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
  const int64_t s0 = a.indptr[row];
  const int nnz = (int)(a.indptr[row + 1] - s0);
  const int64_t e0 = a.bptr ? a.bptr[slot] : s0;
  if (nnz <= a.lds_rows)
    estep_doc<T, STATS, BOUND, true>(a, smem, slot, mem, row, s0, nnz, e0);
  else
    estep_doc<T, STATS, BOUND, false>(a, smem, slot, mem, row, s0, nnz, e0);
}

template <typename T>
void launch_estep(hipStream_t s, const EStepArgs<T>& a, bool stats, bool bound) {
  if (a.n == 0) return;
  const size_t lds = estep_lds_bytes<T>(a.kp, a.lds_rows, a.P);
  const dim3 grid((unsigned)a.n);
  if (stats) {
    static bool set = false;
    if (!set) {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_estep<T, true, false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBudget));
      set = true;
    }
    k_estep<T, true, false><<<grid, kBlock, lds, s>>>(a);
  } else if (bound) {
    static bool set = false;
    if (!set) {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_estep<T, false, true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBudget));
      set = true;
    }
    k_estep<T, false, true><<<grid, kBlock, lds, s>>>(a);
  } else {
    static bool set = false;
    if (!set) {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_estep<T, false, false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBudget));
      set = true;
    }
    k_estep<T, false, false><<<grid, kBlock, lds, s>>>(a);
  }
  KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------
// Sufficient statistics: stat[v][:] = Σ_{entries of term v} r_e · eθ'[doc(e)][:]  — a
// segmented SpMM over the batch's (term, slot) pairs radix-sorted by term.  One wave per chunk of
// kChunk sorted entries, lanes over topics; runs that cross chunk edges go to head/tail partials
// that k_fixup adds in chunk order.  Plain stores, no atomics, bitwise reproducible.
// Topics are processed in slabs of 64·Q columns (blockIdx.y, the slow grid dimension): each wave
// keeps kU·Q gathered eθ' values in flight without spilling at any k, and the waves running
// together share one slab of eθ' (≤ 100 MB at 50k docs) in the MALL.
// ---------------------------------------------------------------------------------------
template <typename T, int Q>
__global__ __launch_bounds__(256) void k_sstats(const uint32_t* __restrict__ skeys,
                                                const uint64_t* __restrict__ svals, int64_t E,
                                                const T* __restrict__ r,
                                                const T* __restrict__ eth, int kp, T* __restrict__ stat,
                                                T* __restrict__ headbuf, T* __restrict__ tailbuf,
                                                int64_t nchunks, StatMap map, int32_t* __restrict__ stamp,
                                                int32_t sid) {
  const int c0 = (int)blockIdx.y * 64 * Q;  // this slab's first topic column
  // kU entries in flight per wave: their (term, r, doc) are read out of the lanes that loaded them
  // (v_readlane: wave-uniform, so the eθ' row address is scalar) and their eθ' rows are all requested
  // before the first is accumulated — the gathers are served by L2 / MALL, and one row at a time
  // left the wave waiting a full round trip per entry.
  constexpr int kU = 8;
  const int lane = threadIdx.x & 63;
  const int64_t chunk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (chunk >= nchunks) return;
  const int64_t p0 = chunk * kChunk;
  const int64_t p1 = (p0 + kChunk < E) ? p0 + kChunk : E;
  const uint32_t first = skeys[p0], last = skeys[p1 - 1];
  const bool part = map.sub >= 0;  // a sub-chunk launch: only its terms' rows (StatMap)
  // a chunk inside one (rank, sub-chunk) term range of another launch has nothing of this one's
  if (part && stat_group(map, first) == stat_group(map, last) && stat_sub(map, first) != map.sub) return;
  const bool start_mid = p0 > 0 && skeys[p0 - 1] == first;
  const bool cont = p1 < E && skeys[p1] == last;
  T acc[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) acc[q] = T(0);
  uint32_t cur = first;
  auto flush = [&](uint32_t v) {
    T* dst;
    if (part && stat_sub(map, v) != map.sub) {  // another launch's row: drop it
#pragma unroll
      for (int q = 0; q < Q; ++q) acc[q] = T(0);
      return;
    }
    if (v == first && start_mid) {
      dst = headbuf + chunk * kp;
    } else if (v == last && cont) {
      dst = tailbuf + chunk * kp;
    } else {
      dst = stat + stat_row(map, v) * kp;
      if (stamp && blockIdx.y == 0 && lane == 0) stamp[v] = sid;  // row v holds this step's sums
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int col = c0 + lane + 64 * q;
      if (col < kp) dst[col] = acc[q];
      acc[q] = T(0);
    }
  };
  for (int64_t pb = p0; pb < p1; pb += 64) {
    const int64_t p = pb + lane;
    uint32_t kv = cur;
    T rv = T(0);
    int32_t dv = 0;
    if (p < p1) kv = skeys[p];
    // this launch's entries (a sub-chunk launch gathers nothing for the other terms)
    const bool mine = p < p1 && (!part || stat_sub(map, kv) == map.sub);
    const uint64_t mmask = part ? __ballot(mine) : ~0ull;
    if (mine) {  // (slot, r) travel with the sorted keys (entry_val); fp64 gathers r[e]
      const uint64_t pv = svals[p];
      dv = (int32_t)(pv >> 32);
      if constexpr (sizeof(T) == 4) rv = __builtin_bit_cast(T, (uint32_t)pv);
      else rv = r[(uint32_t)pv];
    }
    const int cnt = (int)((p1 - pb) < 64 ? (p1 - pb) : 64);
    for (int j0 = 0; j0 < cnt; j0 += kU) {
      uint32_t vk[kU];
      T rk[kU];
      T e[kU][Q];
#pragma unroll
      for (int u = 0; u < kU; ++u) {  // lanes past cnt hold (cur, 0, doc 0): harmless to add
        const int jj = j0 + u < 64 ? j0 + u : 63;
        vk[u] = (uint32_t)__builtin_amdgcn_readlane((int)kv, jj);
        rk[u] = readlane_t(rv, jj);
        const T* er = eth + (int64_t)__builtin_amdgcn_readlane(dv, jj) * kp;
        const bool mu = (mmask >> jj) & 1;  // wave-uniform
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int col = c0 + lane + 64 * q;
          e[u][q] = col < kp && mu ? er[col] : T(0);
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (j0 + u < cnt) {
          if (vk[u] != cur) {
            flush(cur);
            cur = vk[u];
          }
#pragma unroll
          for (int q = 0; q < Q; ++q) acc[q] += rk[u] * e[u][q];
        }
      }
    }
  }
  flush(cur);
}

// Full tiles: kTile consecutive chunks all inside one run (the entries just before and just after the
// tile carry the same term, so — the keys being sorted — every entry of the tile does).  Each such tile's
// head partials are summed here, in chunk order, one wave per tile, into the tail row of its first chunk
// (an interior chunk's tail row is otherwise unused: k_sstats writes its whole sum to the head row).
// k_fixup's owner then steps over a full tile with one add, so the run of a frequent term (thousands
// of chunks at the headline corpus) costs its owner tens of dependent round trips, not hundreds.
constexpr int kTile = 32;
template <typename T, int Q>
__global__ __launch_bounds__(256) void k_fixup_tiles(const uint32_t* __restrict__ skeys, int64_t E, int kp,
                                                     const T* __restrict__ headbuf, T* __restrict__ tailbuf,
                                                     int64_t nchunks, StatMap map) {
  constexpr int kG = 32 / Q;
  const int c0 = (int)blockIdx.y * 64 * Q;
  const int lane = threadIdx.x & 63;
  const int64_t cb = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kTile;
  if (cb == 0 || cb + kTile >= nchunks) return;  // an entry before the tile and one after it
  const uint32_t key = skeys[cb * kChunk - 1];
  if (skeys[(cb + kTile) * kChunk] != key) return;
  if (map.sub >= 0 && stat_sub(map, key) != map.sub) return;  // another sub-chunk launch's row
  T acc[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) acc[q] = T(0);
  for (int g0 = 0; g0 < kTile; g0 += kG) {
    T h[kG][Q];
#pragma unroll
    for (int g = 0; g < kG; ++g)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int col = c0 + lane + 64 * q;
        h[g][q] = col < kp ? headbuf[(cb + g0 + g) * kp + col] : T(0);
      }
#pragma unroll
    for (int g = 0; g < kG; ++g)
#pragma unroll
      for (int q = 0; q < Q; ++q) acc[q] += h[g][q];
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int col = c0 + lane + 64 * q;
    if (col < kp) tailbuf[cb * kp + col] = acc[q];
  }
}

template <typename T, int Q>
__global__ __launch_bounds__(256) void k_fixup(const uint32_t* __restrict__ skeys, int64_t E,
                                               int kp, T* __restrict__ stat,
                                               const T* __restrict__ headbuf,
                                               const T* __restrict__ tailbuf, int64_t nchunks,
                                               StatMap map, int32_t* __restrict__ stamp, int32_t sid) {
  // the run's owner (the chunk where it starts) adds the partials of the chunks the run covers, in
  // chunk order: chunk by chunk up to a kTile boundary, then whole full tiles (k_fixup_tiles' sums),
  // then chunk by chunk to the run's end.  kG chunks / tiles are fetched at a time (keys and partials).
  constexpr int kG = 32 / Q;
  const int c0 = (int)blockIdx.y * 64 * Q;  // this slab's first topic column
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  const int64_t p0 = c * kChunk;
  const int64_t p1 = (p0 + kChunk < E) ? p0 + kChunk : E;
  const uint32_t first = skeys[p0], last = skeys[p1 - 1];
  const bool start_mid = p0 > 0 && skeys[p0 - 1] == first;
  const bool cont = p1 < E && skeys[p1] == last;
  if (!cont || (first == last && start_mid)) return;  // owner = chunk where the run starts
  if (map.sub >= 0 && stat_sub(map, last) != map.sub) return;  // another sub-chunk launch's row
  T acc[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int col = c0 + lane + 64 * q;
    acc[q] = col < kp ? tailbuf[c * kp + col] : T(0);
  }
  bool more = true;
  int64_t cb = c + 1;
  // chunk by chunk over [cb, stop) while the run goes on.  The run's extent within a batch of kG chunks
  // comes from their end keys first (chunk cb is in the run; cb + g is when cb + g − 1 went on past its
  // end), and only those chunks' partials are read — most runs end in the chunk after their owner, and
  // reading kG partials for each of them was ≈ 0.4 GB per launch at the headline
  auto chunks = [&](int64_t stop) {
    while (more && cb < stop) {
      const int m = stop - cb < kG ? (int)(stop - cb) : kG;
      bool go[kG];
      T h[kG][Q];
#pragma unroll
      for (int g = 0; g < kG; ++g) {  // chunk cb+g (all `last` when in the run) goes on past its end?
        const int64_t c2 = cb + g < nchunks ? cb + g : nchunks - 1;
        const int64_t q1 = (c2 * kChunk + kChunk < E) ? c2 * kChunk + kChunk : E;
        go[g] = q1 < E && skeys[q1] == last;
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {  // chunk cb's partial, with the keys
        const int col = c0 + lane + 64 * q;
        h[0][q] = col < kp ? headbuf[cb * kp + col] : T(0);
      }
      int n_in = 1;       // chunks of this batch in the run
      bool gl = go[0];    // the last of them goes on past its end
#pragma unroll
      for (int g = 1; g < kG; ++g)
        if (n_in == g && g < m && go[g - 1]) {
          n_in = g + 1;
          gl = go[g];
        }
#pragma unroll
      for (int g = 1; g < kG; ++g)
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int col = c0 + lane + 64 * q;
          h[g][q] = g < n_in && col < kp ? headbuf[(cb + g) * kp + col] : T(0);
        }
#pragma unroll
      for (int g = 0; g < kG; ++g)
        if (g < n_in)
#pragma unroll
          for (int q = 0; q < Q; ++q) acc[q] += h[g][q];
      more = gl;
      cb += n_in;
    }
  };
  chunks((c + kTile) / kTile * kTile < nchunks ? (c + kTile) / kTile * kTile : nchunks);
  // whole tiles: cb is a tile boundary and the run reached it (the entry before cb is `last`), so the
  // tile is full — k_fixup_tiles summed it — exactly when the entry after it is `last` too
  while (more && cb + kTile < nchunks) {
    bool full[kG];
    T h[kG][Q];
#pragma unroll
    for (int g = 0; g < kG; ++g) {
      const int64_t t = cb + (int64_t)g * kTile;
      const int64_t tc = t < nchunks ? t : nchunks - 1;
      full[g] = t + kTile < nchunks && skeys[(t + kTile) * kChunk] == last;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int col = c0 + lane + 64 * q;
        h[g][q] = col < kp ? tailbuf[tc * kp + col] : T(0);
      }
    }
    bool tiles = true;
#pragma unroll
    for (int g = 0; g < kG; ++g) {
      if (tiles && full[g]) {
#pragma unroll
        for (int q = 0; q < Q; ++q) acc[q] += h[g][q];
        cb += kTile;
      } else {
        tiles = false;
      }
    }
    if (!tiles) break;
  }
  chunks(nchunks);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int col = c0 + lane + 64 * q;
    if (col < kp) stat[stat_row(map, last) * kp + col] = acc[q];
  }
  if (stamp && blockIdx.y == 0 && lane == 0) stamp[last] = sid;
}

template <typename T, int Q>
static void sstats_q(hipStream_t s, const uint32_t* skeys, const uint64_t* svals, int64_t E,
                     const T* r, const T* eth, int kp, T* stat, T* headbuf, T* tailbuf, const StatMap& map,
                     int32_t* stamp, int32_t sid) {
  const int64_t nchunks = ceil_div(E, kChunk);
  const dim3 grid((unsigned)ceil_div(nchunks, 4), (unsigned)ceil_div(kp, 64 * Q));
  k_sstats<T, Q><<<grid, 256, 0, s>>>(skeys, svals, E, r, eth, kp, stat, headbuf, tailbuf, nchunks, map, stamp,
                                      sid);
  KERNEL_CHECK();
  const int64_t ntiles = ceil_div(nchunks, (int64_t)kTile);
  if (ntiles > 1) {
    k_fixup_tiles<T, Q><<<dim3((unsigned)ceil_div(ntiles, 4), grid.y), 256, 0, s>>>(skeys, E, kp, headbuf, tailbuf,
                                                                                   nchunks, map);
    KERNEL_CHECK();
  }
  k_fixup<T, Q><<<grid, 256, 0, s>>>(skeys, E, kp, stat, headbuf, tailbuf, nchunks, map, stamp, sid);
  KERNEL_CHECK();
}

template <typename T>
void launch_sstats(hipStream_t s, const uint32_t* skeys, const uint64_t* svals, int64_t E,
                   const T* r, const T* eth, int kp, T* stat, T* headbuf, T* tailbuf, const StatMap& map,
                   int32_t* stamp, int32_t sid) {
  if (E == 0) return;
  if (stamp && map.sub >= 0) throw Error(STC_ERR_INVALID_ARG, "sstats: row stamps with a sub-chunk map");
  if (kp > 4096) throw Error(STC_ERR_INVALID_ARG, "k > 4096 topics is not supported");
  if (map.sub >= 0 && (map.vs == 0 || map.vsj == 0 || map.nsub < 1 || map.sub >= map.nsub ||
                       (uint64_t)(map.nsub - 1) * map.vsj >= map.vs))
    throw Error(STC_ERR_INVALID_ARG, "sstats: bad sub-chunk map");
  // slab width: ≤ 4 (fp64) / 8 (fp32) columns per lane — the whole row when it is that narrow
  const int q = (kp + 63) / 64;
  constexpr int QMAX = sizeof(T) == 8 ? 4 : 8;
  if (q <= 1) sstats_q<T, 1>(s, skeys, svals, E, r, eth, kp, stat, headbuf, tailbuf, map, stamp, sid);
  else if (q <= 2) sstats_q<T, 2>(s, skeys, svals, E, r, eth, kp, stat, headbuf, tailbuf, map, stamp, sid);
  else if (q <= 4 || QMAX == 4) sstats_q<T, 4>(s, skeys, svals, E, r, eth, kp, stat, headbuf, tailbuf, map, stamp, sid);
  else sstats_q<T, QMAX>(s, skeys, svals, E, r, eth, kp, stat, headbuf, tailbuf, map, stamp, sid);
}

// ---------------------------------------------------------------------------------------
// M-step.  λ is fp64 V×k (term-major, Spark's topicsMatrix orientation); rows of RB terms per
// workgroup, lanes over topics, fixed-order per-topic partial sums (deterministic colsum).
// ---------------------------------------------------------------------------------------

// expElogβ'[v][t] = exp(ψ(λ_vt) − m_v), m_v ≈ max_t ψ(λ_vt): the ROW-scaled part of Spark's
// exp(dirichletExpectation(λ)) — the per-topic factor exp(−ψ(Σ_v λ_vt)) is applied to eθ by the
// E-step (EStepArgs::psic), so a row needs only its own λ and the pass fuses with the λ update.
// m_v only has to be common to the row and to logscale, not the exact maximum: the fp32 build takes
// it from an fp32 DPP max and evaluates the exponential as 2^n · 2^f with the integer/fraction split
// done in fp64, so the fp32 argument never loses the bits of a large |ψ(λ)|.  The fp64 build takes
// m_v = ψ(max_t λ_vt) (ψ is increasing: one ψ per row instead of one per element) and evaluates
// exp(ψ(λ) − m_v) as exp_digamma_minus_d, without a logarithm per element (round 6: config 5's
// M-step was fp64-VALU-bound, 2,934 → 2,337 instructions per row at k = 2000).
__device__ __forceinline__ float exp_scaled(double x, float) {
  const double y = x * 1.4426950408889634;  // log2 e
  const double n = floor(y);
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f((float)(y - n)), (int)n);
}
__device__ __forceinline__ double exp_scaled(double x, double) { return exp(x); }
__device__ __forceinline__ double row_max(double m, float) {
  return (double)wave_max_dpp((float)m);
}
__device__ __forceinline__ double row_max(double m, double) { return wave_max(m); }

// The M-step in ONE pass over the vocabulary rows ([U] submitMiniBatch `statsSum ⊙ expElogβᵀ` +
// updateLambda, then the next minibatch's expElogβ): per row v
//   λ_v ← (1−ρ)λ_v + ρ(stat_v ⊙ Bp_v·D/|B| + η)     (UPDATE; stat ⊙ Bp = Spark's batchResult, §4)
//   Bp_v ← exp(ψ(λ_v) − m_v), logscale_v = m_v      (the next E-step's rows)
// and per block of kRowsPerBlock rows the per-topic partials of Σ_v λ_vt (colpart), reduced by
// k_colsum_reduce in block order.  One wave per row (lane = topic mod 64, Q topics per lane), the
// four waves of a block take rows w, w+4, …; the block's partials are added in wave order, so colsum
// is identical for any vocabulary slicing that keeps the blocks (§6).  UPDATE = false: colsum
// partials and Bp of the current λ (set_topics / init_random).
// five workgroups per CU (≤ 102 VGPRs, no spills; the default budget took 106 and four): the pass is
// latency-bound, one row in flight per wave — M-step 0.361 → 0.330 ms at the headline (6: 48 B of scratch
// per lane, 0.41 ms; the next row's loads issued before this row's ψ / exp, measured slower)
template <typename T, int Q, bool UPDATE>
__global__ __launch_bounds__(256, 5) void k_lambda_eeb(double* __restrict__ lam, const T* __restrict__ stat,
                                                    T* __restrict__ Bp, double* __restrict__ logscale,
                                                    int64_t V, int k, int kp, double rho, double scale,
                                                    double eta, const double* __restrict__ gate,
                                                    double* __restrict__ colpart, double* __restrict__ Bp64,
                                                    const int32_t* __restrict__ stamp, int32_t sid) {
  if (gate && !(gate[0] > 0.0)) return;  // Spark: no non-empty docs ⇒ no update
  __shared__ double s_acc[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t v0 = (int64_t)blockIdx.x * kRowsPerBlock;
  constexpr int QC = Q < 4 ? Q : 4;  // topics per lane whose loads are issued together
  double acc[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) acc[q] = 0.0;
  for (int i = w; i < kRowsPerBlock; i += 4) {
    const int64_t v = v0 + i;
    if (v >= V) break;
    double e[Q];
    double m = -INFINITY;
    // a row no sstats launch of this step wrote (stamp ≠ sid) holds stale sums: read as 0, as the cleared
    // stat row was (0·Bp·scale + η = η bit for bit), and its stat / Bp bytes are not fetched
    const bool live = !UPDATE || !stamp || stamp[v] == sid;
#pragma unroll
    for (int q0 = 0; q0 < Q; q0 += QC) {
      double lv[QC], sv[QC], bv[QC];
#pragma unroll
      for (int j = 0; j < QC; ++j) {
        const int t = lane + 64 * (q0 + j);
        lv[j] = t < k ? lam[v * k + t] : 1.0;
        if (UPDATE) {
          sv[j] = live && t < k ? (double)stat[v * kp + t] : 0.0;
          bv[j] = live && t < k ? (double)Bp[v * kp + t] : 0.0;
        }
      }
#pragma unroll
      for (int j = 0; j < QC; ++j) {
        const int q = q0 + j, t = lane + 64 * q;
        double nl = lv[j];
        if (UPDATE) nl = (1.0 - rho) * nl + rho * (sv[j] * bv[j] * scale + eta);
        if (t < k) {
          if (UPDATE) lam[v * k + t] = nl;
          acc[q] += nl;
        }
        if constexpr (sizeof(T) == 8) {  // ψ is increasing: max_t ψ(λ_vt) = ψ(max_t λ_vt)
          e[q] = nl;
          if (t < k) m = fmax(m, nl);
        } else {
          e[q] = t < k ? digamma_fast_d(nl) : -INFINITY;
          m = fmax(m, e[q]);
        }
      }
    }
    m = row_max(m, T());
    T* br = Bp + v * kp;
    if constexpr (sizeof(T) == 8) {  // one ψ per row, and exp(ψ(λ) − m_v) without a logarithm per element
      m = digamma_fast_d(m);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int t = lane + 64 * q;
        if (t < kp) br[t] = t < k ? exp_digamma_minus_d(e[q], m) : 0.0;
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int t = lane + 64 * q;
        if (t < kp) br[t] = t < k ? exp_scaled(e[q] - m, T()) : T(0);
      }
    }
    if constexpr (sizeof(T) == 4) {  // STC_MIXED: the fp64 rows of the re-solve, at the same m_v
      if (Bp64) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int t = lane + 64 * q;
          if (t < kp) Bp64[v * kp + t] = t < k ? exp(e[q] - m) : 0.0;
        }
      }
    }
    if (lane == 0) logscale[v] = m;
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    s_acc[w][lane] = acc[q];
    __syncthreads();
    const int t = lane + 64 * q;
    if (w == 0 && t < k)
      colpart[(int64_t)blockIdx.x * k + t] = ((s_acc[0][lane] + s_acc[1][lane]) + s_acc[2][lane]) + s_acc[3][lane];
    __syncthreads();
  }
}

// The same pass for many topics (kp > 256): a row per WORKGROUP — thread i owns topics i + 256·j — so
// the loads of a row are spread over 256 lanes instead of one wave's Q·3 registers, and the next row's
// loads are issued before this row's ψ/exp work (software pipelined).  The row max crosses the four
// waves through LDS (double-buffered by row parity: one barrier per row).  Each topic's colsum partial
// is one thread's running sum over the block's rows in row order.
template <typename T, int Q, bool UPDATE>
__global__ __launch_bounds__(256, Q <= 8 ? 3 : 1) void k_lambda_eeb_wide(double* __restrict__ lam, const T* __restrict__ stat,
                                                         T* __restrict__ Bp, double* __restrict__ logscale,
                                                         int64_t V, int k, int kp, double rho, double scale,
                                                         double eta, const double* __restrict__ gate,
                                                         double* __restrict__ colpart, double* __restrict__ Bp64,
                                                         const int32_t* __restrict__ stamp, int32_t sid) {
  if (gate && !(gate[0] > 0.0)) return;
  __shared__ double s_max[2][4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t v0 = (int64_t)blockIdx.x * kRowsPerBlock;
  const int nrow = (int)((V - v0) < kRowsPerBlock ? (V - v0 > 0 ? V - v0 : 0) : kRowsPerBlock);
  double acc[Q], lv[Q], sv[Q], bv[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) acc[q] = 0.0;
  auto load = [&](int64_t v) {
    const bool live = !UPDATE || !stamp || stamp[v] == sid;  // (as k_lambda_eeb)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = tid + 256 * q;
      lv[q] = t < k ? lam[v * k + t] : 1.0;
      if (UPDATE) {
        sv[q] = live && t < k ? (double)stat[v * kp + t] : 0.0;
        bv[q] = live && t < k ? (double)Bp[v * kp + t] : 0.0;
      }
    }
  };
  if (nrow > 0) load(v0);
  for (int i = 0; i < nrow; ++i) {
    const int64_t v = v0 + i;
    double e[Q];
    double m = -INFINITY;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = tid + 256 * q;
      double nl = lv[q];
      if (UPDATE) nl = (1.0 - rho) * nl + rho * (sv[q] * bv[q] * scale + eta);
      if (t < k) {
        if (UPDATE) lam[v * k + t] = nl;
        acc[q] += nl;
      }
      e[q] = nl;
    }
    if (i + 1 < nrow) load(v + 1);  // the next row's loads fly during this row's ψ / exp
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = tid + 256 * q;
      if constexpr (sizeof(T) == 8) {  // (as k_lambda_eeb) the row max of λ, one ψ per row
        if (t < k) m = fmax(m, e[q]);
      } else {
        e[q] = t < k ? digamma_fast_d(e[q]) : -INFINITY;
        m = fmax(m, e[q]);
      }
    }
    m = row_max(m, T());
    if (lane == 0) s_max[i & 1][w] = m;
    __syncthreads();
    m = fmax(fmax(s_max[i & 1][0], s_max[i & 1][1]), fmax(s_max[i & 1][2], s_max[i & 1][3]));
    T* br = Bp + v * kp;
    if constexpr (sizeof(T) == 8) {
      m = digamma_fast_d(m);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int t = tid + 256 * q;
        if (t < kp) br[t] = t < k ? exp_digamma_minus_d(e[q], m) : 0.0;
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int t = tid + 256 * q;
        if (t < kp) br[t] = t < k ? exp_scaled(e[q] - m, T()) : T(0);
      }
    }
    if constexpr (sizeof(T) == 4) {  // STC_MIXED: the fp64 rows of the re-solve, at the same m_v
      if (Bp64) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int t = tid + 256 * q;
          if (t < kp) Bp64[v * kp + t] = t < k ? exp(e[q] - m) : 0.0;
        }
      }
    }
    if (tid == 0) logscale[v] = m;
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int t = tid + 256 * q;
    if (t < k) colpart[(int64_t)blockIdx.x * k + t] = acc[q];
  }
}

template <typename T>
void launch_lambda_eeb(hipStream_t s, bool update, double* lam, const T* stat, T* Bp, double* logscale,
                       int64_t V, int k, int kp, double rho, double scale, double eta, const double* gate,
                       double* colpart, int64_t nblocks, double* Bp64, const int32_t* stamp, int32_t sid) {
  if (nblocks <= 0) return;
  if (kp > 256) {  // a row per workgroup
    const int qw = (kp + 255) / 256;
#define STC_LEEBW(QQ)                                                                                    \
  do {                                                                                                   \
    if (update)                                                                                          \
      k_lambda_eeb_wide<T, QQ, true><<<(unsigned)nblocks, 256, 0, s>>>(lam, stat, Bp, logscale, V, k, kp, \
                                                                        rho, scale, eta, gate, colpart,   \
                                                                        Bp64, stamp, sid);               \
    else                                                                                                 \
      k_lambda_eeb_wide<T, QQ, false><<<(unsigned)nblocks, 256, 0, s>>>(lam, stat, Bp, logscale, V, k,    \
                                                                         kp, rho, scale, eta, gate, colpart, \
                                                                         Bp64, stamp, sid);              \
  } while (0)
    if (qw <= 2) STC_LEEBW(2);
    else if (qw <= 4) STC_LEEBW(4);
    else if (qw <= 8) STC_LEEBW(8);
    else if (qw <= 16) STC_LEEBW(16);
    else throw Error(STC_ERR_INVALID_ARG, "k > 4096 topics is not supported");
#undef STC_LEEBW
    KERNEL_CHECK();
    return;
  }
  const int q = (kp + 63) / 64;
#define STC_LEEB(QQ)                                                                                    \
  do {                                                                                                  \
    if (update)                                                                                         \
      k_lambda_eeb<T, QQ, true><<<(unsigned)nblocks, 256, 0, s>>>(lam, stat, Bp, logscale, V, k, kp,   \
                                                                   rho, scale, eta, gate, colpart, Bp64, stamp, sid); \
    else                                                                                                \
      k_lambda_eeb<T, QQ, false><<<(unsigned)nblocks, 256, 0, s>>>(lam, stat, Bp, logscale, V, k, kp,  \
                                                                    rho, scale, eta, gate, colpart, Bp64, stamp, sid); \
  } while (0)
  if (q <= 1) STC_LEEB(1);
  else if (q <= 2) STC_LEEB(2);
  else STC_LEEB(4);
#undef STC_LEEB
  KERNEL_CHECK();
}

// colsum_t = Σ_b colpart[b][t] in block order, psic_t = ψ(colsum_t) (the E-step's per-topic factor of
// expElogβ) and psic_{k+t} = exp(−ψ(colsum_t))
__global__ __launch_bounds__(256) void k_colsum_reduce(const double* __restrict__ colpart,
                                                       int64_t nblocks, int k,
                                                       const double* __restrict__ gate,
                                                       double* __restrict__ colsum, double* __restrict__ psic) {
  if (gate && !(gate[0] > 0.0)) return;
  __shared__ double s[256];
  const int t = blockIdx.x;
  double acc = 0.0;
  for (int64_t b = threadIdx.x; b < nblocks; b += 256) acc += colpart[b * k + t];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    colsum[t] = s[0];
    const double pc = digamma_fast_d(s[0]);
    psic[t] = pc;
    psic[k + t] = exp(-pc);  // the fp32 kernels' multiplier (an fp32 exponent argument would lose its low bits)
  }
}

void launch_colsum_reduce(hipStream_t s, const double* colpart, int64_t nblocks, int k,
                          const double* gate, double* colsum, double* psic) {
  k_colsum_reduce<<<k, 256, 0, s>>>(colpart, nblocks, k, gate, colsum, psic);
  KERNEL_CHECK();
}

// logphat = Σ_docs E[log θ_d] (fixed order) ; small[k] = #non-empty docs.  Two passes: kLogphatBlocks
// blocks each sum a contiguous range of docs with lanes along the (coalesced) topic rows, then one
// block adds the block partials in block order — the same tree every run.
template <typename T>
__global__ __launch_bounds__(256) void k_logphat_part(const T* __restrict__ elogth,
                                                      const int32_t* __restrict__ nonempty, int64_t n,
                                                      int k, double* __restrict__ part) {
  // block b sums docs [b·per, (b+1)·per) for column t = threadIdx.x (+256·c): four independent loads
  // in flight per thread, the rows of a step contiguous across the block's threads
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * per, i1 = i0 + per < n ? i0 + per : n;
  for (int t = threadIdx.x; t <= k; t += 256) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t i = i0; i < i1; i += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t iu = i + u;
        if (iu < i1) acc[u] += t < k ? (double)elogth[iu * k + t] : (double)nonempty[iu];
      }
    }
    part[(int64_t)blockIdx.x * (k + 1) + t] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
}
// column t's kLogphatBlocks partials: 256 threads × (kLogphatBlocks / 256) loads, then a fixed tree
__global__ __launch_bounds__(256) void k_logphat_final(const double* __restrict__ part, int nb, int k,
                                                       double* __restrict__ small) {
  __shared__ double s[256];
  const int t = blockIdx.x;
  double acc = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) acc += part[(int64_t)b * (k + 1) + t];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) small[t] = s[0];
}

template <typename T>
void launch_logphat(hipStream_t s, const T* elogth, const int32_t* nonempty, int64_t n, int k,
                    double* small, double* part) {
  k_logphat_part<T><<<kLogphatBlocks, 256, 0, s>>>(elogth, nonempty, n, k, part);
  KERNEL_CHECK();
  k_logphat_final<<<k + 1, 256, 0, s>>>(part, kLogphatBlocks, k, small);
  KERNEL_CHECK();
}

// updateAlpha: one Newton step; applied only when every α_t + ρ·dα_t > 0
__global__ __launch_bounds__(256) void k_update_alpha(double* __restrict__ alpha,
                                                      const double* __restrict__ small, int k,
                                                      double rho) {
  extern __shared__ double s_g[];  // gradf[k], q[k]
  __shared__ double s_r[4 * 4];
  const double N = small[k];
  if (!(N > 0.0)) return;
  double* s_q = s_g + k;
  double asum = 0.0, z = 0.0, dz = -INFINITY;
  for (int t = threadIdx.x; t < k; t += 256) asum += alpha[t];
  block_reduce3(asum, z, dz, s_r);
  const double psis = digamma_t<double>(asum);
  double a1 = 0.0, a2 = 0.0;
  for (int t = threadIdx.x; t < k; t += 256) {
    const double al = alpha[t];
    const double g = N * (-(digamma_t<double>(al) - psis) + small[t] / N);
    const double q = -N * trigamma_d(al);
    s_g[t] = g;
    s_q[t] = q;
    a1 += g / q;
    a2 += 1.0 / q;
  }
  double dz2 = -INFINITY;
  block_reduce3(a1, a2, dz2, s_r);
  const double c = N * trigamma_d(asum);
  const double b = a1 / (1.0 / c + a2);
  double bad = 0.0, z2 = 0.0, dz3 = -INFINITY;
  for (int t = threadIdx.x; t < k; t += 256) {
    const double da = -(s_g[t] - b) / s_q[t];
    s_g[t] = da;
    if (!(rho * da + alpha[t] > 0.0)) bad += 1.0;
  }
  block_reduce3(bad, z2, dz3, s_r);
  if (bad == 0.0)
    for (int t = threadIdx.x; t < k; t += 256) alpha[t] += rho * s_g[t];
}

void launch_update_alpha(hipStream_t s, double* alpha, const double* small, int k, double rho) {
  k_update_alpha<<<1, 256, 2 * sizeof(double) * k, s>>>(alpha, small, k, rho);
  KERNEL_CHECK();
}

// λ₀ ~ Gamma(shape, 1/shape) i.i.d., keyed by the k×V element index (identical on every rank)
__global__ __launch_bounds__(256) void k_init_lambda(double* __restrict__ lam, int64_t V, int k,
                                                     uint64_t seed, double shape) {
  const int64_t total = V * k;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t v = e / k;
    const int t = (int)(e - v * k);
    lam[e] = gamma_sample(doc_stream(seed, (uint64_t)t * (uint64_t)V + (uint64_t)v), 0, shape);
  }
}

void launch_init_lambda(hipStream_t s, double* lam, int64_t V, int k, uint64_t seed, double shape) {
  k_init_lambda<<<2048, 256, 0, s>>>(lam, V, k, seed, shape);
  KERNEL_CHECK();
}

// topicsPart of logLikelihoodBound: Σ(η−λ)·Elogβ + Σ(lgamma λ − lgamma η) over the V×k elements; the
// per-topic Σ_k (lgamma(ηV) − lgamma Σ_v λ_vk) term is added on the host (api.hip topics_part)
template <typename T>
__global__ __launch_bounds__(256) void k_topics_bound(const double* __restrict__ lam,
                                                      const double* __restrict__ colsum, int64_t V,
                                                      int k, double eta, double* __restrict__ partials) {
  extern __shared__ double s_psic[];
  __shared__ double s_r[16];
  for (int t = threadIdx.x; t < k; t += 256) s_psic[t] = digamma_t<double>(colsum[t]);
  __syncthreads();
  const int64_t total = V * k;
  const double lge = lgamma(eta);
  double acc = 0.0, z = 0.0, dz = -INFINITY;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e % k);
    const double l = lam[e];
    const double eb = digamma_t<double>(l) - s_psic[t];
    acc += (eta - l) * eb + (lgamma(l) - lge);
  }
  block_reduce3(acc, z, dz, s_r);
  if (threadIdx.x == 0) partials[blockIdx.x] = acc;
}

template <typename T>
void launch_topics_bound(hipStream_t s, const double* lam, const double* colsum, int64_t V, int k,
                         double eta, double* partials, int64_t nblocks) {
  k_topics_bound<T><<<(unsigned)nblocks, 256, sizeof(double) * k, s>>>(lam, colsum, V, k, eta, partials);
  KERNEL_CHECK();
}

template <typename X>
__global__ __launch_bounds__(256) void k_sum(const X* __restrict__ x, int64_t n, double* __restrict__ out) {
  __shared__ double s[256];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) acc += (double)x[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = s[0];
}

void launch_sum_f64(hipStream_t s, const double* x, int64_t n, double* out) {
  k_sum<double><<<1, 256, 0, s>>>(x, n, out);
  KERNEL_CHECK();
}
template <typename T>
void launch_sum_vals(hipStream_t s, const T* x, int64_t n, double* out) {
  k_sum<T><<<1, 256, 0, s>>>(x, n, out);
  KERNEL_CHECK();
}

__global__ void k_last3(const int32_t* a, const int64_t* b, const int32_t* c, int64_t* out) {
  if (threadIdx.x == 0) {
    out[0] = *a;
    out[1] = *b;
    out[2] = *c;
  }
}
void launch_last3(hipStream_t s, const int32_t* a, const int64_t* b, const int32_t* c, int64_t* out) {
  k_last3<<<1, 64, 0, s>>>(a, b, c, out);
  KERNEL_CHECK();
}

__global__ __launch_bounds__(1024) void k_iter_stats(const int32_t* __restrict__ iters,
                                                     const int32_t* __restrict__ nonempty, int64_t n,
                                                     int max_iter, int64_t* __restrict__ out4,
                                                     int64_t* __restrict__ cum2) {
  // one block (the cumulative counters need no atomics); 1024 threads with 16 loads each in flight
  __shared__ int64_t s[4][16];
  int64_t sum = 0, cap = 0, ne = 0;
  int mx = 0;
  for (int64_t b = 0; b < n; b += 16 * 1024) {
    int it[16], nz[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int64_t i = b + u * 1024 + threadIdx.x;
      it[u] = i < n ? iters[i] : 0;
      nz[u] = i < n ? nonempty[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      sum += it[u];
      mx = it[u] > mx ? it[u] : mx;
      cap += (it[u] >= max_iter) ? 1 : 0;
      ne += nz[u];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sum += __shfl_xor(sum, o, 64);
    cap += __shfl_xor(cap, o, 64);
    ne += __shfl_xor(ne, o, 64);
    const int m2 = __shfl_xor(mx, o, 64);
    mx = m2 > mx ? m2 : mx;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s[0][w] = sum;
    s[1][w] = mx;
    s[2][w] = cap;
    s[3][w] = ne;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t r[4] = {0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) {
      r[0] += s[0][j];
      r[1] = s[1][j] > r[1] ? s[1][j] : r[1];
      r[2] += s[2][j];
      r[3] += s[3][j];
    }
    for (int j = 0; j < 4; ++j) out4[j] = r[j];
    if (cum2) {  // cumulative Σ iterations, cap hits
      cum2[0] += r[0];
      cum2[1] += r[2];
    }
  }
}

void launch_iter_stats(hipStream_t s, const int32_t* iters, const int32_t* nonempty, int64_t n,
                       int max_iter, int64_t* out4, int64_t* cum2) {
  k_iter_stats<<<1, 1024, 0, s>>>(iters, nonempty, n, max_iter, out4, cum2);
  KERNEL_CHECK();
}

__global__ __launch_bounds__(256) void k_batch_nnz(const int64_t* __restrict__ indptr,
                                                   const int32_t* __restrict__ batch, int64_t n,
                                                   int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = batch[i];
    out[i] = indptr[r + 1] - indptr[r];
  }
}

void launch_batch_nnz(hipStream_t s, const int64_t* indptr, const int32_t* batch, int64_t n,
                      int64_t* nnz_out) {
  if (n == 0) return;
  int64_t g = ceil_div(n, 256);
  k_batch_nnz<<<(unsigned)(g > 4096 ? 4096 : g), 256, 0, s>>>(indptr, batch, n, nnz_out);
  KERNEL_CHECK();
}

// RDD.sample(withReplacement, fraction): Poisson(f) (with) or Bernoulli(f) (without) per doc
__global__ __launch_bounds__(256) void k_sample(const int64_t* __restrict__ indptr, int64_t D,
                                                double f, int with_repl, uint64_t seed,
                                                int64_t iteration, int rank, int64_t cap,
                                                int32_t* __restrict__ counts,
                                                int64_t* __restrict__ weights,
                                                int32_t* __restrict__ short_counts) {
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < D; d += (int64_t)gridDim.x * 256) {
    const uint64_t st = doc_stream(seed ^ 0x5DEECE66Dull, train_doc_key(iteration, rank, d));
    const double u = rng_uniform(st, 0);
    int c = 0;
    if (with_repl) {
      double p = exp(-f), F = p;
      while (u > F && c < 64) {
        ++c;
        p *= f / c;
        F += p;
      }
    } else {
      c = u < f ? 1 : 0;
    }
    const int64_t nnz = indptr[d + 1] - indptr[d];
    counts[d] = c;
    weights[d] = (int64_t)c * nnz;
    short_counts[d] = nnz <= cap ? c : 0;
  }
}

void launch_sample(hipStream_t s, const int64_t* indptr, int64_t D, double fraction, int with_repl,
                   uint64_t seed, int64_t iteration, int rank, int64_t cap, int32_t* counts,
                   int64_t* weights, int32_t* short_counts) {
  int64_t g = ceil_div(D, 256);
  k_sample<<<(unsigned)(g > 8192 ? 8192 : g), 256, 0, s>>>(indptr, D, fraction, with_repl, seed,
                                                           iteration, rank, cap, counts, weights,
                                                           short_counts);
  KERNEL_CHECK();
}

// Members in doc order (raw position = count_incl[d] − c + j), written to partitioned slots:
// short docs (nnz <= cap) first, long docs after n_short.  All INCLUSIVE scans.
__global__ __launch_bounds__(256) void k_fill_batch(const int64_t* __restrict__ indptr, int64_t D,
                                                    int64_t cap, const int32_t* __restrict__ counts,
                                                    const int32_t* __restrict__ count_incl,
                                                    const int32_t* __restrict__ short_incl,
                                                    int64_t n_short, int32_t* __restrict__ batch_p,
                                                    int32_t* __restrict__ orig_p,
                                                    int64_t* __restrict__ nnz_p) {
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < D; d += (int64_t)gridDim.x * 256) {
    const int c = counts[d];
    if (c == 0) continue;
    const int64_t nnz = indptr[d + 1] - indptr[d];
    const int64_t raw0 = (int64_t)count_incl[d] - c;
    const int64_t sh_before = (int64_t)short_incl[d] - (nnz <= cap ? c : 0);
    const int64_t slot0 = nnz <= cap ? sh_before : n_short + (raw0 - sh_before);
    for (int j = 0; j < c; ++j) {
      batch_p[slot0 + j] = (int32_t)d;
      orig_p[slot0 + j] = (int32_t)(raw0 + j);
      nnz_p[slot0 + j] = nnz;
    }
  }
}

void launch_fill_batch(hipStream_t s, const int64_t* indptr, int64_t D, int64_t cap,
                       const int32_t* counts, const int32_t* count_incl,
                       const int32_t* short_incl, int64_t n_short, int32_t* batch_p,
                       int32_t* orig_p, int64_t* nnz_p) {
  int64_t g = ceil_div(D, 256);
  k_fill_batch<<<(unsigned)(g > 8192 ? 8192 : g), 256, 0, s>>>(indptr, D, cap, counts, count_incl,
                                                               short_incl, n_short, batch_p, orig_p,
                                                               nnz_p);
  KERNEL_CHECK();
}

// slots [0, n) reordered by idx: out[i] = in[idx[i]] for the slot arrays
__global__ __launch_bounds__(256) void k_permute_slots(const int32_t* __restrict__ idx, int64_t n,
                                                       const int32_t* __restrict__ batch, const int32_t* __restrict__ orig,
                                                       const int64_t* __restrict__ nnz, int32_t* __restrict__ batch2,
                                                       int32_t* __restrict__ orig2, int64_t* __restrict__ nnz2) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int32_t j = idx[i];
    batch2[i] = batch[j];
    orig2[i] = orig[j];
    nnz2[i] = nnz[j];
  }
}
__global__ __launch_bounds__(256) void k_iota(int32_t* __restrict__ x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] = (int32_t)i;
}
void launch_permute_slots(hipStream_t s, const int32_t* idx, int64_t n, const int32_t* batch, const int32_t* orig,
                          const int64_t* nnz, int32_t* batch2, int32_t* orig2, int64_t* nnz2) {
  if (n == 0) return;
  const int64_t g = ceil_div(n, 256);
  k_permute_slots<<<(unsigned)(g > 4096 ? 4096 : g), 256, 0, s>>>(idx, n, batch, orig, nnz, batch2, orig2, nnz2);
  KERNEL_CHECK();
}
// The sstats pairs of an fp64 launch built from the batch alone (api.hip presort): entry e = bptr[slot] + n
// of slot `slot` is the slot's n-th CSR entry, with key its term and value entry_val(slot, e) — exactly what
// the rows E-step kernels write in their close phase (fp64 carries the entry index, not r), so the radix sort
// can run beside the E-step instead of after it.  One wave per slot.
__global__ __launch_bounds__(256) void k_entry_pairs(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
                                                     const int32_t* __restrict__ batch, const int64_t* __restrict__ bptr,
                                                     int64_t n, uint32_t* __restrict__ keys, uint64_t* __restrict__ vals) {
  const int lane = threadIdx.x & 63;
  for (int64_t slot = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6; slot < n; slot += ((int64_t)gridDim.x * 256) >> 6) {
    const int64_t row = batch[slot], s0 = indptr[row], nnz = indptr[row + 1] - s0, e0 = bptr[slot];
    for (int64_t j = lane; j < nnz; j += 64) {
      keys[e0 + j] = (uint32_t)indices[s0 + j];
      vals[e0 + j] = entry_val<double>(slot, e0 + j, 0.0);
    }
  }
}
void launch_entry_pairs(hipStream_t s, const int64_t* indptr, const int32_t* indices, const int32_t* batch,
                        const int64_t* bptr, int64_t n, uint32_t* keys, uint64_t* vals) {
  if (n == 0) return;
  const int64_t g = ceil_div(n, 4);
  k_entry_pairs<<<(unsigned)(g > 8192 ? 8192 : g), 256, 0, s>>>(indptr, indices, batch, bptr, n, keys, vals);
  KERNEL_CHECK();
}
void launch_iota(hipStream_t s, int32_t* x, int64_t n) {
  if (n == 0) return;
  const int64_t g = ceil_div(n, 256);
  k_iota<<<(unsigned)(g > 4096 ? 4096 : g), 256, 0, s>>>(x, n);
  KERNEL_CHECK();
}

// host-injected membership: flags + stable partition into [short | long] slots
__global__ __launch_bounds__(256) void k_part_flags(const int64_t* __restrict__ indptr,
                                                    const int32_t* __restrict__ batch, int64_t n,
                                                    int64_t cap, int64_t* __restrict__ nnz_out,
                                                    int32_t* __restrict__ short_flag) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = batch ? (int64_t)batch[i] : i;  // nullptr: identity rows
    const int64_t nnz = indptr[r + 1] - indptr[r];
    nnz_out[i] = nnz;
    short_flag[i] = nnz <= cap ? 1 : 0;
  }
}

void launch_part_flags(hipStream_t s, const int64_t* indptr, const int32_t* batch, int64_t n,
                       int64_t cap, int64_t* nnz_out, int32_t* short_flag) {
  if (n == 0) return;
  int64_t g = ceil_div(n, 256);
  k_part_flags<<<(unsigned)(g > 4096 ? 4096 : g), 256, 0, s>>>(indptr, batch, n, cap, nnz_out, short_flag);
  KERNEL_CHECK();
}

__global__ __launch_bounds__(256) void k_part_scatter(const int32_t* __restrict__ batch,
                                                      const int64_t* __restrict__ nnz, int64_t n,
                                                      const int32_t* __restrict__ short_flag,
                                                      const int32_t* __restrict__ short_incl,
                                                      int32_t* __restrict__ batch_p,
                                                      int32_t* __restrict__ orig_p,
                                                      int64_t* __restrict__ nnz_p) {
  const int64_t n_short = n > 0 ? short_incl[n - 1] : 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t sh = short_incl[i];
    const int64_t slot = short_flag[i] ? sh - 1 : n_short + (i - sh);
    batch_p[slot] = batch ? batch[i] : (int32_t)i;
    orig_p[slot] = (int32_t)i;
    nnz_p[slot] = nnz[i];
  }
}

void launch_part_scatter(hipStream_t s, const int32_t* batch, const int64_t* nnz, int64_t n,
                         const int32_t* short_flag, const int32_t* short_incl, int32_t* batch_p,
                         int32_t* orig_p, int64_t* nnz_p) {
  if (n == 0) return;
  int64_t g = ceil_div(n, 256);
  k_part_scatter<<<(unsigned)(g > 4096 ? 4096 : g), 256, 0, s>>>(batch, nnz, n, short_flag, short_incl,
                                                                 batch_p, orig_p, nnz_p);
  KERNEL_CHECK();
}

__global__ __launch_bounds__(256) void k_transpose_kv(const double* __restrict__ lam, int64_t V, int k,
                                                      double* __restrict__ out, int32_t* __restrict__ idx) {
  const int64_t total = V * k;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e / V);
    const int64_t v = e - (int64_t)t * V;
    out[e] = lam[v * k + t];
    idx[e] = (int32_t)v;
  }
}

void launch_transpose_kv(hipStream_t s, const double* lam, int64_t V, int k, double* out_kv,
                         int32_t* idx_kv) {
  k_transpose_kv<<<4096, 256, 0, s>>>(lam, V, k, out_kv, idx_kv);
  KERNEL_CHECK();
}

// Spark's sstats from the scaled stat: stat'_vt = stat_vt · e^{m_v} · e^{−ψc_t} (r carries e^{m_v},
// eθ the per-topic e^{−ψ(colsum_t)}), so stat_vt = stat'_vt · exp(ψc_t − m_v)
template <typename T>
__global__ __launch_bounds__(256) void k_unscale_stat(const T* __restrict__ stat,
                                                      const double* __restrict__ logscale,
                                                      const double* __restrict__ psic, int64_t V,
                                                      int k, int kp, double* __restrict__ out) {
  const int64_t total = V * k;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t v = e / k;
    const int t = (int)(e - v * k);
    out[e] = (double)stat[v * kp + t] * exp(psic[t] - logscale[v]);
  }
}

template <typename T>
void launch_unscale_stat(hipStream_t s, const T* stat, const double* logscale, const double* psic, int64_t V,
                         int k, int kp, double* out_vk) {
  k_unscale_stat<T><<<4096, 256, 0, s>>>(stat, logscale, psic, V, k, kp, out_vk);
  KERNEL_CHECK();
}

// γ₀ of a launch's members ahead of the E-step: one thread per (slot, topic), the counter RNG each
// E-step kernel would otherwise run in its prologue (the same gamma_sample, key and stream), written
// member-major for EStepArgs::gamma0.  The E-step prologues are latency-bound per document and the team
// kernels drew every topic of the document in every member; here the draws fill the chip.
template <typename T>
__global__ __launch_bounds__(256) void k_gamma0(const int32_t* __restrict__ batch, const int32_t* __restrict__ orig,
                                                int64_t n, int k, uint64_t seed, int64_t iteration, int rank,
                                                int key_mode, int64_t doc_id_base, double shape, T* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * k) return;
  const int64_t slot = i / k;
  const int t = (int)(i - slot * k);
  const int64_t mem = orig ? (int64_t)orig[slot] : slot;
  const int64_t row = batch ? (int64_t)batch[slot] : slot;
  const uint64_t key = key_mode == 0 ? train_doc_key(iteration, rank, mem) : (uint64_t)(doc_id_base + row);
  out[mem * k + t] = (T)gamma_sample(doc_stream(seed, key), t, shape);
}

template <typename T>
void launch_gamma0(hipStream_t s, const int32_t* batch, const int32_t* orig, int64_t n, int k, uint64_t seed,
                   int64_t iteration, int rank, int key_mode, int64_t doc_id_base, double shape, T* out) {
  if (n <= 0) return;
  k_gamma0<T><<<(unsigned)ceil_div(n * k, (int64_t)256), 256, 0, s>>>(batch, orig, n, k, seed, iteration, rank,
                                                                      key_mode, doc_id_base, shape, out);
  KERNEL_CHECK();
}

// ---- STC_MIXED: the fp64 re-solve of the fp32 E-step's slowly converging documents -------------------
// slots whose member is non-empty and took more than `thr` fp32 iterations: those with nnz ≤ cap64 (the fp64
// fast kernels' row capacity) from position 0 up (count cnt[0]), the others from position n − 1 down
// (count cnt[1]); each position holds the slot's row, member, entry offset and the slot itself.  The order
// within a list is the atomics' (every document's outputs are its own, so results do not depend on it).
__global__ void k_mixed_list(const int64_t* __restrict__ indptr, const int32_t* __restrict__ batch,
                             const int32_t* __restrict__ orig, const int64_t* __restrict__ bptr,
                             const int32_t* __restrict__ iters, const int32_t* __restrict__ nonempty, int64_t n,
                             int thr, int64_t cap64, int32_t* __restrict__ lbatch, int32_t* __restrict__ lorig,
                             int64_t* __restrict__ lbptr, int32_t* __restrict__ lslot, int32_t* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t mem = orig ? orig[i] : (int32_t)i;
  if (!nonempty[mem] || iters[mem] <= thr) return;
  const int64_t row = batch ? batch[i] : i;
  const int64_t nnz = indptr[row + 1] - indptr[row];
  const int64_t j = nnz <= cap64 ? (int64_t)atomicAdd(&cnt[0], 1) : n - 1 - (int64_t)atomicAdd(&cnt[1], 1);
  lbatch[j] = (int32_t)row;
  lorig[j] = mem;
  lbptr[j] = bptr ? bptr[i] : indptr[row];
  lslot[j] = (int32_t)i;
}
void launch_mixed_list(hipStream_t s, const int64_t* indptr, const int32_t* batch, const int32_t* orig,
                       const int64_t* bptr, const int32_t* iters, const int32_t* nonempty, int64_t n, int thr,
                       int64_t cap64, int32_t* lbatch, int32_t* lorig, int64_t* lbptr, int32_t* lslot, int32_t* cnt) {
  HIP_CHECK(hipMemsetAsync(cnt, 0, 2 * sizeof(int32_t), s));
  if (n <= 0) return;
  k_mixed_list<<<(unsigned)ceil_div(n, (int64_t)256), 256, 0, s>>>(indptr, batch, orig, bptr, iters, nonempty, n, thr,
                                                                  cap64, lbatch, lorig, lbptr, lslot, cnt);
  KERNEL_CHECK();
}
// the re-solved documents' fp64 outputs into the fp32 step buffers: eθ' and E[log θ] per slot, r and the
// sstats sort value (slot, fp32 r) per entry, γ per member (when given); one workgroup per listed document
// (list positions [0, ms) and [n − ml, n))
__global__ __launch_bounds__(256) void k_mixed_fixup(const int64_t* __restrict__ indptr, const int32_t* __restrict__ lbatch,
                                                     const int32_t* __restrict__ lorig, const int64_t* __restrict__ lbptr,
                                                     const int32_t* __restrict__ lslot, int64_t n, int ms, int ml, int k,
                                                     int kp, const double* __restrict__ eth64,
                                                     const double* __restrict__ elogth64, const double* __restrict__ r64,
                                                     const double* __restrict__ gamma64, float* __restrict__ eth,
                                                     float* __restrict__ elogth, float* __restrict__ r,
                                                     uint64_t* __restrict__ vals, float* __restrict__ gamma) {
  const int jj = blockIdx.x;
  const int64_t j = jj < ms ? jj : n - ml + (jj - ms);
  const int64_t slot = lslot[j], mem = lorig[j], row = lbatch[j], e0 = lbptr[j];
  const int64_t nnz = indptr[row + 1] - indptr[row];
  for (int t = threadIdx.x; t < kp; t += blockDim.x) {
    eth[slot * kp + t] = (float)eth64[j * kp + t];
    if (t < k) {
      elogth[slot * k + t] = (float)elogth64[j * k + t];
      if (gamma) gamma[mem * k + t] = (float)gamma64[mem * k + t];
    }
  }
  for (int64_t e = threadIdx.x; e < nnz; e += blockDim.x) {
    const float rv = (float)r64[e0 + e];
    r[e0 + e] = rv;
    if (vals) vals[e0 + e] = entry_val<float>(slot, e0 + e, rv);
  }
}
void launch_mixed_fixup(hipStream_t s, const int64_t* indptr, const int32_t* lbatch, const int32_t* lorig,
                        const int64_t* lbptr, const int32_t* lslot, int64_t n, int ms, int ml, int k, int kp,
                        const double* eth64, const double* elogth64, const double* r64, const double* gamma64,
                        float* eth, float* elogth, float* r, uint64_t* vals, float* gamma) {
  if (ms + ml <= 0) return;
  k_mixed_fixup<<<(unsigned)(ms + ml), 256, 0, s>>>(indptr, lbatch, lorig, lbptr, lslot, n, ms, ml, k, kp, eth64,
                                                    elogth64, r64, gamma64, eth, elogth, r, vals, gamma);
  KERNEL_CHECK();
}
__global__ void k_to_f32(const double* __restrict__ in, float* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}
void launch_to_f32(hipStream_t s, const double* in, float* out, int64_t n) {
  if (n <= 0) return;
  k_to_f32<<<(unsigned)std::min<int64_t>(ceil_div(n, (int64_t)256), 65536), 256, 0, s>>>(in, out, n);
  KERNEL_CHECK();
}

#define STC_INSTANTIATE(T)                                                                        \
  template void launch_gamma0<T>(hipStream_t, const int32_t*, const int32_t*, int64_t, int, uint64_t, int64_t, \
                                 int, int, int64_t, double, T*);                                  \
  template size_t estep_lds_bytes<T>(int, int, int);                                              \
  template int estep_lds_rows<T>(int, int, int);                                                  \
  template void launch_estep<T>(hipStream_t, const EStepArgs<T>&, bool, bool);                    \
  template void launch_sstats<T>(hipStream_t, const uint32_t*, const uint64_t*, int64_t, const T*, \
                                 const T*, int, T*, T*, T*, const StatMap&, int32_t*, int32_t);   \
  template void launch_lambda_eeb<T>(hipStream_t, bool, double*, const T*, T*, double*, int64_t, int, \
                                     int, double, double, double, const double*, double*, int64_t, double*, \
                                     const int32_t*, int32_t);                                    \
  template void launch_logphat<T>(hipStream_t, const T*, const int32_t*, int64_t, int, double*, double*);  \
  template void launch_topics_bound<T>(hipStream_t, const double*, const double*, int64_t, int,   \
                                       double, double*, int64_t);                                 \
  template void launch_sum_vals<T>(hipStream_t, const T*, int64_t, double*);                      \
  template void launch_unscale_stat<T>(hipStream_t, const T*, const double*, const double*, int64_t, int, \
                                       int, double*);

STC_INSTANTIATE(float)
STC_INSTANTIATE(double)

}  // namespace lda
}  // namespace stc
