// lda_wide.hip — K6 for many topics (k > 128 fp32, k > 104 fp64; BASELINE configs 4 and 5): one
// document per 512-thread workgroup, topics across the lanes, the document's rows along each lane.
//
// Same fixed point as k_estep / [U] OnlineLDAOptimizer.variationalTopicInference (lda.hip has the
// row-scaled numerics).  Lane l owns the Q adjacent topics [Q·l, Q·l + Q) (k ≤ 512·Q) and holds, for
// every row n of the document, its Q entries of B = expElogβ'[ids, :]:
//   rows n <  NR          in VGPRs (B[n][q], NR·Q values per lane),
//   rows n <  NR + NL     in LDS (NL set per launch from the LDS left over),
//   rows n >= NR + NL     re-read from the row-scaled expElogβ' in global memory (L2 / MALL) every pass
// — config 5 (k = 2000, nnz ≤ 50) is fully resident; config 4 (k = 500, nnz ≈ 372, a 744 KB fp32 block
// against a 512 KB register file) streams its tail.
//   φ_n = B_n·eθ : Q lane-local FMAs per row; 16-row chunks are reduce-scattered over the wave (swap32,
//     swap16, row_half_mirror, quad_perm, then row_ror:8 / quad_perm all-reduce), each wave's row sums
//     meet in LDS, and lane n sums the eight in a fixed order ⇒ r_n = cts_n/φ_n (broadcast via LDS).
//   s = Bᵀr : lane-local (every lane holds all rows of its topics) — no reduction at all.
//   γ, ψ(γ), exp on the lane's own topics.  ψ(Σγ') from Σγ' = Σα + Σ_n r_n·(φ_n − ε'_n) (exact in
//     real arithmetic), summed by the r lanes next to r — two barriers per iteration.
#include "estep_common.h"

namespace stc {
namespace lda {

namespace {

constexpr int kWThreads = 512;          // threads per document
constexpr int kWWaves = kWThreads / 64;
constexpr int kWRows = 512;             // max nnz of a document this kernel takes (LDS arrays)
constexpr int kWChunk = 16;             // rows per Phase A reduce-scatter
constexpr size_t kWLds = 160 * 1024;    // one workgroup per CU: all of the CU's LDS

template <typename T>
struct WTr;
template <>
struct WTr<float> {
  static __device__ __forceinline__ float wsum(float v) { return wave_sum_dpp(v); }
  static __device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
  static __device__ __forceinline__ float eth(float g, float cs) { return __expf(digamma_fast(g) - cs); }
  static __device__ __forceinline__ float psi(float x) { return digamma_fast(x); }
  static __device__ __forceinline__ float eps_floor() { return kTiny; }
  static __device__ __forceinline__ float eps_cap() { return 3.0e38f; }
  // 16 values → this lane's row of the chunk, summed over the wave (see the header)
  static __device__ __forceinline__ float rs16(const float* x, int lane) {
    float a[8], b[4], c[2];
    swap_add_n<true, 8>(x, x + 8, a);   // bit 5
    swap_add_n<false, 4>(a, a + 4, b);  // bit 4
    c[0] = rs_dpp<DPP_ROW_HALF_MIRROR>(b[0], b[2], lane & 4);
    c[1] = rs_dpp<DPP_ROW_HALF_MIRROR>(b[1], b[3], lane & 4);
    float d = rs_dpp<DPP_QP_3210>(c[0], c[1], lane & 2);
    d += dpp_f<DPP_ROW_ROR8>(d);        // bit 3 (all-reduce: both lanes hold the sum)
    d += dpp_f<DPP_QP_1032>(d);         // bit 0
    return d;
  }
  // 8 values → this lane's row (bits 5, 4, 2 reduce-scatter; bits 3, 1, 0 all-reduce)
  static __device__ __forceinline__ float rs8(const float* x, int lane) {
    float a[4], b[2];
    swap_add_n<true, 4>(x, x + 4, a);
    swap_add_n<false, 2>(a, a + 2, b);
    float d = rs_dpp<DPP_ROW_HALF_MIRROR>(b[0], b[1], lane & 4);
    d += dpp_f<DPP_ROW_ROR8>(d);
    d += dpp_f<DPP_QP_1032>(d);
    d += dpp_f<DPP_QP_2301>(d);
    return d;
  }
};
template <>
struct WTr<double> {
  static __device__ __forceinline__ double wsum(double v) { return wave_sum_d(v); }
  static __device__ __forceinline__ double rcp(double x) { return rcp_nr(x); }
  static __device__ __forceinline__ double eth(double g, double cs) { return exp_digamma_minus_d(g, cs); }
  static __device__ __forceinline__ double psi(double x) { return digamma_fast_d(x); }
  static __device__ __forceinline__ double eps_floor() { return 0.0; }
  static __device__ __forceinline__ double eps_cap() { return 1e300; }
  static __device__ __forceinline__ double rs16(const double* x, int lane) {
    double a[8], b[4], c[2];
    swap_add_nd<true, 8>(x, x + 8, a);
    swap_add_nd<false, 4>(a, a + 4, b);
    c[0] = rs_dpp_d<DPP_ROW_HALF_MIRROR>(b[0], b[2], lane & 4);
    c[1] = rs_dpp_d<DPP_ROW_HALF_MIRROR>(b[1], b[3], lane & 4);
    double d = rs_dpp_d<DPP_QP_3210>(c[0], c[1], lane & 2);
    d += dpp_d<DPP_ROW_ROR8>(d);
    d += dpp_d<DPP_QP_1032>(d);
    return d;
  }
  static __device__ __forceinline__ double rs8(const double* x, int lane) {
    double a[4], b[2];
    swap_add_nd<true, 4>(x, x + 4, a);
    swap_add_nd<false, 2>(a, a + 2, b);
    double d = rs_dpp_d<DPP_ROW_HALF_MIRROR>(b[0], b[1], lane & 4);
    d += dpp_d<DPP_ROW_ROR8>(d);
    d += dpp_d<DPP_QP_1032>(d);
    d += dpp_d<DPP_QP_2301>(d);
    return d;
  }
};
// the chunk row a lane holds after rs16 (levels bit 5, 4, 2, 1 halve the set; bits 3 and 0 all-reduce)
__device__ __forceinline__ int rs16_row(int lane) {
  return 8 * ((lane >> 5) & 1) + 4 * ((lane >> 4) & 1) + 2 * ((lane >> 2) & 1) + ((lane >> 1) & 1);
}
// CH-row chunks (16, or 8 where the register budget is tight): the reduction, the row a lane ends
// with, and the lanes that publish it (one per row)
template <typename T, int CH>
__device__ __forceinline__ T rs_chunk(const T* x, int lane) {
  if constexpr (CH == 16) return WTr<T>::rs16(x, lane);
  else return WTr<T>::rs8(x, lane);
}
template <int CH>
__device__ __forceinline__ int rs_row(int lane) {
  if constexpr (CH == 16) return rs16_row(lane);
  else return 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 2) & 1);
}
template <int CH>
__device__ __forceinline__ bool rs_pub(int lane) { return (lane & (CH == 16 ? 9 : 11)) == 0; }
// rows per Phase A chunk: 8 for fp64 with ≥ 2 topics per lane (room for more register rows)
template <typename T, int Q>
constexpr int wide_chunk() { return sizeof(T) == 8 && Q >= 2 ? 8 : kWChunk; }

// Q adjacent topics [t0, t0 + Q) of row `row` (pitch kp), zero past kp
template <typename T, int Q>
__device__ __forceinline__ void load_q(const T* __restrict__ Bp, int64_t row, int kp, int t0, T* out) {
  const T* p = Bp + row * kp + t0;
  if (t0 + Q <= kp) {
    if constexpr (sizeof(T) * Q % 16 == 0) {
#pragma unroll
      for (int i = 0; i < (int)(sizeof(T) * Q / 16); ++i) {
        const float4 v = reinterpret_cast<const float4*>(p)[i];
        __builtin_memcpy(out + i * (16 / sizeof(T)), &v, 16);
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) out[q] = p[q];
    }
  } else {
#pragma unroll
    for (int q = 0; q < Q; ++q) out[q] = (t0 + q < kp) ? p[q] : T(0);
  }
}

// the lane's Q entries of rows n0 .. n0+15 past the register rows: from LDS (n < nres), streamed from
// global memory (n < nnz; every load issued before any is used), zero past nnz
template <typename T, int Q, int LB>
__device__ __forceinline__ void rows_q(const T* __restrict__ Bp, const int* ids, const T* sB, int kp, int t0, int nr,
                                       int nres, int nnz, int n0, T (*y)[Q]) {
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int n = n0 + i;
    if (n < nres && n < nnz) {
      const T* p = sB + (int64_t)(n - nr) * (kWThreads * Q) + t0;
#pragma unroll
      for (int q = 0; q < Q; ++q) y[i][q] = p[q];
    } else if (n < nnz) {
      load_q<T, Q>(Bp, (int64_t)ids[n], kp, t0, y[i]);
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) y[i][q] = T(0);
    }
  }
}

template <typename T>
struct WLds {
  T xs[kWWaves][kWRows];  // per-wave row sums of φ (Phase A)
  T rr[kWRows];           // r_n = cts_n / φ_n, broadcast to every lane (Phase B)
  T red[2][kWWaves];      // [0]: Σ|Δγ| of the last update, [1]: Σ_n r_n·dot_n (ψ(Σγ') identity)
  int ids[kWRows];        // term ids (the streamed rows' addresses without a dependent index load)
  double bd[kWWaves][4];  // bound partials
};

template <typename T>
__host__ __device__ constexpr size_t wide_lds_fixed() {
  return (sizeof(WLds<T>) + 255) / 256 * 256;
}

#ifndef WIDE_LB_BYTES
#define WIDE_LB_BYTES 64  // streamed-row loads in flight per lane (bytes)
#endif
#ifndef WIDE_NR64_Q1
#define WIDE_NR64_Q1 64
#endif
#ifndef WIDE_NR64_Q2
#define WIDE_NR64_Q2 24
#endif
#ifndef WIDE_NR64_Q4
#define WIDE_NR64_Q4 8
#endif
template <typename T, int Q, int NR, bool STATS, bool BOUND>
__global__ __launch_bounds__(kWThreads) void k_estep_wide(EStepArgs<T> a, int nl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  WLds<T>& sm = *reinterpret_cast<WLds<T>*>(smem);
  T* const sB = reinterpret_cast<T*>(smem + wide_lds_fixed<T>());  // [nl][512·Q]
  using Tr = WTr<T>;
  constexpr int CH = wide_chunk<T, Q>();
  constexpr int LB = (int)(WIDE_LB_BYTES / (sizeof(T) * Q)) < CH ? (int)(WIDE_LB_BYTES / (sizeof(T) * Q)) : CH;
  if ((int64_t)blockIdx.x >= a.n) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t slot = a.slot0 + blockIdx.x;
  const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
  const int64_t mem = a.orig ? (int64_t)a.orig[slot] : slot;
  const int64_t s0 = a.indptr[row];
  const int nnz = (int)(a.indptr[row + 1] - s0);
  const int64_t e0 = a.bptr ? a.bptr[slot] : s0;
  const int k = a.k, kp = a.kp, t0 = Q * tid;
  const int nres = NR + nl;  // rows resident in VGPRs + LDS

  // ---- per-row scalars of the rows this thread owns as an "r lane": n = tid, tid + 512 (< kWRows)
  constexpr int RL = kWRows / kWThreads;
  T cts[RL], eps[RL];
  int any = 0;
#pragma unroll
  for (int j = 0; j < RL; ++j) {
    const int n = tid + kWThreads * j;
    const bool v = n < nnz;
    const int64_t pos = s0 + (v && a.order ? a.order[s0 + n] : n);
    const int id = v ? a.indices[pos] : 0;
    cts[j] = v ? a.values[pos] : T(0);
    sm.ids[n] = id;  // published by the __syncthreads_or below
    // Spark's 1e-100 in the row-scaled space (lda.hip): ε'_n = 1e-100·e^{−m_v}, kept finite (a row whose
    // e^{−m_v} overflows has an all-zero unscaled expElogβ in Spark and contributes nothing; r ≈ 0 here)
    eps[j] = v ? fmin(fmax((T)fmin(exp(kLogEps - a.logscale[id]), 1e300), Tr::eps_floor()), Tr::eps_cap()) : T(0);
    any |= (cts[j] != T(0));
  }
  const bool nonempty = __syncthreads_or(any) != 0;

  // ---- γ₀ / α of this lane's topics
  uint64_t stream = 0;
  if (!a.gamma0) {
    const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem) : (uint64_t)(a.doc_id_base + row);
    stream = doc_stream(a.seed, key);
  }
  T gam[Q], alp[Q], eth[Q];
  T gs = T(0), as = T(0);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int t = t0 + q;
    gam[q] = t < k ? (a.gamma0 ? a.gamma0[mem * k + t] : (T)gamma_sample(stream, t, a.gamma_shape)) : T(0);
    alp[q] = t < k ? (T)a.alpha[t] : T(0);
    gs += gam[q];
    as += alp[q];
  }
  if (!nonempty) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = t0 + q;
      if (t < k) {
        if (a.gamma) a.gamma[mem * k + t] = T(0);
        if (STATS) a.elogth[slot * k + t] = T(0);
      }
      if (STATS && t < kp) a.eth[slot * kp + t] = T(0);
    }
#pragma unroll
    for (int j = 0; j < RL; ++j) {
      const int n = tid + kWThreads * j;
      if (n < nnz) {
        a.r[e0 + n] = T(0);
        if (STATS) {
          a.keys[e0 + n] = (uint32_t)sm.ids[n];
          a.vals[e0 + n] = entry_val<T>(slot, e0 + n, T(0));
        }
      }
    }
    if (tid == 0) {
      if (a.iters) a.iters[mem] = 0;
      if (a.nonempty) a.nonempty[mem] = 0;
      if (BOUND) a.bound[mem] = 0.0;
    }
    return;
  }
  // Σγ₀, Σα, Σcts over the block (one LDS round)
  {
    T ct = T(0);
#pragma unroll
    for (int j = 0; j < RL; ++j) ct += cts[j];
    gs = Tr::wsum(gs);
    as = Tr::wsum(as);
    ct = Tr::wsum(ct);
    if (lane == 0) {
      sm.xs[wave][0] = gs;
      sm.xs[wave][1] = as;
      sm.xs[wave][2] = ct;
    }
    __syncthreads();
    gs = sm.xs[0][0];
    as = sm.xs[0][1];
#pragma unroll
    for (int w = 1; w < kWWaves; ++w) {
      gs += sm.xs[w][0];
      as += sm.xs[w][1];
    }
    __syncthreads();  // xs is reused by Phase A
  }

  // ---- the document block: rows < NR in VGPRs, rows < NR + nl in LDS (coalesced Q-wide loads)
  T B[NR > 0 ? NR : 1][Q];
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    if (n < nnz) load_q<T, Q>(a.Bp, (int64_t)sm.ids[n], kp, t0, B[n]);
    else {
#pragma unroll
      for (int q = 0; q < Q; ++q) B[n][q] = T(0);
    }
  }
  for (int n = NR; n < nres && n < nnz; ++n) {
    T x[Q];
    load_q<T, Q>(a.Bp, (int64_t)sm.ids[n], kp, t0, x);
#pragma unroll
    for (int q = 0; q < Q; ++q) sB[(int64_t)(n - NR) * (kWThreads * Q) + t0 + q] = x[q];  // read back by this lane
  }

  T cs = Tr::psi(gs);  // ψ(Σγ) of the current γ
#pragma unroll
  for (int q = 0; q < Q; ++q) eth[q] = (t0 + q < k) ? Tr::eth(gam[q], cs) : T(0);
  T dg = T(0);  // Σ_q |Δγ| of this lane's topics in the last update
  int it = 0;
  double b_tok = 0.0, c_tok = 0.0;
  const T kd = (T)k;
  while (true) {
    // Phase A: per-wave row sums of B_n·eθ, 16 rows at a time — register rows (compile-time indices;
    // their zero padding past nnz gives zero sums), then the LDS / streamed rows
#pragma unroll
    for (int c = 0; c < NR / CH; ++c) {
      if (CH * c < nnz) {
        T x[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          T acc = T(0);
#pragma unroll
          for (int q = 0; q < Q; ++q) acc = fma(B[CH * c + i][q], eth[q], acc);
          x[i] = acc;
        }
        const T v = rs_chunk<T, CH>(x, lane);
        const int n = CH * c + rs_row<CH>(lane);
        if (rs_pub<CH>(lane) && n < nnz) sm.xs[wave][n] = v;
      }
    }
    for (int n0 = NR; n0 < nnz; n0 += CH) {
      T x[CH];
#pragma unroll
      for (int b = 0; b < CH; b += LB) {
        T y[LB][Q];
        rows_q<T, Q, LB>(a.Bp, sm.ids, sB, kp, t0, NR, nres, nnz, n0 + b, y);  // LB rows' loads in flight
#pragma unroll
        for (int i = 0; i < LB; ++i) {
          T acc = T(0);
#pragma unroll
          for (int q = 0; q < Q; ++q) acc = fma(y[i][q], eth[q], acc);
          x[b + i] = acc;
        }
      }
      const T v = rs_chunk<T, CH>(x, lane);
      const int n = n0 + rs_row<CH>(lane);
      if (rs_pub<CH>(lane) && n < nnz) sm.xs[wave][n] = v;
    }
    const T dsum_w = Tr::wsum(dg);
    if (lane == 0) sm.red[0][wave] = dsum_w;
    __syncthreads();  // (1) row sums and Σ|Δγ| published
    T dsum = sm.red[0][0];
#pragma unroll
    for (int w = 1; w < kWWaves; ++w) dsum += sm.red[0][w];
    // Spark: while (meanGammaChange > 1e-3); block-uniform
    const bool last = (it > 0 && dsum / kd <= T(1e-3)) || it >= a.max_iter;
    T rd = T(0);
#pragma unroll
    for (int j = 0; j < RL; ++j) {
      const int n = tid + kWThreads * j;
      if (n < nnz) {
        T dot = sm.xs[0][n];
#pragma unroll
        for (int w = 1; w < kWWaves; ++w) dot += sm.xs[w][n];
        const T r = cts[j] * Tr::rcp(dot + eps[j]);
        sm.rr[n] = r;
        rd = fma(r, dot, rd);
        if (BOUND && last && cts[j] != T(0)) {
          b_tok += (double)cts[j] * (log(fmax((double)dot, 1e-300)) + a.logscale[sm.ids[n]]);
          c_tok += (double)cts[j];
        }
      }
    }
    rd = Tr::wsum(rd);
    if (lane == 0) sm.red[1][wave] = rd;
    __syncthreads();  // (2) r and Σ r·dot published
    if (last) break;
    T sg = sm.red[1][0];
#pragma unroll
    for (int w = 1; w < kWWaves; ++w) sg += sm.red[1][w];
    cs = Tr::psi(as + sg);  // ψ(Σγ') = ψ(Σα + Σ_n r_n·dot_n)

    // Phase B: s_q = Σ_n B[n][q]·r_n, lane-local
    T s[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) s[q] = T(0);
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      if (n < nnz) {
        const T r = sm.rr[n];
#pragma unroll
        for (int q = 0; q < Q; ++q) s[q] = fma(B[n][q], r, s[q]);
      }
    }
    for (int n0 = NR; n0 < nnz; n0 += LB) {
      T y[LB][Q];
      rows_q<T, Q, LB>(a.Bp, sm.ids, sB, kp, t0, NR, nres, nnz, n0, y);
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const T r = n0 + i < nnz ? sm.rr[n0 + i] : T(0);
#pragma unroll
        for (int q = 0; q < Q; ++q) s[q] = fma(y[i][q], r, s[q]);
      }
    }
    // γ ← eθ ⊙ s + α ; eθ = exp(ψ(γ) − ψ(Σγ'))
    dg = T(0);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (t0 + q < k) {
        const T gn = fma(eth[q], s[q], alp[q]);
        dg += fabs(gn - gam[q]);
        gam[q] = gn;
        eth[q] = Tr::eth(gn, cs);
      }
    }
    ++it;
  }

  // ---- outputs
#pragma unroll
  for (int j = 0; j < RL; ++j) {
    const int n = tid + kWThreads * j;
    if (n < nnz) {
      const T r = sm.rr[n];
      a.r[e0 + n] = r;
      if (STATS) {
        a.keys[e0 + n] = (uint32_t)sm.ids[n];
        a.vals[e0 + n] = entry_val<T>(slot, e0 + n, r);
      }
    }
  }
  // exact Σγ of the final γ
  double gsd = 0.0;
#pragma unroll
  for (int q = 0; q < Q; ++q) gsd += (double)gam[q];
  gsd = wave_sum(gsd);
  if (lane == 0) sm.bd[wave][0] = gsd;
  __syncthreads();
  double gsum = 0.0;
  for (int w = 0; w < kWWaves; ++w) gsum += sm.bd[w][0];
  const double psisum = digamma_t<double>(gsum);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int t = t0 + q;
    if (t < k) {
      if (a.gamma) a.gamma[mem * k + t] = gam[q];
      if (STATS) a.elogth[slot * k + t] = (T)(digamma_t<double>((double)gam[q]) - psisum);
    }
    if (STATS && t < kp) a.eth[slot * kp + t] = t < k ? eth[q] : T(0);  // the eθ the last φ used
  }
  if (tid == 0) {
    if (a.iters) a.iters[mem] = it;
    if (a.nonempty) a.nonempty[mem] = 1;
  }
  if (BOUND) {
    double topic = 0.0, asum = 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = t0 + q;
      if (t < k) {
        const double gd = (double)gam[q], al = a.alpha[t];
        topic += (al - gd) * (digamma_t<double>(gd) - psisum) + (lgamma(gd) - lgamma(al));
        asum += al;
      }
    }
    topic = wave_sum(topic);
    asum = wave_sum(asum);
    const double tok = wave_sum(b_tok), ct = wave_sum(c_tok);
    __syncthreads();  // bd[·][0] reads above are done
    if (lane == 0) {
      sm.bd[wave][0] = topic;
      sm.bd[wave][1] = asum;
      sm.bd[wave][2] = tok;
      sm.bd[wave][3] = ct;
    }
    __syncthreads();
    if (tid == 0) {
      double tp = 0.0, aw = 0.0, tk = 0.0, cw = 0.0;
      for (int w = 0; w < kWWaves; ++w) {
        tp += sm.bd[w][0];
        aw += sm.bd[w][1];
        tk += sm.bd[w][2];
        cw += sm.bd[w][3];
      }
      // token terms used the loop's ψ(Σγ') (cs) in eθ; move them to the exact ψ(Σγ)
      a.bound[mem] = tk + cw * ((double)cs - psisum) + tp + (lgamma(aw) - lgamma(gsum));
    }
  }
}

// register rows per (T, Q): NR·Q·sizeof(T)/4 ≈ 128 VGPRs, so 512 threads keep two waves per SIMD
// (fp32 Q = 1 — config 4's k = 500 — takes 176 rows: 227 VGPRs, no spills, the most the register
// file holds at two waves per SIMD; its streamed tail is what bounds that config)
template <typename T, int Q>
constexpr int wide_nr() {
  return (sizeof(T) == 4 && Q == 1) ? 176
         : (sizeof(T) == 8 && Q == 1) ? WIDE_NR64_Q1
         : sizeof(T) == 8 && Q >= 2 ? (Q == 2 ? WIDE_NR64_Q2 : WIDE_NR64_Q4)  // fp64: 8-row chunks
                                    : (int)(128 * 4 / (sizeof(T) * Q)) / kWChunk * kWChunk;
}

template <typename T, int Q>
void launch_q(hipStream_t s, const EStepArgs<T>& a, bool stats, bool bound) {
  constexpr int NR = wide_nr<T, Q>();
  const size_t fixed = wide_lds_fixed<T>();
  const size_t row_bytes = sizeof(T) * kWThreads * Q;
  const int nl = (int)((kWLds - fixed) / row_bytes);
  const size_t lds = fixed + (size_t)nl * row_bytes;
  auto go = [&](auto kern) {
    HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    kern<<<dim3((unsigned)a.n), kWThreads, lds, s>>>(a, nl);
    KERNEL_CHECK();
  };
  if (stats) go(k_estep_wide<T, Q, NR, true, false>);
  else if (bound) go(k_estep_wide<T, Q, NR, false, true>);
  else go(k_estep_wide<T, Q, NR, false, false>);
}

}  // namespace

int wide_row_cap(int k) { return k <= kWThreads * 4 ? kWRows : 0; }

template <typename T>
void launch_estep_wide(hipStream_t s, const EStepArgs<T>& a, bool stats, bool bound) {
  if (a.n == 0) return;
  if (a.k <= kWThreads) launch_q<T, 1>(s, a, stats, bound);
  else if (a.k <= 2 * kWThreads) launch_q<T, 2>(s, a, stats, bound);
  else if (a.k <= 4 * kWThreads) launch_q<T, 4>(s, a, stats, bound);
  else throw Error(STC_ERR_INVALID_ARG, "wide E-step: k > 2048");
}

template void launch_estep_wide<float>(hipStream_t, const EStepArgs<float>&, bool, bool);
template void launch_estep_wide<double>(hipStream_t, const EStepArgs<double>&, bool, bool);

}  // namespace lda
}  // namespace stc
