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
#include "psi64.h"
#include "team_exchange.h"

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
  // eθ' = exp(ψ(g) − cs)·exp(−ψc): pc holds exp(−ψc) (an fp32 argument − ψc would lose its low bits)
  static __device__ __forceinline__ float eth(float g, float cs, float pc) { return __expf(digamma_fast(g) - cs) * pc; }
  static __device__ __forceinline__ float pcload(const double* psic, int k, int t) { return (float)psic[k + t]; }
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
  // eθ' = exp(ψ(g) − cs − ψc): pc holds ψc
  static __device__ __forceinline__ double eth(double g, double cs, double pc) {
#if WIDE_PSI_V2
    return exp_digamma_minus_v2<2>(g, cs + pc);  // psi64.h: branch-free, constants as SGPR operands
#else
    return exp_digamma_minus_d(g, cs + pc);
#endif
  }
  static __device__ __forceinline__ double pcload(const double* psic, int k, int t) { (void)k; return psic[t]; }
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
// global memory (n < nnz; every load issued before any is used), zero past nnz.  t0: the lane's first
// topic (global column); its LDS column is Q·lane-in-block (the topic-split team's t0 is offset)
template <typename T, int Q, int LB>
__device__ __forceinline__ void rows_q(const T* __restrict__ Bp, const int* ids, const T* sB, int kp, int t0, int nr,
                                       int nres, int nnz, int n0, T (*y)[Q]) {
  const int lc = Q * (int)threadIdx.x;
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int n = n0 + i;
    if (n < nres && n < nnz) {
      const T* p = sB + (int64_t)(n - nr) * (kWThreads * Q) + lc;
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

// the document block's resident rows: rows < NR into registers, rows < nres into LDS (sB), every
// row of a batch loaded before any is stored (rows past `nrows` read term 0 and are zeroed), so the
// loads of a batch are in flight together rather than one memory round trip per row
template <typename T, int Q, int NR>
__device__ __forceinline__ void load_block(const T* __restrict__ Bp, const int* ids, int nrows, int nres, T* sB,
                                           int kp, int t0, T (*B)[Q]) {
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    T x[Q];
    load_q<T, Q>(Bp, n < nrows ? (int64_t)ids[n] : 0, kp, t0, x);
#pragma unroll
    for (int q = 0; q < Q; ++q) B[n][q] = n < nrows ? x[q] : T(0);
  }
  const int lend = nres < nrows ? nres : nrows;
  const int lc = Q * (int)threadIdx.x;  // LDS column (t0 is the global one)
  for (int n0 = NR; n0 < lend; n0 += 8) {
    T x[8][Q];
#pragma unroll
    for (int i = 0; i < 8; ++i) load_q<T, Q>(Bp, n0 + i < lend ? (int64_t)ids[n0 + i] : 0, kp, t0, x[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (n0 + i < lend) {
#pragma unroll
        for (int q = 0; q < Q; ++q) sB[(int64_t)(n0 + i - NR) * (kWThreads * Q) + lc + q] = x[i][q];  // read back by this lane
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

#ifndef WIDE_PSI_V2
// fp64 γ update through psi64.h's chain (as k_estep_rows64) instead of exp_digamma_minus_d + libm exp:
// one ψ/exp form across the fp64 E-step kernels; measured neutral at config 4 (277 ms either way over
// 20 steps after 10 warm-up), parity unchanged
#define WIDE_PSI_V2 1
#endif
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
  static_assert(NR % 8 == 0 && NR % CH == 0, "Phase A takes register rows CH, Phase B 8 at a time");
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
  T gam[Q], alp[Q], pc[Q], eth[Q];  // pc: expElogβ's per-topic factor (WTr::pcload)
  T gs = T(0), as = T(0);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int t = t0 + q;
    gam[q] = t < k ? (a.gamma0 ? a.gamma0[mem * k + t] : (T)gamma_sample(stream, t, a.gamma_shape)) : T(0);
    alp[q] = t < k ? (T)a.alpha[t] : T(0);
    pc[q] = t < k ? Tr::pcload(a.psic, k, t) : T(0);
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
  load_block<T, Q, NR>(a.Bp, sm.ids, nnz, nres, sB, kp, t0, B);

  for (int n = nnz + tid; n < kWRows; n += kWThreads) sm.rr[n] = T(0);  // Phase B reads rows in 8s
  T cs = Tr::psi(gs);  // ψ(Σγ) of the current γ
#pragma unroll
  for (int q = 0; q < Q; ++q) eth[q] = (t0 + q < k) ? Tr::eth(gam[q], cs, pc[q]) : T(0);
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
    // register rows without per-row branches (rows past nnz: B = 0, r = 0), so the r loads of
    // consecutive rows are in flight together instead of one LDS round trip per row
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      const T r = sm.rr[n];
#pragma unroll
      for (int q = 0; q < Q; ++q) s[q] = fma(B[n][q], r, s[q]);
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
        eth[q] = Tr::eth(gn, cs, pc[q]);
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

// ---------------------------------------------------------------------------------------------
// k_estep_wide_mc — the same fixed point with one document's ROWS split over a team of P workgroups
// (P CUs), so a block larger than one CU's registers + LDS (fp64 config 4: 371 × 500 × 8 B = 1.5 MB;
// fp64 config 5: 44 × 2000 × 8 B = 0.7 MB) stays resident instead of being re-streamed from the MALL
// twice per iteration.  Member m holds rows [m·nnz/P, (m+1)·nnz/P) for all topics:
//   φ_n, r_n  : local (a member has every topic of its rows);
//   s = Bᵀr   : a partial per member, exchanged once per iteration with Σ_n r_n·φ_n (the ψ(Σγ')
//               identity); every member sums the P partials in member order, so γ, eθ and the stop
//               rule are bit-identical in every member and the team leaves the loop together.
// Persistent: G = 8·P·⌊CUs/(8P)⌋ blocks (one per CU: the kernel takes all 160 KB of LDS), launched
// once the occupancy check says the grid is resident (launch_resident); team members share blockIdx % 8 (one XCD,
// for L2 locality, and for the plain granule stores below).  Exchange (cdna_hip_programming.md
// Guideline 16, R2: the data is the flag): every value travels in a 16-byte granule {epoch, value}
// written by ONE 16-B buffer store and read by 16-B sc1 (L1-bypassing) buffer loads (untorn on gfx950);
// each consumer wave re-reads its granules until
// every tag equals the epoch — no flag, no fence, no block barrier.  Granules double-buffered by epoch
// parity (a member can run at most one exchange ahead, so a slot never holds a newer epoch than the
// one awaited).  Every spin is bounded: on timeout the kernel sets the timeout word and every team
// leaves (the host reports it as an error).
// the exchange primitives (granules, bounded spins) live in team_exchange.h, shared with lda_team64.hip

template <typename T, int Q, int NR, bool STATS>
__global__ __launch_bounds__(kWThreads) void k_estep_wide_mc(EStepArgs<T> a, int nl, WideTeam wt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  WLds<T>& sm = *reinterpret_cast<WLds<T>*>(smem);
  T* const sB = reinterpret_cast<T*>(smem + wide_lds_fixed<T>());  // [nl][512·Q]
  __shared__ int s_abort;
  using Tr = WTr<T>;
  constexpr int CH = wide_chunk<T, Q>();
  static_assert(NR % 8 == 0 && NR % CH == 0, "Phase A takes register rows CH, Phase B 8 at a time");
  constexpr int LB = (int)(WIDE_LB_BYTES / (sizeof(T) * Q)) < CH ? (int)(WIDE_LB_BYTES / (sizeof(T) * Q)) : CH;
  const int P = wt.P;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = (int)blockIdx.x, il = b / 8;
  const int member = il % P, team = (il / P) * 8 + (b % 8), nteams = (int)gridDim.x / P;
  const bool pub = !(team == 0 && member == wt.fault_member);  // debug: a member that never publishes
  // this team's granules [parity][member][xstride], 16 B each
  const int team_granules = 2 * P * (int)wt.xstride;
  unsigned char* const xb = reinterpret_cast<unsigned char*>(wt.xbuf) + (int64_t)team * team_granules * 16;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(xb, 0, team_granules * 16, 0x00020000);
  const int k = a.k, kp = a.kp, t0 = Q * tid;
  unsigned epoch = 0;
  if (tid == 0) s_abort = 0;
  STAMP_DECL

  for (int64_t j = team; j < a.n; j += nteams) {
    const int64_t slot = a.slot0 + j;
    const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
    const int64_t mem = a.orig ? (int64_t)a.orig[slot] : slot;
    const int64_t s0 = a.indptr[row];
    const int nnz = (int)(a.indptr[row + 1] - s0);
    const int64_t e0 = a.bptr ? a.bptr[slot] : s0;
    const int lo = (int)((int64_t)member * nnz / P), hi = (int)((int64_t)(member + 1) * nnz / P);
    const int nloc = hi - lo;  // this member's rows (≤ 512 / P ... ≤ 512)
    const int nres = NR + nl;

    // ---- every row's count (the document's emptiness is a team-wide decision); this member's rows
    T cts = T(0), eps = T(0);
    int any = 0;
    if (tid < nnz) {
      const int64_t pos = s0 + (a.order ? a.order[s0 + tid] : tid);
      any = a.values[pos] != T(0);
    }
    if (tid < nloc) {
      const int n = lo + tid;
      const int64_t pos = s0 + (a.order ? a.order[s0 + n] : n);
      const int id = a.indices[pos];
      cts = a.values[pos];
      sm.ids[tid] = id;
      eps = fmin(fmax((T)fmin(exp(kLogEps - a.logscale[id]), 1e300), Tr::eps_floor()), Tr::eps_cap());
    }
    const bool nonempty = __syncthreads_or(any) != 0;

    uint64_t stream = 0;
    if (!a.gamma0) {
      const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem) : (uint64_t)(a.doc_id_base + row);
      stream = doc_stream(a.seed, key);
    }
    T gam[Q], alp[Q], pc[Q], eth[Q];  // pc: expElogβ's per-topic factor (WTr::pcload)
    T gs = T(0), as = T(0);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = t0 + q;
      gam[q] = t < k ? (a.gamma0 ? a.gamma0[mem * k + t] : (T)gamma_sample(stream, t, a.gamma_shape)) : T(0);
      alp[q] = t < k ? (T)a.alpha[t] : T(0);
      pc[q] = t < k ? Tr::pcload(a.psic, k, t) : T(0);
      gs += gam[q];
      as += alp[q];
    }
    if (!nonempty) {
      if (member == 0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int t = t0 + q;
          if (t < k) {
            if (a.gamma) a.gamma[mem * k + t] = T(0);
            if (STATS) a.elogth[slot * k + t] = T(0);
          }
          if (STATS && t < kp) a.eth[slot * kp + t] = T(0);
        }
        if (tid == 0) {
          if (a.iters) a.iters[mem] = 0;
          if (a.nonempty) a.nonempty[mem] = 0;
        }
      }
      if (tid < nloc) {
        const int n = lo + tid;
        a.r[e0 + n] = T(0);
        if (STATS) {
          a.keys[e0 + n] = (uint32_t)sm.ids[tid];
          a.vals[e0 + n] = entry_val<T>(slot, e0 + n, T(0));
        }
      }
      __syncthreads();  // sm.ids is rewritten by the next document
      continue;
    }
    // Σγ₀, Σα over the block (identical in every member)
    gs = Tr::wsum(gs);
    as = Tr::wsum(as);
    if (lane == 0) {
      sm.xs[wave][0] = gs;
      sm.xs[wave][1] = as;
    }
    __syncthreads();
    gs = sm.xs[0][0];
    as = sm.xs[0][1];
#pragma unroll
    for (int w = 1; w < kWWaves; ++w) {
      gs += sm.xs[w][0];
      as += sm.xs[w][1];
    }
    __syncthreads();

    // ---- this member's block: local rows < NR in VGPRs, < NR + nl in LDS, the rest streamed
    T B[NR > 0 ? NR : 1][Q];
    load_block<T, Q, NR>(a.Bp, sm.ids, nloc, nres, sB, kp, t0, B);

    if (tid >= nloc) sm.rr[tid] = T(0);  // Phase B reads rows in 8s (published by barrier (1))
    T cs = Tr::psi(gs);
#pragma unroll
    for (int q = 0; q < Q; ++q) eth[q] = (t0 + q < k) ? Tr::eth(gam[q], cs, pc[q]) : T(0);
    T dg = T(0);
    int it = 0;
    const T kd = (T)k;
    T rfin = T(0);
    STAMP(0);  // per-document preamble: counts, γ₀, the block's loads
    while (true) {
      // Phase A over the local rows (as k_estep_wide)
#pragma unroll
      for (int c = 0; c < NR / CH; ++c) {
        if (CH * c < nloc) {
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
          if (rs_pub<CH>(lane) && n < nloc) sm.xs[wave][n] = v;
        }
      }
      for (int n0 = NR; n0 < nloc; n0 += CH) {
        T x[CH];
#pragma unroll
        for (int bb = 0; bb < CH; bb += LB) {
          T y[LB][Q];
          rows_q<T, Q, LB>(a.Bp, sm.ids, sB, kp, t0, NR, nres, nloc, n0 + bb, y);
#pragma unroll
          for (int i = 0; i < LB; ++i) {
            T acc = T(0);
#pragma unroll
            for (int q = 0; q < Q; ++q) acc = fma(y[i][q], eth[q], acc);
            x[bb + i] = acc;
          }
        }
        const T v = rs_chunk<T, CH>(x, lane);
        const int n = n0 + rs_row<CH>(lane);
        if (rs_pub<CH>(lane) && n < nloc) sm.xs[wave][n] = v;
      }
      const T dsum_w = Tr::wsum(dg);
      if (lane == 0) sm.red[0][wave] = dsum_w;
      STAMP(1);  // Phase A
      __syncthreads();  // (1) row sums and Σ|Δγ| published (and any wave's give-up in s_abort)
      if (s_abort) break;
      T dsum = sm.red[0][0];
#pragma unroll
      for (int w = 1; w < kWWaves; ++w) dsum += sm.red[0][w];
      const bool last = (it > 0 && dsum / kd <= T(1e-3)) || it >= a.max_iter;  // team-uniform
      T rd = T(0);
      if (tid < nloc) {
        T dot = sm.xs[0][tid];
#pragma unroll
        for (int w = 1; w < kWWaves; ++w) dot += sm.xs[w][tid];
        const T r = cts * Tr::rcp(dot + eps);
        sm.rr[tid] = r;
        rfin = r;
        rd = fma(r, dot, rd);
      }
      rd = Tr::wsum(rd);
      if (lane == 0) sm.red[1][wave] = rd;
      __syncthreads();  // (2) r and Σ r·dot published
      STAMP(2);  // barriers, r, Σ r·φ
      if (last) break;
      T sgl = sm.red[1][0];
#pragma unroll
      for (int w = 1; w < kWWaves; ++w) sgl += sm.red[1][w];

      // Phase B: this member's partial s over its rows
      T s[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) s[q] = T(0);
#pragma unroll
      for (int n = 0; n < NR; ++n) {  // no per-row branches (rows past nloc: B = 0, r = 0)
        const T r = sm.rr[n];
#pragma unroll
        for (int q = 0; q < Q; ++q) s[q] = fma(B[n][q], r, s[q]);
      }
      for (int n0 = NR; n0 < nloc; n0 += LB) {
        T y[LB][Q];
        rows_q<T, Q, LB>(a.Bp, sm.ids, sB, kp, t0, NR, nres, nloc, n0, y);
#pragma unroll
        for (int i = 0; i < LB; ++i) {
          const T r = n0 + i < nloc ? sm.rr[n0 + i] : T(0);
#pragma unroll
          for (int q = 0; q < Q; ++q) s[q] = fma(y[i][q], r, s[q]);
        }
      }
      STAMP(3);  // Phase B
      // ---- exchange: publish (s partial, Σ r·dot partial) as epoch granules, then every wave
      // collects the other members' granules for its lanes' topics; sums in member order
      ++epoch;
      const int base = (int)(epoch & 1) * P * (int)wt.xstride;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (pub && t0 + q < kp) put_granule<T>(rs, base + member * (int)wt.xstride + t0 + q, epoch, s[q]);
      if (pub && tid == 0) put_granule<T>(rs, base + member * (int)wt.xstride + kp, epoch, sgl);
      T st[Q];
      T sg = T(0);
#pragma unroll
      for (int q = 0; q < Q; ++q) st[q] = T(0);
      for (int m = 0; m < P; ++m) {
        if (m == member) {
#pragma unroll
          for (int q = 0; q < Q; ++q) st[q] += s[q];
          sg += sgl;
          continue;
        }
        const int g0 = base + m * (int)wt.xstride;
        T v[Q], vs = T(0);
#ifdef STC_TEAM_NOWAIT  // timing-only diagnostic build: read whatever is there (wrong results)
        if (true) {
          get_granule<T>(rs, g0 + kp, epoch, vs);
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            v[q] = T(0);
            if (t0 + q < kp) get_granule<T>(rs, g0 + t0 + q, epoch, v[q]);
          }
          vs = T(0);
#pragma unroll
          for (int q = 0; q < Q; ++q) v[q] = T(0);
        } else
#endif
        for (unsigned spins = 0;; ++spins) {
          // the Σ r·dot granule is the same for every lane: lane 0 polls it, the wave takes it by readlane
          bool ok = lane != 0 || get_granule<T>(rs, g0 + kp, epoch, vs);
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            v[q] = T(0);
            if (t0 + q < kp) ok &= get_granule<T>(rs, g0 + t0 + q, epoch, v[q]);
          }
          if (__all(ok)) break;
          if (spin_give_up(spins, wt.tmo, wt.spin_limit)) {
            if (lane == 0) s_abort = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        vs = readlane_t(vs, 0);
#pragma unroll
        for (int q = 0; q < Q; ++q) st[q] += v[q];
        sg += vs;
      }
      STAMP(4);  // exchange (publish + wait + member-order sums)
      cs = Tr::psi(as + sg);
      dg = T(0);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (t0 + q < k) {
          const T gn = fma(eth[q], st[q], alp[q]);
          dg += fabs(gn - gam[q]);
          gam[q] = gn;
          eth[q] = Tr::eth(gn, cs, pc[q]);
        }
      }
      ++it;
      STAMP(5);  // γ, ψ/exp
    }
    if (s_abort) return;  // a team timed out: every block leaves (the host re-runs the one-CU kernel)

    // ---- outputs: this member's rows; the topic-level ones from member 0
    if (tid < nloc) {
      const int n = lo + tid;
      a.r[e0 + n] = rfin;
      if (STATS) {
        a.keys[e0 + n] = (uint32_t)sm.ids[tid];
        a.vals[e0 + n] = entry_val<T>(slot, e0 + n, rfin);
      }
    }
    if (member == 0) {
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
        if (STATS && t < kp) a.eth[slot * kp + t] = t < k ? eth[q] : T(0);
      }
      if (tid == 0) {
        if (a.iters) a.iters[mem] = it;
        if (a.nonempty) a.nonempty[mem] = 1;
      }
    }
    __syncthreads();  // LDS (ids, xs, rr, bd, sB) is rewritten by the next document
    STAMP(6);  // outputs
  }
  STAMP_FLUSH
}

// ---------------------------------------------------------------------------------------------
// k_estep_wide_tc's LDS: the per-row arrays sized by the launch's longest document (xr rows, ≥ NR so the
// register rows past nnz read r = 0) instead of WLds's 512, so the CU's LDS holds more block rows — at
// config 5 (k = 2000, ≈ 44 rows) 15 → 19 LDS rows next to the 24 register rows, and a document's rows
// are streamed from L2 in Phase A and B of every iteration only past 43 instead of 39
template <typename T>
struct TcLds {
  T red[2][kWWaves];      // [0]: Σ|Δγ| of the last update, [1]: Σ_n r_n·dot_n
  double bd[kWWaves][4];  // Σγ partials
};
template <typename T>
__host__ __device__ constexpr size_t tc_lds_head() {
  return (sizeof(TcLds<T>) + 255) / 256 * 256;
}
// xs [kWWaves][xr] T, rr [xr] T, ids [xr] int
template <typename T>
__host__ __device__ constexpr size_t tc_lds_fixed(int xr) {
  return (tc_lds_head<T>() + (size_t)xr * ((kWWaves + 1) * sizeof(T) + sizeof(int)) + 255) / 256 * 256;
}

// k_estep_wide_tc — a team of P workgroups per document with the TOPICS split (k > 512: config 5's
// k = 2000 in fp64, whose 44 × 2000 × 8 B block is 4.5× what one CU keeps resident at 4 topics per
// lane).  Member m owns topics [m·512Q, (m+1)·512Q) and every row of the document, so s = Bᵀr and the
// γ / eθ update are local and the team exchanges only each member's φ partials (nnz values) plus its
// Σ|Δγ| (the stop rule) once per iteration — 44 values at config 5 instead of the row split's 2000.
// Every member adds the P partials in member order, so φ, r, Σ r·φ and the stop rule are identical in
// every member.  ψ(Σγ₀) and Σα come from all k topics in every member (γ₀ is counter-RNG keyed); the
// final Σγ (E[log θ] for logphat) is one more exchange.  Grid, granules, bounds: as k_estep_wide_mc.
template <typename T, int Q, int NR, bool STATS>
__global__ __launch_bounds__(kWThreads) void k_estep_wide_tc(EStepArgs<T> a, int nl, WideTeam wt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  TcLds<T>& sm = *reinterpret_cast<TcLds<T>*>(smem);
  const int xr = wt.xrows;                                           // ≥ every nnz of the launch, ≥ NR
  T* const xs = reinterpret_cast<T*>(smem + tc_lds_head<T>());       // [kWWaves][xr] φ partials per wave
  T* const rr = xs + kWWaves * xr;                                   // [xr] r_n
  int* const ids = reinterpret_cast<int*>(rr + xr);                  // [xr] term ids
  T* const sB = reinterpret_cast<T*>(smem + tc_lds_fixed<T>(xr));    // [nl][512·Q]
  __shared__ int s_abort;
  using Tr = WTr<T>;
  constexpr int CH = wide_chunk<T, Q>();
  static_assert(NR % 8 == 0 && NR % CH == 0, "Phase A takes register rows CH, Phase B 8 at a time");
  constexpr int LB = (int)(WIDE_LB_BYTES / (sizeof(T) * Q)) < CH ? (int)(WIDE_LB_BYTES / (sizeof(T) * Q)) : CH;
  constexpr int GD = kWRows, GS = kWRows + 1;  // granule slots: row partials [0, nnz), Σ|Δγ|, Σγ
  const int P = wt.P;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = (int)blockIdx.x, il = b / 8;
  const int member = il % P, team = (il / P) * 8 + (b % 8), nteams = (int)gridDim.x / P;
  const bool pub_ok = !(team == 0 && member == wt.fault_member);  // debug: a member that never publishes
  const int team_granules = 2 * P * (int)wt.xstride;
  unsigned char* const xb = reinterpret_cast<unsigned char*>(wt.xbuf) + (int64_t)team * team_granules * 16;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(xb, 0, team_granules * 16, 0x00020000);
  const int k = a.k, kp = a.kp, kP = kWThreads * Q;
  const int t0 = member * kP + Q * tid;  // this lane's first topic
  unsigned epoch = 0;
  if (tid == 0) s_abort = 0;
  STAMP_DECL

  // one exchange: publish `mine` at slot `idx` (if `pub`), then the member-order sum of slot `idx`
  // over the team (every lane of a wave takes part in the poll; `need` = this lane reads the slot)
  auto exchange = [&](int idx, T mine, bool pub, bool need) -> T {
    const int base = (int)(epoch & 1) * P * (int)wt.xstride;
    if (pub && pub_ok) put_granule<T>(rs, base + member * (int)wt.xstride + idx, epoch, mine);
    T sum = T(0);
    for (int m = 0; m < P; ++m) {
      T v = T(0);
      if (m == member) {
        v = mine;
      } else {
        for (unsigned spins = 0;; ++spins) {
          const bool ok = !need || get_granule<T>(rs, base + m * (int)wt.xstride + idx, epoch, v);
          if (__all(ok)) break;
          if (spin_give_up(spins, wt.tmo, wt.spin_limit)) {
            if (lane == 0) s_abort = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      sum += v;
    }
    return sum;
  };

  for (int64_t j = team; j < a.n; j += nteams) {
    const int64_t slot = a.slot0 + j;
    const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
    const int64_t mem = a.orig ? (int64_t)a.orig[slot] : slot;
    const int64_t s0 = a.indptr[row];
    const int nnz = (int)(a.indptr[row + 1] - s0);
    const int64_t e0 = a.bptr ? a.bptr[slot] : s0;
    const int nres = NR + nl;
    if (nnz > xr) {  // longer than the launch's max_row said: the whole launch goes to the one-CU kernel
      if (tid == 0) __hip_atomic_store(wt.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }

    T cts = T(0), eps = T(0);
    int any = 0;
    if (tid < nnz) {
      const int64_t pos = s0 + (a.order ? a.order[s0 + tid] : tid);
      const int id = a.indices[pos];
      cts = a.values[pos];
      ids[tid] = id;
      eps = fmin(fmax((T)fmin(exp(kLogEps - a.logscale[id]), 1e300), Tr::eps_floor()), Tr::eps_cap());
      any = cts != T(0);
    }
    const bool nonempty = __syncthreads_or(any) != 0;

    uint64_t stream = 0;
    if (!a.gamma0) {
      const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem) : (uint64_t)(a.doc_id_base + row);
      stream = doc_stream(a.seed, key);
    }
    T gam[Q], alp[Q], pc[Q], eth[Q];  // pc: expElogβ's per-topic factor (WTr::pcload)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = t0 + q;
      gam[q] = t < k ? (a.gamma0 ? a.gamma0[mem * k + t] : (T)gamma_sample(stream, t, a.gamma_shape)) : T(0);
      alp[q] = t < k ? (T)a.alpha[t] : T(0);
      pc[q] = t < k ? Tr::pcload(a.psic, k, t) : T(0);
    }
    if (!nonempty) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int t = t0 + q;
        if (t < k) {
          if (a.gamma) a.gamma[mem * k + t] = T(0);
          if (STATS) a.elogth[slot * k + t] = T(0);
        }
        if (STATS && t < kp && q + Q * tid < kP) a.eth[slot * kp + t] = T(0);
      }
      if (member == 0) {
        if (tid < nnz) {
          a.r[e0 + tid] = T(0);
          if (STATS) {
            a.keys[e0 + tid] = (uint32_t)ids[tid];
            a.vals[e0 + tid] = entry_val<T>(slot, e0 + tid, T(0));
          }
        }
        if (tid == 0) {
          if (a.iters) a.iters[mem] = 0;
          if (a.nonempty) a.nonempty[mem] = 0;
        }
      }
      __syncthreads();
      continue;
    }
    // Σγ₀ and Σα over all k topics, in the same order in every member (lane l: topics l·Q + q of every
    // member's range)
    T gs = T(0), as = T(0);
    for (int m = 0; m < P; ++m) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int t = m * kP + Q * tid + q;
        if (t < k) {
          gs += m == member ? gam[q] : (a.gamma0 ? a.gamma0[mem * k + t] : (T)gamma_sample(stream, t, a.gamma_shape));
          as += (T)a.alpha[t];
        }
      }
    }
    gs = Tr::wsum(gs);
    as = Tr::wsum(as);
    if (lane == 0) {
      xs[wave * xr] = gs;
      xs[wave * xr + 1] = as;
    }
    __syncthreads();
    gs = xs[0];
    as = xs[1];
#pragma unroll
    for (int w = 1; w < kWWaves; ++w) {
      gs += xs[w * xr];
      as += xs[w * xr + 1];
    }
    __syncthreads();

    STAMP(0);  // per-document preamble: ids, ε', γ₀, Σγ₀ / Σα
    // the block of this member's topics: rows < NR in VGPRs, < NR + nl in LDS, the rest streamed
    T B[NR > 0 ? NR : 1][Q];
    load_block<T, Q, NR>(a.Bp, ids, nnz, nres, sB, kp, t0, B);
    if (tid >= nnz && tid < xr) rr[tid] = T(0);

    T cs = Tr::psi(gs);
#pragma unroll
    for (int q = 0; q < Q; ++q) eth[q] = (t0 + q < k) ? Tr::eth(gam[q], cs, pc[q]) : T(0);
    T dg = T(0);
    int it = 0;
    const T kd = (T)k;
    T rfin = T(0);
    STAMP(1);  // the block's loads, the first eθ
    while (true) {
      // Phase A: this member's φ partials, as k_estep_wide
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
          if (rs_pub<CH>(lane) && n < nnz) xs[wave * xr + n] = v;
        }
      }
      for (int n0 = NR; n0 < nnz; n0 += CH) {
        T x[CH];
#pragma unroll
        for (int bb = 0; bb < CH; bb += LB) {
          T y[LB][Q];
          rows_q<T, Q, LB>(a.Bp, ids, sB, kp, t0, NR, nres, nnz, n0 + bb, y);
#pragma unroll
          for (int i = 0; i < LB; ++i) {
            T acc = T(0);
#pragma unroll
            for (int q = 0; q < Q; ++q) acc = fma(y[i][q], eth[q], acc);
            x[bb + i] = acc;
          }
        }
        const T v = rs_chunk<T, CH>(x, lane);
        const int n = n0 + rs_row<CH>(lane);
        if (rs_pub<CH>(lane) && n < nnz) xs[wave * xr + n] = v;
      }
      const T dsum_w = Tr::wsum(dg);
      if (lane == 0) sm.red[0][wave] = dsum_w;
      __syncthreads();  // (1) row sums and Σ|Δγ| published (and any wave's give-up in s_abort)
      STAMP(2);  // Phase A + barrier 1
      if (s_abort) break;
      ++epoch;
      T dotp = T(0);
      if (tid < nnz) {
        dotp = xs[tid];
#pragma unroll
        for (int w = 1; w < kWWaves; ++w) dotp += xs[w * xr + tid];
      }
      T dsp = sm.red[0][0];
#pragma unroll
      for (int w = 1; w < kWWaves; ++w) dsp += sm.red[0][w];
      // one exchange round for both: each lane's row partial and every member's Σ|Δγ| partial
      T dot = T(0), dsum = T(0);
      {
        const int base = (int)(epoch & 1) * P * (int)wt.xstride;
        const bool row = tid < nnz;
        if (pub_ok && row) put_granule<T>(rs, base + member * (int)wt.xstride + tid, epoch, dotp);
        if (pub_ok && tid == 0) put_granule<T>(rs, base + member * (int)wt.xstride + GD, epoch, dsp);
        for (int m = 0; m < P; ++m) {
          T v = T(0), w = T(0);
          if (m == member) {
            v = dotp;
            w = dsp;
          } else {
            for (unsigned spins = 0;; ++spins) {
              // the Σ|Δγ| granule is the same for every lane: lane 0 polls it (readlane below) — 512 threads
              // polling one granule were most of the requests queued at this CU per poll round
              bool ok = lane != 0 || get_granule<T>(rs, base + m * (int)wt.xstride + GD, epoch, w);
              if (row) ok &= get_granule<T>(rs, base + m * (int)wt.xstride + tid, epoch, v);
              if (__all(ok)) break;
              if (spin_give_up(spins, wt.tmo, wt.spin_limit)) {
                if (lane == 0) s_abort = 1;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
            w = readlane_t(w, 0);
          }
          dot += row ? v : T(0);
          dsum += w;
        }
      }
      STAMP(3);  // exchange: publish, poll, member-order sums
      const bool last = (it > 0 && dsum / kd <= T(1e-3)) || it >= a.max_iter;  // team-uniform
      T rd = T(0);
      if (tid < nnz) {
        const T r = cts * Tr::rcp(dot + eps);
        rr[tid] = r;
        rfin = r;
        rd = fma(r, dot, rd);
      }
      rd = Tr::wsum(rd);
      if (lane == 0) sm.red[1][wave] = rd;
      __syncthreads();  // (2) r and Σ r·dot published
      STAMP(4);  // r, Σ r·φ, barrier 2
      if (last || s_abort) break;
      T sg = sm.red[1][0];
#pragma unroll
      for (int w = 1; w < kWWaves; ++w) sg += sm.red[1][w];
      cs = Tr::psi(as + sg);

      // Phase B: s over every row for this member's topics (local)
      T s[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) s[q] = T(0);
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const T r = rr[n];
#pragma unroll
        for (int q = 0; q < Q; ++q) s[q] = fma(B[n][q], r, s[q]);
      }
      for (int n0 = NR; n0 < nnz; n0 += LB) {
        T y[LB][Q];
        rows_q<T, Q, LB>(a.Bp, ids, sB, kp, t0, NR, nres, nnz, n0, y);
#pragma unroll
        for (int i = 0; i < LB; ++i) {
          const T r = n0 + i < nnz ? rr[n0 + i] : T(0);
#pragma unroll
          for (int q = 0; q < Q; ++q) s[q] = fma(y[i][q], r, s[q]);
        }
      }
      dg = T(0);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (t0 + q < k) {
          const T gn = fma(eth[q], s[q], alp[q]);
          dg += fabs(gn - gam[q]);
          gam[q] = gn;
          eth[q] = Tr::eth(gn, cs, pc[q]);
        }
      }
      ++it;
      STAMP(5);  // ψ(Σγ'), Phase B, γ / eθ
    }
    if (s_abort) return;  // a team timed out: every block leaves (the host re-runs the one-CU kernel)

    // ---- outputs: rows from member 0 (identical in every member); this member's topics
    if (member == 0 && tid < nnz) {
      a.r[e0 + tid] = rfin;
      if (STATS) {
        a.keys[e0 + tid] = (uint32_t)ids[tid];
        a.vals[e0 + tid] = entry_val<T>(slot, e0 + tid, rfin);
      }
    }
    // exact Σγ of the final γ over the team (E[log θ] = ψ(γ) − ψ(Σγ))
    double gsd = 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) gsd += (double)gam[q];
    gsd = wave_sum(gsd);
    if (lane == 0) sm.bd[wave][0] = gsd;
    __syncthreads();
    double gpart = 0.0;
    for (int w = 0; w < kWWaves; ++w) gpart += sm.bd[w][0];
    ++epoch;
    const double gsum = (double)exchange(GS, (T)gpart, tid == 0, true);
    if (s_abort) return;
    const double psisum = digamma_t<double>(gsum);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int t = t0 + q;
      if (t < k) {
        if (a.gamma) a.gamma[mem * k + t] = gam[q];
        if (STATS) a.elogth[slot * k + t] = (T)(digamma_t<double>((double)gam[q]) - psisum);
      }
      if (STATS && t < kp && q + Q * tid < kP) a.eth[slot * kp + t] = t < k ? eth[q] : T(0);
    }
    if (member == 0 && tid == 0) {
      if (a.iters) a.iters[mem] = it;
      if (a.nonempty) a.nonempty[mem] = 1;
    }
    __syncthreads();  // LDS (ids, xs, rr, bd, sB) is rewritten by the next document
    STAMP(6);  // outputs, the final Σγ exchange
  }
  STAMP_FLUSH
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

// the team kernel's register rows: WIDE_MC_NR_CUT Phase-A chunks fewer than the one-CU kernel (its
// persistent loop holds more live state; measured: the spills of the uncut form sit outside the inner
// loop, so the default cuts nothing)
#ifndef WIDE_MC_NR_CUT
#define WIDE_MC_NR_CUT 0
#endif
template <typename T, int Q>
constexpr int wide_nr_mc() {
  return wide_nr<T, Q>() - WIDE_MC_NR_CUT * wide_chunk<T, Q>();
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

// rows one CU keeps resident (VGPRs + LDS) for this (T, k): the team size for a document of nnz rows
template <typename T>
int wide_resident_rows(int k) {
  auto rows = [](auto q) {
    constexpr int Q = decltype(q)::value;
    const size_t row_bytes = sizeof(T) * kWThreads * Q;
    return wide_nr_mc<T, Q>() + (int)((kWLds - wide_lds_fixed<T>() - 256) / row_bytes);
  };
  if (k <= kWThreads) return rows(std::integral_constant<int, 1>{});
  if (k <= 2 * kWThreads) return rows(std::integral_constant<int, 2>{});
  return rows(std::integral_constant<int, 4>{});
}

// The persistent team grid, launched only if every block can be resident at once: the kernel's
// occupancy (blocks per CU at this LDS size) × the device's CUs must cover the grid (false: nothing
// launched, the caller runs the one-CU kernel).  A plain launch, not hipLaunchCooperativeKernel: the
// cooperative launch path made every profiled process (rocprofv3 --kernel-trace) fault at exit inside
// the HSA runtime's teardown, after the profiler's finalisation (r03 exit probe: libamdhip64 exit
// handler → libhsa-runtime64, on a /dev/dri mapping already released).  Residency is checked here; a
// block that is nonetheless not co-resident (another process on the device) only delays its team, and
// the bounded spins turn a delay past the limit into a timeout word, on which the host re-runs the
// same slots on the one-CU kernel (api.hip launch_split).
inline bool launch_resident(const void* kern, int blocks, size_t lds, void** args, hipStream_t s) {
  int dev = 0, cus = 0, per_cu = 0;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kWThreads, lds));
  if ((int64_t)per_cu * cus < blocks) return false;
  HIP_CHECK(hipLaunchKernel(kern, dim3((unsigned)blocks), dim3(kWThreads), args, lds, s));
  return true;
}

template <typename T, int Q>
bool launch_q_mc(hipStream_t s, const EStepArgs<T>& a, bool stats, const WideTeam& wt) {
  bool ok = true;
  constexpr int NR = wide_nr_mc<T, Q>();
  const size_t fixed = wide_lds_fixed<T>();
  const size_t row_bytes = sizeof(T) * kWThreads * Q;
  int nl = (int)((kWLds - fixed - 256) / row_bytes);  // 256 B for the kernel's own static word
  const size_t lds = fixed + (size_t)nl * row_bytes;
  auto go = [&](auto kern) {
    HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    EStepArgs<T> aa = a;
    WideTeam ww = wt;
    void* args[] = {&aa, &nl, &ww};
    ok = launch_resident((const void*)kern, wt.blocks, lds, args, s);
  };
  if (stats) go(k_estep_wide_mc<T, Q, NR, true>);
  else go(k_estep_wide_mc<T, Q, NR, false>);
  return ok;
}

template <typename T, int Q>
bool launch_q_tc(hipStream_t s, const EStepArgs<T>& a, bool stats, WideTeam wt) {
  bool ok = true;
  constexpr int NR = wide_nr_mc<T, Q>();
  // the per-row arrays: the launch's longest document (every one when unknown), at least the register rows
  const int mr = wt.max_row >= 0 && wt.max_row <= kWRows ? wt.max_row : kWRows;
  wt.xrows = (std::max(mr, std::max(NR, 2)) + 1) / 2 * 2;
  const size_t fixed = tc_lds_fixed<T>(wt.xrows);
  const size_t row_bytes = sizeof(T) * kWThreads * Q;
  int nl = (int)((kWLds - fixed - 256) / row_bytes);
  const size_t lds = fixed + (size_t)nl * row_bytes;
  auto go = [&](auto kern) {
    HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    EStepArgs<T> aa = a;
    WideTeam ww = wt;
    void* args[] = {&aa, &nl, &ww};
    ok = launch_resident((const void*)kern, wt.blocks, lds, args, s);
  };
  if (stats) go(k_estep_wide_tc<T, Q, NR, true>);
  else go(k_estep_wide_tc<T, Q, NR, false>);
  return ok;
}

// topic split: member topics 512·Q with Q = ⌈k / (512·P)⌉ ≤ 4
template <typename T>
bool launch_estep_wide_tc(hipStream_t s, const EStepArgs<T>& a, bool stats, const WideTeam& wt) {
  if (a.n == 0) return true;
  const int q = (a.k + kWThreads * wt.P - 1) / (kWThreads * wt.P);
  if (q <= 1) return launch_q_tc<T, 1>(s, a, stats, wt);
  if (q <= 2) return launch_q_tc<T, 2>(s, a, stats, wt);
  if (q <= 4) return launch_q_tc<T, 4>(s, a, stats, wt);
  throw Error(STC_ERR_INVALID_ARG, "topic-split team E-step: k > 2048·P");
}
template bool launch_estep_wide_tc<float>(hipStream_t, const EStepArgs<float>&, bool, const WideTeam&);
template bool launch_estep_wide_tc<double>(hipStream_t, const EStepArgs<double>&, bool, const WideTeam&);

template <typename T>
bool launch_estep_wide_mc(hipStream_t s, const EStepArgs<T>& a, bool stats, const WideTeam& wt) {
  if (a.n == 0) return true;
  if (a.k <= kWThreads) return launch_q_mc<T, 1>(s, a, stats, wt);
  if (a.k <= 2 * kWThreads) return launch_q_mc<T, 2>(s, a, stats, wt);
  if (a.k <= 4 * kWThreads) return launch_q_mc<T, 4>(s, a, stats, wt);
  throw Error(STC_ERR_INVALID_ARG, "wide E-step: k > 2048");
}

template int wide_resident_rows<float>(int);
template int wide_resident_rows<double>(int);
template bool launch_estep_wide_mc<float>(hipStream_t, const EStepArgs<float>&, bool, const WideTeam&);
template bool launch_estep_wide_mc<double>(hipStream_t, const EStepArgs<double>&, bool, const WideTeam&);

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

namespace stc {
namespace lda {
STC_STAMP_READER(stc_debug_stamps_wide)
}  // namespace lda
}  // namespace stc
