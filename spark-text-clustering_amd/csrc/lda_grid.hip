// lda_grid.hip — K6 fast path, v2: one document per workgroup of W wavefronts; inside a wave the
// lanes form a 2 × 32 grid — two topic groups × 32 row lanes — so each lane holds up to 6 rows of
// the document's expElogβ' block restricted to KL topics.
//
// Same fixed point as k_estep / [U] OnlineLDAOptimizer.variationalTopicInference (lda.hip has the
// row-scaled numerics), for fp32, k <= 128, nnz <= 32·RMAX:
//   lane bit 3 = topic group g; bits {0,1,2,4,5} = row lane rl; row n = 32·j + rl (j < R, with
//   R = ⌈nnz/32⌉ chosen per document — the rows padding costs at most 31 of the 32·R).
//   wave w, group g own topics [t0, t0 + KL), t0 = (2w + g)·KL.
//   φ_n = B_n·eθ' : lane-local packed FMAs over the group's KL topics, + the other group's partial
//     through one DPP row_ror:8 add (lane i ↔ i^8), then the W wave partials meet in LDS behind one
//     barrier and every wave sums them in the same order ⇒ bit-identical φ and r everywhere.
//   s = Bᵀr : lane-local packed FMAs, reduce-scattered over the 32 row lanes only (permlane32 and
//     permlane16 swaps, then row_half_mirror / quad_perm involutions, all of which keep bit 3):
//     KL values per lane instead of the 52 a topic-split layout (two waves of 52 topics) would hold.
//   γ, ψ(γ), exp on the owned topic (one per lane); eθ' of the group slice back through LDS.
//   ψ(Σγ') from Σγ' = Σα + Σ_n cts_n − Σ_n cts_n·ε'_n/φ_n: a per-document constant unless a ballot
//   finds a row whose ε' is visible at fp32 resolution.
#include "estep_common.h"

namespace stc {
namespace lda {

namespace {

// (waves per document, topics per lane group, max rows per lane, waves per SIMD)
template <int W_, int KL_, int RMAX_, int OCC_>
struct GShape {
  static constexpr int W = W_, KL = KL_, RMAX = RMAX_, OCC = OCC_;
  static constexpr int KLP = (KL + 3) / 4 * 4;  // LDS slice pitch (ds_read_b128 granules)
};
using G32 = GShape<1, 16, 8, 2>;   // k <= 32
using G64 = GShape<2, 16, 8, 2>;   // k <= 64
using G104 = GShape<2, 26, 6, 2>;  // k <= 104 (k = 100: 4 groups of 26 topics)
using G104L = GShape<2, 26, 8, 1>; // k <= 104, documents of 193–256 rows (all eight row sets in VGPRs)
using G128 = GShape<4, 16, 8, 2>;  // k <= 128

template <class S>
struct GLds {
  float eth[S::W][2][S::KLP] __attribute__((aligned(16)));
  // the load stage (one 32-row step of the wave's 2·KL columns) is dead once the loop starts
  union {
    float phi[2][S::W][S::RMAX][64];
    float stage[S::W][32 * 2 * S::KL];
  } __attribute__((aligned(16)));
  float red[2][S::W][2];
  double bd[S::W][2];
};

// cross-wave exchange of nd φ partials per lane + two wave-uniform scalars; one barrier; every
// wave combines them in the same order (for W = 2 a commutative sum of two) ⇒ bit-identical results
// in every wave.  Double-buffered by parity: a buffer is reused only after every wave has passed the
// following barrier (and so finished reading it).
template <class S>
__device__ __forceinline__ void xchg(GLds<S>& sm, int b, int wave, int lane, float* dot, int nd, float& x,
                                     float& y) {
  constexpr int W = S::W;
  if constexpr (W > 1) {
    // addresses from one lane-dependent base (hoisted by the compiler) plus wave-uniform offsets
    float* const base = &sm.phi[0][0][0][0] + lane;
    constexpr int BS = S::W * S::RMAX * 64, WS = S::RMAX * 64;
    float* const mine = base + (b * BS + wave * WS);
#pragma unroll
    for (int j = 0; j < nd; ++j) mine[64 * j] = dot[j];
    if (lane == 0) {
      sm.red[b][wave][0] = x;
      sm.red[b][wave][1] = y;
    }
    __syncthreads();
    if constexpr (W == 2) {
      const int o = wave ^ 1;
      const float* const other = base + (b * BS + o * WS);
#pragma unroll
      for (int j = 0; j < nd; ++j) dot[j] += other[64 * j];
      x += sm.red[b][o][0];
      y += sm.red[b][o][1];
    } else {
#pragma unroll
      for (int j = 0; j < nd; ++j) {
        float d = sm.phi[b][0][j][lane];
#pragma unroll
        for (int w = 1; w < W; ++w) d += sm.phi[b][w][j][lane];
        dot[j] = d;
      }
      x = sm.red[b][0][0];
      y = sm.red[b][0][1];
#pragma unroll
      for (int w = 1; w < W; ++w) {
        x += sm.red[b][w][0];
        y += sm.red[b][w][1];
      }
    }
  }
}

// Per-lane document state shared by the R-independent prologue / epilogue (emitted once per
// kernel) and the R-specialised core (loads, fixed point, token outputs): keeping the once-per-
// document code — fp64 γ₀ sampling, fp64 ψ / lgamma of the outputs — out of the R instances keeps
// the kernel's code small enough for the instruction cache.
struct GDoc {
  int lane, wave, g, rl, nnz, k, kp, t0, tl, t, it;
  bool ok, own;
  int64_t slot, row, mem, s0, e0;
  float gam, alp, pc, eth, cs, gsum, asum;  // pc = exp(−ψ(Σ_v λ_vt)) of the owned topic (EStepArgs::psic)
  double b_tok, c_tok;
#ifdef STC_STAMP
  unsigned long long st0;  // kernel entry (stamp build): the preamble's cycles go to stamp slot 11
#endif
};

template <class S, int R, bool STATS, bool BOUND>
__device__ __forceinline__ bool grid_core(const EStepArgs<float>& a, GLds<S>& sm, GDoc& d) {
  constexpr int W = S::W, KL = S::KL, KLP = S::KLP, H = KL / 2;
  constexpr int N1 = hup(KL), N2 = hup(N1), N3 = hup(N2), N4 = hup(N3), N5 = hup(N4);
  static_assert(KL % 2 == 0 && N5 == 1 && R >= 1 && R <= S::RMAX, "shape");
  STAMP_DECL
#ifdef STC_STAMP
  st_acc[11] += st_last - d.st0;
#endif
  const int lane = d.lane, wave = d.wave, rl = d.rl, nnz = d.nnz, kp = d.kp;
  const int64_t s0 = d.s0, e0 = d.e0;
  float* const my_eth = sm.eth[d.wave][d.g];

  // ---- load, in two dependent rounds with every address valid (no per-load branches, so the loads
  // of a round are in flight together): (1) ids and counts; (2) m_v for ε' and the B rows.  Rows past
  // nnz read entry 0 / term 0 and are zeroed; columns past kp are clamped into the row and zeroed.
  f2 B[R][H];
  float cts[R], eps[R], rr[R];
  int ids[R];
  int any = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int n = 32 * j + rl;
    const bool v = n < nnz;
    const int64_t e = v ? s0 + n : 0;
    const int id = a.indices[e];
    const float c = a.values[e];
    ids[j] = v ? id : 0;
    cts[j] = v ? c : 0.f;
    any |= (cts[j] != 0.f);
    rr[j] = 0.f;
  }
  double ls[R];
#pragma unroll
  for (int j = 0; j < R; ++j) ls[j] = a.logscale[ids[j]];
  // B rows, coalesced: per 32-row step the wave copies its 2·KL columns of the 32 rows with 16-byte
  // loads (consecutive lanes → consecutive pieces of one row), stages them in LDS and every lane
  // picks up its (row, group) part — instead of 8-byte gathers that touch a cache line per lane.
  constexpr int C4 = 2 * KL / 4;                 // float4 pieces per staged row
  constexpr int NP = (32 * C4 + 63) / 64;        // pieces per lane per step
  static_assert((2 * KL) % 4 == 0, "stage rows are float4 multiples");
  const int wcol = wave * 2 * KL;                // the wave's first column
  float* const stg = sm.stage[wave];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    float4 pc[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int c = lane + 64 * i;
      const int srow = c / C4, q = c - srow * C4;
      // the term id of row 32j + srow from the group-0 lane holding it
      const int src_lane = (srow & 7) | ((srow >> 3) << 4);
      const int id = __builtin_amdgcn_ds_bpermute(src_lane << 2, ids[j]);
      const int col = wcol + 4 * q;
      const float4 x = *reinterpret_cast<const float4*>(a.Bp + (int64_t)id * kp + min(col, kp - 4));
      const bool keep = c < 32 * C4 && 32 * j + srow < nnz && col < kp;
      pc[i] = keep ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int c = lane + 64 * i;
      if (c < 32 * C4) *reinterpret_cast<float4*>(stg + 4 * c) = pc[i];  // row c / C4, piece c % C4
    }
    __builtin_amdgcn_wave_barrier();  // one wave writes and reads its stage; LDS is in order per wave
    const float* mine = stg + rl * 2 * KL + d.g * KL;
#pragma unroll
    for (int p = 0; p < H; ++p) {
      const float2 x = *reinterpret_cast<const float2*>(mine + 2 * p);
      B[j][p] = f2{x.x, x.y};
    }
    __builtin_amdgcn_wave_barrier();
  }
  STAMP(10);
  // ε'_n = max(1e-100 / e^{m_n}, FLT_MIN), held as 2^24·ε'_n (φ = dot + 2^-24·that is exact): the
  // ballot below asks 2^24·ε' ≥ φ directly.  Padding rows hold −2^24 (φ = −1, r = −0, never live).
#pragma unroll
  for (int j = 0; j < R; ++j)
    eps[j] = (32 * j + rl < nnz) ? 16777216.f * max_nonneg(__expf((float)(kLogEps - ls[j])), kTiny) : -16777216.f;
  bool nonempty;
  if constexpr (W > 1) nonempty = __syncthreads_or(any) != 0;
  else nonempty = __any(any);

  if (nonempty) {
    float gsum = d.gsum, asum = d.asum, dsum = 0.f, dummy = 0.f;
    xchg<S>(sm, 1, wave, lane, nullptr, 0, gsum, asum);
    d.asum = asum;
    // eθ' = exp(ψ(γ) − ψ(Σγ) − ψc_t): Spark's exp(E[log θ]) times expElogβ's per-topic factor; inside the loop ψ(Σγ') comes from
    // the Σα + Σcts − Σ cts·ε'/φ identity, so without live ε' it is one constant per document
    float cs = digamma_fast(gsum);
    float ct = 0.f;
#pragma unroll
    for (int j = 0; j < R; ++j) ct += cts[j];
    const float ctot = 0.5f * wave_sum_dpp(ct);  // Σ_n cts_n (each row is held by both groups)
    const float cs_flat = digamma_fast(asum + ctot);
    const float alp = d.alp, pc = d.pc;
    float gam = d.gam, eth = d.own ? __expf(digamma_fast(gam) - cs) * pc : 0.f;
    if (d.own) my_eth[d.tl] = eth;
    __builtin_amdgcn_wave_barrier();  // the slices are read back only by this wave
    int it = 0;
    const float k_tol = 1e-3f * (float)d.k;
    float dg = 0.f;  // |Δγ| of the owned topic in the last update
    STAMP(0);
    while (true) {
      // Phase A: φ_n = B_n·eθ + ε'_n ; r_n = cts_n / φ_n
      float dot[R];
      {
        f2 acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = f2{0.f, 0.f};
#pragma unroll
        for (int c = 0; c < KLP / 4; ++c) {
          const float4 e = *reinterpret_cast<const float4*>(my_eth + 4 * c);
          const f2 e01 = f2{e.x, e.y}, e23 = f2{e.z, e.w};
#pragma unroll
          for (int j = 0; j < R; ++j) {
            acc[j] = __builtin_elementwise_fma(B[j][2 * c], e01, acc[j]);
            if (2 * c + 1 < H) acc[j] = __builtin_elementwise_fma(B[j][2 * c + 1], e23, acc[j]);
          }
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const float x = acc[j].x + acc[j].y;
          dot[j] = x + dpp_f<DPP_ROW_ROR8>(x);  // + the other topic group (i ↔ i^8): commutative
        }
      }
      // Σ|Δγ| of the last update, reduced here rather than at the end of that update: the DPP chain
      // shares a basic block with Phase A's LDS reads and FMAs, which hide its latency
      dsum = wave_sum_dpp(dg);
      STAMP(1);
      xchg<S>(sm, it & 1, wave, lane, dot, R, dsum, dummy);  // Σ|Δγ| of the last update rides along
      STAMP(2);
      // wave-uniform by construction (dsum is the same in every lane); readfirstlane tells the compiler,
      // so the loop is a scalar loop: no exec-mask bookkeeping, the counter and offsets in SGPRs
      const bool last =
          __builtin_amdgcn_readfirstlane((int)((it > 0 && dsum <= k_tol) || it >= a.max_iter)) != 0;
      uint64_t eps_live = 0;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const float ph = fmaf(eps[j], 0x1p-24f, dot[j]);
        rr[j] = cts[j] * __builtin_amdgcn_rcpf(ph);
        // ε' ≥ 2^-24·φ: visible in Σγ' (a row with cts = 0 only costs time)
        eps_live |= __builtin_amdgcn_ballot_w64(eps[j] >= ph);
        if (BOUND && last && d.g == 0 && cts[j] != 0.f) {
          d.b_tok += (double)cts[j] * ((double)__logf(fmaxf(dot[j], kTiny)) + a.logscale[ids[j]]);
          d.c_tok += (double)cts[j];
        }
      }
      STAMP(3);
      if (last) break;
      // ψ(Σγ') for the next eθ from Σγ' = Σα + Σ_n cts_n − Σ_n cts_n·ε'_n/φ_n (exact in real
      // arithmetic).  The ε' part is below the fp32 resolution of Σγ' unless some row has
      // ε'_n ≥ 2^-24·φ_n (a ballot); only then is it reduced.  The decision and the sums are the same
      // in every wave (like φ and r), so every wave scales its eθ slice identically.
      float cs_next = cs_flat;
      if (eps_live) {
        float e = 0.f;
#pragma unroll
        for (int j = 0; j < R; ++j)  // cts·ε'/φ as cts·(1 − dot/φ): 0 for padding, cts when ε' = ∞
          e = fmaf(cts[j], 1.f - dot[j] * __builtin_amdgcn_rcpf(fmaf(eps[j], 0x1p-24f, dot[j])), e);
        cs_next = digamma_fast(asum + ctot - 0.5f * wave_sum_dpp(e));  // each row is held twice
      }
      STAMP(4);

      // Phase B: s = Bᵀr over the group's KL topics, then reduce-scatter over the 32 row lanes
      float flat[KL];
#pragma unroll
      for (int p = 0; p < H; ++p) {
        f2 x = f2{0.f, 0.f};
#pragma unroll
        for (int j = 0; j < R; ++j) x = __builtin_elementwise_fma(B[j][p], f2{rr[j], rr[j]}, x);
        flat[2 * p] = x.x;
        flat[2 * p + 1] = x.y;
      }
      STAMP(5);
      float ys1[N1];
#pragma unroll
      for (int q = 0; q < N1; ++q) ys1[q] = (N1 + q < KL) ? flat[N1 + q] : 0.f;
      float p1[N1];
      swap_add_n<true, N1>(flat, ys1, p1);  // bit 5
      float ys2[N2];
#pragma unroll
      for (int q = 0; q < N2; ++q) ys2[q] = (N2 + q < N1) ? p1[N2 + q] : 0.f;
      float p2[N2];
      swap_add_n<false, N2>(p1, ys2, p2);  // bit 4
      float p3[N3];
#pragma unroll
      for (int q = 0; q < N3; ++q)
        p3[q] = rs_dpp<DPP_ROW_HALF_MIRROR>(p2[q], (N3 + q < N2) ? p2[N3 + q] : 0.f, lane & 4);
      float p4[N4];
#pragma unroll
      for (int q = 0; q < N4; ++q)
        p4[q] = rs_dpp<DPP_QP_3210>(p3[q], (N4 + q < N3) ? p3[N4 + q] : 0.f, lane & 2);
      float y5 = 0.f;
      if constexpr (N5 < N4) y5 = p4[N5];
      const float s_own = rs_dpp<DPP_QP_1032>(p4[0], y5, lane & 1);
      STAMP(6);

      // Phase C: γ ← eθ ⊙ s + α on the owned topic (lanes without one keep γ = 0 and dg = 0)
      {
        const float gn = fmaf(eth, s_own, alp);
        dg = d.own ? fabsf(gn - gam) : 0.f;
        gam = d.own ? gn : gam;
      }
      STAMP(7);
      // Phase D: eθ' = exp(ψ(γ) − ψ(Σγ) − ψc) into the group's LDS slice; computed in every lane (no
      // exec-mask region), stored by the owners
      cs = cs_next;
      eth = d.own ? __expf(digamma_fast(d.own ? gam : 1.f) - cs) * pc : 0.f;
      if (d.own) my_eth[d.tl] = eth;
      __builtin_amdgcn_wave_barrier();
      ++it;
      STAMP(8);
    }
    d.gam = gam;
    d.eth = eth;
    d.cs = cs;
    d.it = it;
  }
  // ---- token-level outputs (wave 0's group-0 lanes hold each row once)
  if (wave == 0 && d.g == 0) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int n = 32 * j + rl;
      if (n < nnz) {
        a.r[e0 + n] = rr[j];
        if (STATS) {
          a.keys[e0 + n] = (uint32_t)ids[j];
          a.vals[e0 + n] = entry_val<float>(d.slot, e0 + n, rr[j]);
        }
      }
    }
  }
  STAMP(9);
  STAMP_FLUSH
  return nonempty;
}

// one document of slot `slot` with thread index `tid` (the resident long-document kernel passes a
// per-document laundered copy, so nothing lane-dependent is hoisted out of its document loop);
// SKIPLONG: leave documents past S::RMAX row sets to the long-document kernel
template <class S, bool STATS, bool BOUND, bool SKIPLONG>
__device__ __forceinline__ void grid_doc(const EStepArgs<float>& a, GLds<S>& sm, int64_t slot_, int tid) {
  constexpr int W = S::W, KL = S::KL;
  constexpr int N1 = hup(KL), N2 = hup(N1), N3 = hup(N2), N4 = hup(N3), N5 = hup(N4);
  GDoc d;
#ifdef STC_STAMP
  d.st0 = stamp_now();
#endif
  d.lane = tid & 63;
  d.wave = tid >> 6;
  d.g = (d.lane >> 3) & 1;
  d.rl = (d.lane & 7) | ((d.lane >> 4) << 3);
  d.slot = slot_;
  d.row = a.batch ? (int64_t)a.batch[d.slot] : d.slot;
  d.mem = a.orig ? (int64_t)a.orig[d.slot] : d.slot;
  d.s0 = a.indptr[d.row];
  d.nnz = (int)(a.indptr[d.row + 1] - d.s0);
  if (SKIPLONG && ((d.nnz + 31) >> 5) > S::RMAX) return;
  d.e0 = a.bptr ? a.bptr[d.slot] : d.s0;
  d.k = a.k;
  d.kp = a.kp;
  d.t0 = (2 * d.wave + d.g) * KL;
  // the topic this lane owns after the reduce-scatter (levels: bit 5, 4, 2, 1, 0)
  const int lane = d.lane;
  int tl = (lane & 1) ? N5 : 0;
  bool ok = tl < N4;
  tl += (lane & 2) ? N4 : 0;
  ok &= tl < N3;
  tl += (lane & 4) ? N3 : 0;
  ok &= tl < N2;
  tl += (lane & 16) ? N2 : 0;
  ok &= tl < N1;
  tl += (lane & 32) ? N1 : 0;
  ok &= tl < KL;
  d.tl = tl;
  d.ok = ok;
  d.t = d.t0 + tl;
  d.own = ok && d.t < d.k;
  const int k = d.k, kp = d.kp, t = d.t;
  const int64_t mem = d.mem, slot = d.slot;
  // ---- γ₀, α on the owned topic; Σγ, Σα over the wave's topics
  uint64_t stream = 0;
  if (!a.gamma0) {
    const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem) : (uint64_t)(a.doc_id_base + d.row);
    stream = doc_stream(a.seed, key);
  }
  d.gam = d.own ? (a.gamma0 ? a.gamma0[mem * k + t] : (float)gamma_sample(stream, t, a.gamma_shape)) : 0.f;
  d.alp = d.own ? (float)a.alpha[t] : 0.f;
  d.pc = d.own ? (float)a.psic[d.k + t] : 0.f;
  d.gsum = wave_sum_dpp(d.gam);
  d.asum = wave_sum_dpp(d.alp);
  for (int i = lane; i < 2 * S::KLP; i += 64) (&sm.eth[d.wave][0][0])[i] = 0.f;  // pads stay zero
  d.eth = 0.f;
  d.cs = 0.f;
  d.it = 0;
  d.b_tok = 0.0;
  d.c_tok = 0.0;

  // rows per lane for this document (block-uniform); the partition guarantees nnz <= 32·RMAX
  bool nonempty = false;
  switch ((d.nnz + 31) >> 5) {
    case 0:
    case 1: nonempty = grid_core<S, 1, STATS, BOUND>(a, sm, d); break;
    case 2: nonempty = grid_core<S, 2, STATS, BOUND>(a, sm, d); break;
    case 3: nonempty = grid_core<S, 3, STATS, BOUND>(a, sm, d); break;
    case 4: nonempty = grid_core<S, 4, STATS, BOUND>(a, sm, d); break;
    case 5: nonempty = grid_core<S, 5, STATS, BOUND>(a, sm, d); break;
    case 6: nonempty = grid_core<S, 6, STATS, BOUND>(a, sm, d); break;
    default:
      if constexpr (S::RMAX >= 8) {
        if (d.nnz <= 224) nonempty = grid_core<S, 7, STATS, BOUND>(a, sm, d);
        else nonempty = grid_core<S, 8, STATS, BOUND>(a, sm, d);
      }
      break;
  }

  // ---- topic-level outputs, once per kernel
  const int wave = d.wave;
  if (!nonempty) {
    if (d.own) {
      if (a.gamma) a.gamma[mem * k + t] = 0.f;
      if (STATS) a.elogth[slot * k + t] = 0.f;
    }
    if (STATS && d.ok && t < kp) a.eth[slot * kp + t] = 0.f;
    if (wave == 0 && lane == 0) {
      if (a.iters) a.iters[mem] = 0;
      if (a.nonempty) a.nonempty[mem] = 0;
      if (BOUND) a.bound[mem] = 0.0;
    }
    return;
  }
  // exact Σγ of the final γ (outputs and bound); the loop's last barrier used buffer it & 1
  float gsum = wave_sum_dpp(d.own ? d.gam : 0.f), dummy = 0.f;
  xchg<S>(sm, (d.it + 1) & 1, wave, lane, nullptr, 0, gsum, dummy);
  const double psisum = digamma_t<double>((double)gsum);
  if (d.own) {
    if (a.gamma) a.gamma[mem * k + t] = d.gam;
    if (STATS) a.elogth[slot * k + t] = (float)(digamma_t<double>((double)d.gam) - psisum);
  }
  if (STATS && d.ok && t < kp) a.eth[slot * kp + t] = sm.eth[wave][d.g][d.tl];  // the eθ' φ used
  if (wave == 0 && lane == 0) {
    if (a.iters) a.iters[mem] = d.it;
    if (a.nonempty) a.nonempty[mem] = 1;
  }
  if (BOUND) {
    // token terms from the group-0 lanes of wave 0 (each row once); topic terms summed over waves
    double topic = 0.0, as = 0.0;
    if (d.own) {
      const double gd = (double)d.gam, al = a.alpha[t];
      const double el = digamma_t<double>(gd) - psisum;
      topic = (al - gd) * el + (lgamma(gd) - lgamma(al));
      as = al;
    }
    topic = wave_sum(topic);
    as = wave_sum(as);
    const double tok = wave_sum(d.b_tok), ct = wave_sum(d.c_tok);
    if (lane == 0) {
      sm.bd[wave][0] = topic;
      sm.bd[wave][1] = as;
    }
    if constexpr (W > 1) __syncthreads();
    if (wave == 0 && lane == 0) {
      double tp = 0.0, asw = 0.0;
      for (int w = 0; w < W; ++w) {
        tp += sm.bd[w][0];
        asw += sm.bd[w][1];
      }
      const double elog_max = (double)d.cs - psisum;  // log of the scale eθ carried (≈ 0)
      a.bound[mem] = tok + ct * elog_max + tp + (lgamma(asw) - lgamma((double)gsum));
    }
  }
}

// one workgroup per slot; SKIPLONG: the long-document kernel takes the documents past S::RMAX sets
template <class S, bool STATS, bool BOUND, bool SKIPLONG>
__global__ __launch_bounds__(64 * S::W, S::OCC) void k_estep_grid(EStepArgs<float> a) {
  __shared__ GLds<S> sm;
  if ((int64_t)blockIdx.x >= a.n) return;
  grid_doc<S, STATS, BOUND, SKIPLONG>(a, sm, a.slot0 + blockIdx.x, (int)threadIdx.x);
}

// the same on a resident grid taking tickets (as lda_rows64.hip k_estep_rows64_pers): the next ticket is
// requested at a document's start and read at its end; tid laundered per document
template <class S, bool STATS, bool BOUND, bool SKIPLONG>
__global__ __launch_bounds__(64 * S::W, S::OCC) void k_estep_grid_pers(EStepArgs<float> a, int32_t* ticket) {
  __shared__ GLds<S> sm;
  __shared__ int s_tk;
  if (threadIdx.x == 0) s_tk = atomicAdd(ticket, 1);
  __syncthreads();
  int cur = s_tk;
  while (cur < a.n) {
    __syncthreads();  // every thread has read s_tk
    int nxt = 0;
    if (threadIdx.x == 0) nxt = atomicAdd(ticket, 1);
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    grid_doc<S, STATS, BOUND, SKIPLONG>(a, sm, a.slot0 + cur, tid);
    if (threadIdx.x == 0) s_tk = nxt;
    __syncthreads();  // LDS is the next document's; s_tk published
    cur = s_tk;
  }
}

// the launch's documents past `rows` rows into a.long_list (word 0 the count, then slot offsets)
__global__ void k_grid_long_list(EStepArgs<float> a, int rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int64_t slot = a.slot0 + i;
  const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
  if ((int)(a.indptr[row + 1] - a.indptr[row]) > rows) a.long_list[1 + atomicAdd(&a.long_list[0], 1)] = (int32_t)i;
}

// the listed long documents on a resident grid (as lda_rows64.hip's long-document kernel)
template <class S, bool STATS, bool BOUND>
__global__ __launch_bounds__(64 * S::W, S::OCC) void k_estep_grid_long(EStepArgs<float> a) {
  __shared__ GLds<S> sm;
  const int cnt = a.long_list[0];
  for (int j = blockIdx.x; j < cnt; j += gridDim.x) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    grid_doc<S, STATS, BOUND, false>(a, sm, a.slot0 + a.long_list[1 + j], tid);
    __syncthreads();  // LDS is the next document's
  }
}

// diagnostic: STC_GRID_LDS_PAD bytes of unused dynamic LDS per workgroup lower the occupancy
// (e.g. 80000 → one wave per SIMD), to read the stamps' per-phase latencies without a partner wave
size_t lds_pad() {
  static const size_t v = [] {
    const char* e = getenv("STC_GRID_LDS_PAD");
    return e ? (size_t)atol(e) : (size_t)0;
  }();
  return v;
}

#ifndef GRID_PERSIST
#define GRID_PERSIST 1  // the documents on a resident grid taking tickets (1) or one workgroup per slot (0)
#endif
template <class S, bool SKIPLONG>
bool launch_g_persist(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  if (!GRID_PERSIST || !a.long_list || lds_pad() != 0 || bound) return false;  // (the bound kernels spill resident)
  int32_t* ticket = a.long_list + a.n + 1;  // the word past the long-document list (api.hip reserves it)
  auto go = [&](const void* kern) {
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * S::W, 0));
    if (per_cu < 1) return false;
    HIP_CHECK(hipMemsetAsync(ticket, 0, sizeof(int32_t), s));
    EStepArgs<float> aa = a;
    void* args[] = {&aa, &ticket};
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(a.n, (int64_t)per_cu * cus));
    HIP_CHECK(hipLaunchKernel(kern, dim3((unsigned)blocks), dim3(64 * S::W), args, 0, s));
    return true;
  };
  if (stats) return go((const void*)k_estep_grid_pers<S, true, false, SKIPLONG>);
  return go((const void*)k_estep_grid_pers<S, false, false, SKIPLONG>);
}
template <class S, bool SKIPLONG = false>
void launch_g(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  if (launch_g_persist<S, SKIPLONG>(s, a, stats, bound)) return;
  const dim3 grid((unsigned)a.n);
  const int threads = 64 * S::W;
  const size_t pad = lds_pad();
  if (stats) k_estep_grid<S, true, false, SKIPLONG><<<grid, threads, pad, s>>>(a);
  else if (bound) k_estep_grid<S, false, true, SKIPLONG><<<grid, threads, pad, s>>>(a);
  else k_estep_grid<S, false, false, SKIPLONG><<<grid, threads, pad, s>>>(a);
  KERNEL_CHECK();
}
// documents of S::RMAX < sets ≤ L::RMAX: listed on the device, run by L's kernel on a resident grid
// (one workgroup per SIMD pair at one wave per SIMD), then the rest by S's kernel
template <class S, class L>
void launch_g_split(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  if (!a.long_list) throw Error(STC_ERR_STATE, "grid E-step: no long-document list buffer");
  HIP_CHECK(hipMemsetAsync(a.long_list, 0, sizeof(int32_t), s));
  k_grid_long_list<<<dim3((unsigned)((a.n + 255) / 256)), 256, 0, s>>>(a, 32 * S::RMAX);
  KERNEL_CHECK();
  int dev = 0, cus = 0;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int threads = 64 * L::W;
  auto run = [&](auto kern) {
    int per_cu = 0;  // workgroups resident per CU at this kernel's registers / LDS
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0));
    const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(a.n, (int64_t)cus * std::max(1, per_cu))));
    kern<<<grid, threads, 0, s>>>(a);
  };
  if (stats) run(k_estep_grid_long<L, true, false>);
  else if (bound) run(k_estep_grid_long<L, false, true>);
  else run(k_estep_grid_long<L, false, false>);
  KERNEL_CHECK();
  launch_g<S, true>(s, a, stats, bound);
}

}  // namespace

int grid_row_cap(int k) {
  if (k <= 64) return 32 * G64::RMAX;
  if (k <= 104) return 32 * G104L::RMAX;
  if (k <= 128) return 32 * G128::RMAX;
  return 0;
}
int grid_onchip_rows(int k) { return k > 64 && k <= 104 ? 32 * G104::RMAX : grid_row_cap(k); }

void launch_estep_grid(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound, bool long_docs) {
  if (a.n == 0) return;
  if (a.k <= 32) launch_g<G32>(s, a, stats, bound);
  else if (a.k <= 64) launch_g<G64>(s, a, stats, bound);
  else if (a.k <= 104) {
    if (long_docs) launch_g_split<G104, G104L>(s, a, stats, bound);
    else launch_g<G104>(s, a, stats, bound);
  }
  else if (a.k <= 128) launch_g<G128>(s, a, stats, bound);
  else throw Error(STC_ERR_INVALID_ARG, "grid E-step: k > 128");
}

}  // namespace lda
}  // namespace stc

STC_STAMP_READER(stc_debug_stamps_grid)
