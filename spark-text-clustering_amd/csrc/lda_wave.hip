// lda_wave.hip — K6 fast path: one document per workgroup of W wavefronts, the topics split
// across the waves, the document block held in VGPRs.
//
// Same fixed point as k_estep / [U] OnlineLDAOptimizer.variationalTopicInference (see lda.hip for
// the row-scaled numerics), specialised for fp32, k <= 128 and nnz <= 64·ROWS:
//   wave w owns the topic slice [w·KW, (w+1)·KW); lane l of every wave holds rows n = l, l+64, …
//   (ROWS of them) of B = expElogβ'[ids, slice] — ROWS·KW floats, small enough for two waves per
//   SIMD without AGPR spills.
//   φ_n = B_n·eθ' : each wave dots its own slice (eθ' from its LDS slice with ds_read_b128); the W
//     partials meet in LDS behind one barrier and every wave sums them in the same order, so all
//     waves hold bit-identical φ and r.
//   s = Bᵀr : lane-local products reduce-scattered across the 64 lanes over the wave's slice only
//     (v_permlane32/16 swaps halve the set twice, then four DPP involutions) — every lane ends
//     owning ⌈KW/64⌉ topics, where γ, ψ(γ) and exp run; no cross-wave traffic.
//   Σ|Δγ| of each update rides along with the next φ exchange; ψ(Σγ) for eθ comes from the
//   identity Σγ' = Σα + Σ_n r_n·dot_n, which every wave holds without an exchange.
// Per inner iteration and lane: 2·ROWS·KW FMAs, ~100 permute/add/select, one barrier (W > 1).
#include "estep_common.h"

namespace stc {
namespace lda {

namespace {

// (waves per document, topics per wave, rows per lane, waves per SIMD the registers allow)
template <int W_, int KW_, int ROWS_, int OCC_>
struct Shape {
  static constexpr int W = W_, KW = KW_, ROWS = ROWS_, OCC = OCC_;
};
// k <= 64 / <= 104 / <= 128.  k = 100: slices [0,52) and [52,100), 16-byte aligned row offsets.
using Shape64 = Shape<2, 32, 4, 2>;
using Shape104 = Shape<2, 52, 3, 2>;
using Shape128 = Shape<4, 32, 3, 2>;
// alternatives kept selectable for measurement (STC_WAVE_SHAPE=1..)
using Shape104b = Shape<4, 28, 3, 3>;
using Shape104c = Shape<4, 28, 4, 2>;
using Shape104d = Shape<3, 36, 3, 3>;

template <int KW>
constexpr int lvl(int L) {
  int n = KW;
  for (int i = 0; i < L; ++i) n = hup(n);
  return n;
}

template <class S, bool STATS, bool BOUND>
__global__ __launch_bounds__(64 * S::W, S::OCC) void k_estep_split(EStepArgs<float> a) {
  constexpr int W = S::W, KW = S::KW, ROWS = S::ROWS;
  constexpr int C4 = KW / 4;
  constexpr int N1 = lvl<KW>(1), N2 = lvl<KW>(2), N3 = lvl<KW>(3), N4 = lvl<KW>(4), N5 = lvl<KW>(5),
                N6 = lvl<KW>(6);
  constexpr int H = KW / 2;  // topic pairs per row
  static_assert(KW % 4 == 0 && N1 == H && H % 2 == 0 && N6 >= 1, "shape");
  __shared__ __attribute__((aligned(16))) float s_eth[W][KW];
  __shared__ float s_phi[2][W][ROWS][64];
  __shared__ float s_red[2][W][3];
  __shared__ double s_bd[W][2];

  if ((int64_t)blockIdx.x >= a.n) return;
  STAMP_DECL
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t slot = a.slot0 + blockIdx.x;
  const int64_t mem = a.orig ? (int64_t)a.orig[slot] : slot;
  const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
  const int64_t s0 = a.indptr[row];
  const int nnz = (int)(a.indptr[row + 1] - s0);
  const int64_t e0 = a.bptr ? a.bptr[slot] : s0;
  const int k = a.k, kp = a.kp;
  const int t0 = wave * KW;  // first topic of this wave's slice (multiple of 4)
  float* const my_eth = s_eth[wave];

  // topics owned after the reduce-scatter: slot s ↦ slice index tl[s]; owned only if the relative
  // index stays inside every level's set (odd-sized sets are padded by one zero) and is a topic
  int tl[N6];
  bool own[N6];
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    int r = s;
    bool v = true;
    r += (lane & 1) ? N6 : 0;
    v &= r < N5;
    r += (lane & 2) ? N5 : 0;
    v &= r < N4;
    r += (lane & 4) ? N4 : 0;
    v &= r < N3;
    r += (lane & 8) ? N3 : 0;
    v &= r < N2;
    r += (lane & 16) ? N2 : 0;
    v &= r < N1;
    r += (lane & 32) ? N1 : 0;
    v &= r < KW;
    tl[s] = v ? r : 0;
    own[s] = v && t0 + r < k;
  }

  // ---- load the document: ids, counts, ε-log-scales and this wave's slice of the B rows
  f2 B[ROWS][H];  // B[j][p] = topics (2p, 2p+1) of row j: packed-FMA operands
  float cts[ROWS], lse[ROWS], rr[ROWS];
  int ids[ROWS];
  int any = 0;
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int n = j * 64 + lane;
    const bool v = n < nnz;
    ids[j] = v ? a.indices[s0 + n] : 0;
    cts[j] = v ? a.values[s0 + n] : 0.f;
    lse[j] = v ? (float)(kLogEps - a.logscale[ids[j]]) : 0.f;
    any |= (cts[j] != 0.f);
    const float4* src = reinterpret_cast<const float4*>(a.Bp + (int64_t)ids[j] * kp + t0);
#pragma unroll
    for (int c = 0; c < C4; ++c) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (v && t0 + 4 * c < kp) x = src[c];
      B[j][2 * c] = f2{x.x, x.y};
      B[j][2 * c + 1] = f2{x.z, x.w};
    }
  }
  bool nonempty;
  if constexpr (W > 1) nonempty = __syncthreads_or(any) != 0;
  else nonempty = __any(any);
  if (!nonempty) {
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      if (own[s]) {
        const int t = t0 + tl[s];
        if (a.gamma) a.gamma[mem * k + t] = 0.f;
        if (STATS) a.elogth[slot * k + t] = 0.f;
      }
    }
    if (STATS)
      for (int t = lane; t < KW && t0 + t < kp; t += 64) a.eth[slot * kp + t0 + t] = 0.f;
    if (wave == 0) {
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        const int n = j * 64 + lane;
        if (n < nnz) {
          a.r[e0 + n] = 0.f;
          if (STATS) {
            a.keys[e0 + n] = (uint32_t)ids[j];
            a.vals[e0 + n] = entry_val<float>(slot, e0 + n, 0.f);
          }
        }
      }
      if (lane == 0) {
        if (a.iters) a.iters[mem] = 0;
        if (a.nonempty) a.nonempty[mem] = 0;
        if (BOUND) a.bound[mem] = 0.0;
      }
    }
    return;
  }

  // Cross-wave exchange: each wave publishes its φ partials (ROWS per lane) and up to two wave-
  // uniform scalars; one barrier; every wave combines them in the same order (a sum of two is
  // commutative, so for W = 2 each wave adds the other's values to its own) ⇒ bit-identical
  // results in every wave.  Double-buffered by parity: a wave can only reuse a buffer after every
  // wave has passed the following barrier (and so finished reading it).
  auto exchange = [&](int b, float* dot, int nd, float& x, float& y) {
    if constexpr (W > 1) {
#pragma unroll
      for (int j = 0; j < nd; ++j) s_phi[b][wave][j][lane] = dot[j];
      if (lane == 0) {
        s_red[b][wave][0] = x;
        s_red[b][wave][1] = y;
      }
      __syncthreads();
      if constexpr (W == 2) {
        const int o = wave ^ 1;
#pragma unroll
        for (int j = 0; j < nd; ++j) dot[j] += s_phi[b][o][j][lane];
        x += s_red[b][o][0];
        y += s_red[b][o][1];
      } else {
#pragma unroll
        for (int j = 0; j < nd; ++j) {
          float d = s_phi[b][0][j][lane];
#pragma unroll
          for (int w = 1; w < W; ++w) d += s_phi[b][w][j][lane];
          dot[j] = d;
        }
        x = s_red[b][0][0];
        y = s_red[b][0][1];
#pragma unroll
        for (int w = 1; w < W; ++w) {
          x += s_red[b][w][0];
          y += s_red[b][w][1];
        }
      }
    }
  };

  // ---- γ₀ for the owned topics
  uint64_t stream = 0;
  if (!a.gamma0) {
    const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem) : (uint64_t)(a.doc_id_base + row);
    stream = doc_stream(a.seed, key);
  }
  float gam[N6], eth[N6], alp[N6];
  float gsum = 0.f, asum = 0.f;
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    const int t = t0 + tl[s];
    gam[s] = own[s] ? (a.gamma0 ? a.gamma0[mem * k + t] : (float)gamma_sample(stream, t, a.gamma_shape)) : 0.f;
    alp[s] = own[s] ? (float)a.alpha[t] : 0.f;
    gsum += gam[s];
    asum += alp[s];
  }
  for (int t = lane; t < KW; t += 64) my_eth[t] = 0.f;  // slice padding (t0 + t >= k) stays zero
  gsum = wave_sum_dpp(gsum);
  asum = wave_sum_dpp(asum);
  exchange(1, nullptr, 0, gsum, asum);
  // eθ = exp(ψ(γ) − c) with c = ψ(Σγ): Spark's own (unscaled) exp(E[log θ]).  Inside the loop Σγ of
  // the next γ comes from Σ_t γ'_t = Σα + Σ_n r_n·dot_n (exact in real arithmetic), which every wave
  // holds identically — no exchange, off the critical path.  c is only a common scale: φ, r and
  // the statistics are invariant to it, so rounding in Σγ̃ does not move the fixed point.
  float cs = digamma_fast(gsum);
  // ε'_n = max(1e-100 / e^{m_n}, FLT_MIN): Spark's φ epsilon in the row-scaled space
  float eps[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) eps[j] = max_nonneg(__expf(lse[j]), kTiny);
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    eth[s] = own[s] ? __expf(digamma_fast(gam[s]) - cs) : 0.f;
    if (own[s]) my_eth[tl[s]] = eth[s];
  }
  __builtin_amdgcn_wave_barrier();  // the slice is read back only by this wave

  int it = 0;
  float dsum = 0.f, dummy = 0.f;
  double b_tok = 0.0, c_tok = 0.0;
  STAMP(0);  // load + γ₀ + first eθ
  while (true) {
    // Phase A: φ_n = B_n·eθ + ε'_n ; r_n = cts_n / φ_n
    // (even and odd topics accumulate in the two halves of a packed pair)
    float dot[ROWS];
    {
      f2 acc[ROWS];
#pragma unroll
      for (int j = 0; j < ROWS; ++j) acc[j] = f2{0.f, 0.f};
#pragma unroll
      for (int c = 0; c < C4; ++c) {
        const float4 e = *reinterpret_cast<const float4*>(my_eth + 4 * c);
        const f2 e01 = f2{e.x, e.y}, e23 = f2{e.z, e.w};
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {  // rows past nnz are zero: no per-row branches
          acc[j] = __builtin_elementwise_fma(B[j][2 * c], e01, acc[j]);
          acc[j] = __builtin_elementwise_fma(B[j][2 * c + 1], e23, acc[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < ROWS; ++j) dot[j] = acc[j].x + acc[j].y;
    }
    STAMP(1);  // phase A: eθ LDS reads + φ FMAs
    // Σ|Δγ| of the update that produced the current γ rides along
    exchange(it & 1, dot, ROWS, dsum, dummy);
    STAMP(2);  // cross-wave φ exchange (LDS + barrier)
    const bool last = (it > 0 && dsum <= 1e-3f * (float)k) || it >= a.max_iter;
    float sg = 0.f;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      rr[j] = cts[j] * __builtin_amdgcn_rcpf(dot[j] + eps[j]);
      sg = fmaf(rr[j], dot[j], sg);
      if (BOUND && last && cts[j] != 0.f) {
        b_tok += (double)cts[j] * ((double)__logf(fmaxf(dot[j], kTiny)) + a.logscale[ids[j]]);
        c_tok += (double)cts[j];
      }
    }
    STAMP(3);  // r = cts/φ, Σ r·dot
    if (last) break;
    const float cs_next = digamma_fast(asum + wave_sum_dpp(sg));  // ψ(Σγ') for the next eθ
    STAMP(4);  // ψ(Σγ')

    // Phase B: s = Bᵀ r over the slice, reduce-scattered so the lane owns p6[0 .. N6)
    // (pairs: topics (2p, 2p+1) → xs, (N1+2p, N1+2p+1) → ys; r_j broadcast to both halves)
    float xs[N1], ys[N1];
#pragma unroll
    for (int p = 0; p < H / 2; ++p) {
      f2 x = f2{0.f, 0.f}, y = f2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        const f2 rj = f2{rr[j], rr[j]};
        x = __builtin_elementwise_fma(B[j][p], rj, x);
        y = __builtin_elementwise_fma(B[j][H / 2 + p], rj, y);
      }
      xs[2 * p] = x.x;
      xs[2 * p + 1] = x.y;
      ys[2 * p] = y.x;
      ys[2 * p + 1] = y.y;
    }
    STAMP(5);  // phase B FMAs
    float p1[N1];
    swap_add_n<true, N1>(xs, ys, p1);
    float ys2[N2];
#pragma unroll
    for (int q = 0; q < N2; ++q) ys2[q] = (N2 + q < N1) ? p1[N2 + q] : 0.f;
    float p2[N2];
    swap_add_n<false, N2>(p1, ys2, p2);
    float p3[N3];
#pragma unroll
    for (int q = 0; q < N3; ++q)
      p3[q] = rs_dpp<DPP_ROW_MIRROR>(p2[q], (N3 + q < N2) ? p2[N3 + q] : 0.f, lane & 8);
    float p4[N4];
#pragma unroll
    for (int q = 0; q < N4; ++q)
      p4[q] = rs_dpp<DPP_ROW_HALF_MIRROR>(p3[q], (N4 + q < N3) ? p3[N4 + q] : 0.f, lane & 4);
    float p5[N5];
#pragma unroll
    for (int q = 0; q < N5; ++q)
      p5[q] = rs_dpp<DPP_QP_3210>(p4[q], (N5 + q < N4) ? p4[N5 + q] : 0.f, lane & 2);
    float p6[N6];
#pragma unroll
    for (int q = 0; q < N6; ++q)
      p6[q] = rs_dpp<DPP_QP_1032>(p5[q], (N6 + q < N5) ? p5[N6 + q] : 0.f, lane & 1);
    STAMP(6);  // reduce-scatter

    // Phase C: γ ← eθ ⊙ s + α on the owned topics; this wave's Σ|Δγ|
    dsum = 0.f;
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      if (own[s]) {
        const float g = fmaf(eth[s], p6[s], alp[s]);
        dsum += fabsf(g - gam[s]);
        gam[s] = g;
      }
    }
    dsum = wave_sum_dpp(dsum);
    STAMP(7);  // phase C: γ, Σ|Δγ|
    // Phase D: eθ = exp(ψ(γ) − ψ(Σγ)) into the wave's LDS slice
    cs = cs_next;
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      if (own[s]) {
        eth[s] = __expf(digamma_fast(gam[s]) - cs);
        my_eth[tl[s]] = eth[s];
      }
    }
    __builtin_amdgcn_wave_barrier();
    ++it;
    STAMP(8);  // phase D: ψ/exp, eθ to LDS
  }

  // exact Σγ of the final γ (outputs and bound); the loop's last barrier used buffer it & 1
  gsum = 0.f;
#pragma unroll
  for (int s = 0; s < N6; ++s) gsum += gam[s];
  gsum = wave_sum_dpp(gsum);
  exchange((it + 1) & 1, nullptr, 0, gsum, dummy);

  // ---- outputs: topic-level from each wave's slice, token-level from wave 0
  const double psisum = digamma_t<double>((double)gsum);
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    if (own[s]) {
      const int t = t0 + tl[s];
      if (a.gamma) a.gamma[mem * k + t] = gam[s];
      if (STATS) a.elogth[slot * k + t] = (float)(digamma_t<double>((double)gam[s]) - psisum);
    }
  }
  if (STATS)  // the eθ' φ was computed with (slice pads are zero)
    for (int t = lane; t < KW && t0 + t < kp; t += 64) a.eth[slot * kp + t0 + t] = my_eth[t];
  if (wave == 0) {
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int n = j * 64 + lane;
      if (n < nnz) {
        a.r[e0 + n] = rr[j];
        if (STATS) {
          a.keys[e0 + n] = (uint32_t)ids[j];
          a.vals[e0 + n] = entry_val<float>(slot, e0 + n, rr[j]);
        }
      }
    }
    if (lane == 0) {
      if (a.iters) a.iters[mem] = it;
      if (a.nonempty) a.nonempty[mem] = 1;
    }
  }
  if (BOUND) {
    // token terms are identical in every wave (taken from wave 0); topic terms summed over waves
    double topic = 0.0, asum = 0.0;
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      if (own[s]) {
        const double g = (double)gam[s], al = a.alpha[t0 + tl[s]];
        const double el = digamma_t<double>(g) - psisum;
        topic += (al - g) * el + (lgamma(g) - lgamma(al));
        asum += al;
      }
    }
    topic = wave_sum(topic);
    asum = wave_sum(asum);
    const double tok = wave_sum(b_tok), ct = wave_sum(c_tok);
    if (lane == 0) {
      s_bd[wave][0] = topic;
      s_bd[wave][1] = asum;
    }
    if constexpr (W > 1) __syncthreads();
    if (wave == 0 && lane == 0) {
      double tp = 0.0, as = 0.0;
      for (int w = 0; w < W; ++w) {
        tp += s_bd[w][0];
        as += s_bd[w][1];
      }
      const double elog_max = (double)cs - psisum;  // log of the scale eθ carried (≈ 0)
      a.bound[mem] = tok + ct * elog_max + tp + (lgamma(as) - lgamma((double)gsum));
    }
  }
  STAMP(9);  // outputs
  STAMP_FLUSH
}

template <class S>
void launch_shape(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  const dim3 grid((unsigned)a.n);
  const int threads = 64 * S::W;
  if (stats) k_estep_split<S, true, false><<<grid, threads, 0, s>>>(a);
  else if (bound) k_estep_split<S, false, true><<<grid, threads, 0, s>>>(a);
  else k_estep_split<S, false, false><<<grid, threads, 0, s>>>(a);
  KERNEL_CHECK();
}

int shape_override() {
  static const int v = [] {
    const char* e = getenv("STC_WAVE_SHAPE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

bool use_grid() {
  static const bool v = [] {
    const char* e = getenv("STC_WAVE_KERNEL");
    return !(e && std::strcmp(e, "split") == 0);
  }();
  return v;
}

}  // namespace

int wave_kmax(int k) {
  if (k <= 64) return 64;
  if (k <= 104) return 104;
  if (k <= 128) return 128;
  return 0;
}

int wave_row_cap(int k) {
  if (use_grid()) return grid_row_cap(k);
  switch (wave_kmax(k)) {
    case 64: return 64 * Shape64::ROWS;
    case 104:
      switch (shape_override()) {
        case 1: return 64 * Shape104b::ROWS;
        case 2: return 64 * Shape104c::ROWS;
        case 3: return 64 * Shape104d::ROWS;
        default: return 64 * Shape104::ROWS;
      }
    case 128: return 64 * Shape128::ROWS;
    default: return 0;
  }
}

void launch_estep_wave(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  if (a.n == 0) return;
  if (use_grid()) return launch_estep_grid(s, a, stats, bound);
  switch (wave_kmax(a.k)) {
    case 64: launch_shape<Shape64>(s, a, stats, bound); break;
    case 104:
      switch (shape_override()) {
        case 1: launch_shape<Shape104b>(s, a, stats, bound); break;
        case 2: launch_shape<Shape104c>(s, a, stats, bound); break;
        case 3: launch_shape<Shape104d>(s, a, stats, bound); break;
        default: launch_shape<Shape104>(s, a, stats, bound); break;
      }
      break;
    case 128: launch_shape<Shape128>(s, a, stats, bound); break;
    default: throw Error(STC_ERR_INVALID_ARG, "wave E-step: k > 128");
  }
}

}  // namespace lda
}  // namespace stc

STC_STAMP_READER(stc_debug_stamps)
