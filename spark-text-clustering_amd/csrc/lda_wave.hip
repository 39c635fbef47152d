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
//   Σ|Δγ|, Σγ and max γ meet in LDS behind a second barrier: eθ' must share one scale across waves.
// Per inner iteration and lane: 2·ROWS·KW FMAs, ~120 permute/add/select, two barriers (W > 1).
#include "lda_kernels.h"

namespace stc {
namespace lda {

namespace {

constexpr double kLogEps = -230.25850929940458;  // ln(1e-100): Spark's φ epsilon (see lda.hip)
constexpr float kTiny = 1.17549435e-38f;         // FLT_MIN

template <int KMAX>
struct SplitShape;  // serves k <= KMAX
template <>
struct SplitShape<64> {
  static constexpr int W = 2, KW = 32, ROWS = 4;
};
template <>
struct SplitShape<104> {  // k = 100: slices [0,52) and [52,100) — 16-byte aligned row offsets
  static constexpr int W = 2, KW = 52, ROWS = 3;
};
template <>
struct SplitShape<128> {
  static constexpr int W = 4, KW = 32, ROWS = 3;
};

constexpr int hup(int n) { return (n + 1) / 2; }
template <int KW>
constexpr int lvl(int L) {
  int n = KW;
  for (int i = 0; i < L; ++i) n = hup(n);
  return n;
}

// reduce-scatter step through a DPP involution (row_mirror / row_half_mirror / quad_perm): lanes
// with the role bit clear keep topic set X, the others Y; the partner sends the set it drops.
template <int CTRL>
__device__ __forceinline__ float rs_dpp(float x, float y, bool hi) {
  const float keep = hi ? y : x;
  const float send = hi ? x : y;
  return keep + dpp_f<CTRL>(send);
}
constexpr int DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_QP_3210 = 0x1B, DPP_QP_1032 = 0xB1;

template <int KMAX, bool STATS, bool BOUND>
__global__ __launch_bounds__(64 * SplitShape<KMAX>::W, 2) void k_estep_split(EStepArgs<float> a) {
  constexpr int W = SplitShape<KMAX>::W, KW = SplitShape<KMAX>::KW, ROWS = SplitShape<KMAX>::ROWS;
  constexpr int C4 = KW / 4;
  constexpr int N1 = lvl<KW>(1), N2 = lvl<KW>(2), N3 = lvl<KW>(3), N4 = lvl<KW>(4), N5 = lvl<KW>(5),
                N6 = lvl<KW>(6);
  static_assert(KW % 4 == 0 && N6 >= 1, "shape");
  // one buffer each suffices: the φ barrier and the reduction barrier alternate, so a wave can
  // only overwrite a buffer after every wave has passed the other barrier (and read it).
  __shared__ __attribute__((aligned(16))) float s_eth[W][KW];
  __shared__ float s_phi[W][ROWS][64];
  __shared__ float s_red[W][3];
  __shared__ double s_bd[W][2];

  if ((int64_t)blockIdx.x >= a.n) return;
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
  float B[ROWS][KW];
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
      B[j][4 * c + 0] = x.x;
      B[j][4 * c + 1] = x.y;
      B[j][4 * c + 2] = x.z;
      B[j][4 * c + 3] = x.w;
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
            a.vals[e0 + n] = (uint32_t)(e0 + n);
            a.edoc[e0 + n] = (int32_t)slot;
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

  // (Σ, Σ, max) over the whole document: wave all-reduce, then the W waves through LDS in a fixed
  // order, so every wave gets bit-identical totals (and therefore the same stopping decision)
  auto block_reduce = [&](float& x, float& y, float& m) {
    x = wave_sum_dpp(x);
    y = wave_sum_dpp(y);
    m = wave_max_dpp(m);
    if constexpr (W > 1) {
      if (lane == 0) {
        s_red[wave][0] = x;
        s_red[wave][1] = y;
        s_red[wave][2] = m;
      }
      __syncthreads();
      x = s_red[0][0];
      y = s_red[0][1];
      m = s_red[0][2];
#pragma unroll
      for (int w = 1; w < W; ++w) {
        x += s_red[w][0];
        y += s_red[w][1];
        m = fmaxf(m, s_red[w][2]);
      }
    }
  };

  // ---- γ₀ for the owned topics, eθ' = exp(ψ(γ) − ψ(max γ))
  uint64_t stream = 0;
  if (!a.gamma0) {
    const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem) : (uint64_t)(a.doc_id_base + row);
    stream = doc_stream(a.seed, key);
  }
  float gam[N6], eth[N6], alp[N6];
  float gsum = 0.f, gmax = 0.f, dsum = 0.f;
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    const int t = t0 + tl[s];
    gam[s] = own[s] ? (a.gamma0 ? a.gamma0[mem * k + t] : (float)gamma_sample(stream, t, a.gamma_shape)) : 0.f;
    alp[s] = own[s] ? (float)a.alpha[t] : 0.f;
    gsum += gam[s];
    gmax = fmaxf(gmax, gam[s]);
  }
  for (int t = lane; t < KW; t += 64) my_eth[t] = 0.f;  // slice padding (t0 + t >= k) stays zero
  block_reduce(gsum, dsum, gmax);
  float psimax = digamma_fast(gmax);
  float lmax = psimax - digamma_fast(gsum);
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    eth[s] = own[s] ? __expf(digamma_fast(gam[s]) - psimax) : 0.f;
    if (own[s]) my_eth[tl[s]] = eth[s];
  }
  __builtin_amdgcn_wave_barrier();  // the slice is read back only by this wave

  int it = 0;
  bool done = false;
  double b_tok = 0.0, c_tok = 0.0;
  while (true) {
    // Phase A: φ_n = B_n·eθ' + ε'_n ; r_n = cts_n / φ_n
    float dot[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) dot[j] = 0.f;
#pragma unroll
    for (int c = 0; c < C4; ++c) {
      const float4 e = *reinterpret_cast<const float4*>(my_eth + 4 * c);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {  // rows past nnz are zero: no per-row branches
        dot[j] = fmaf(B[j][4 * c + 0], e.x, dot[j]);
        dot[j] = fmaf(B[j][4 * c + 1], e.y, dot[j]);
        dot[j] = fmaf(B[j][4 * c + 2], e.z, dot[j]);
        dot[j] = fmaf(B[j][4 * c + 3], e.w, dot[j]);
      }
    }
    if constexpr (W > 1) {
#pragma unroll
      for (int j = 0; j < ROWS; ++j) s_phi[wave][j][lane] = dot[j];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        float d = s_phi[0][j][lane];
#pragma unroll
        for (int w = 1; w < W; ++w) d += s_phi[w][j][lane];
        dot[j] = d;
      }
    }
    const bool last = done || it >= a.max_iter;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const float phi = dot[j] + fmaxf(__expf(lse[j] - lmax), kTiny);
      rr[j] = cts[j] * __builtin_amdgcn_rcpf(phi);
      if (BOUND && last && cts[j] != 0.f) {
        b_tok += (double)cts[j] * ((double)__logf(fmaxf(dot[j], kTiny)) + a.logscale[ids[j]]);
        c_tok += (double)cts[j];
      }
    }
    if (last) break;

    // Phase B: s = Bᵀ r over the slice, reduce-scattered so the lane owns p6[0 .. N6)
    float p1[N1];
#pragma unroll
    for (int q = 0; q < N1; ++q) {
      float x = 0.f, y = 0.f;
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        x = fmaf(B[j][q], rr[j], x);
        if (N1 + q < KW) y = fmaf(B[j][N1 + q], rr[j], y);
      }
      p1[q] = swap32_pair(x, true, y);
    }
    float p2[N2];
#pragma unroll
    for (int q = 0; q < N2; ++q) p2[q] = swap16_pair(p1[q], true, (N2 + q < N1) ? p1[N2 + q] : 0.f);
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

    // Phase C: γ ← eθ' ⊙ s + α on the owned topics; Σ|Δγ|, Σγ, max γ over the document
    dsum = 0.f;
    gsum = 0.f;
    gmax = 0.f;
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      if (own[s]) {
        const float g = fmaf(eth[s], p6[s], alp[s]);
        dsum += fabsf(g - gam[s]);
        gam[s] = g;
        gsum += g;
        gmax = fmaxf(gmax, g);
      }
    }
    block_reduce(dsum, gsum, gmax);
    // Phase D: eθ' = exp(ψ(γ) − ψ(max γ)) into the wave's LDS slice
    psimax = digamma_fast(gmax);
    lmax = psimax - digamma_fast(gsum);
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      if (own[s]) {
        eth[s] = __expf(digamma_fast(gam[s]) - psimax);
        my_eth[tl[s]] = eth[s];
      }
    }
    __builtin_amdgcn_wave_barrier();
    ++it;
    done = dsum <= 1e-3f * (float)k;
  }

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
          a.vals[e0 + n] = (uint32_t)(e0 + n);
          a.edoc[e0 + n] = (int32_t)slot;
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
      const double elog_max = digamma_t<double>((double)gmax) - psisum;
      a.bound[mem] = tok + ct * elog_max + tp + (lgamma(as) - lgamma((double)gsum));
    }
  }
}

template <int KMAX>
void launch_kmax(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  const dim3 grid((unsigned)a.n);
  const int threads = 64 * SplitShape<KMAX>::W;
  if (stats) k_estep_split<KMAX, true, false><<<grid, threads, 0, s>>>(a);
  else if (bound) k_estep_split<KMAX, false, true><<<grid, threads, 0, s>>>(a);
  else k_estep_split<KMAX, false, false><<<grid, threads, 0, s>>>(a);
  KERNEL_CHECK();
}

}  // namespace

int wave_kmax(int k) {
  if (k <= 64) return 64;
  if (k <= 104) return 104;
  if (k <= 128) return 128;
  return 0;
}

int wave_row_cap(int k) {
  switch (wave_kmax(k)) {
    case 64: return 64 * SplitShape<64>::ROWS;
    case 104: return 64 * SplitShape<104>::ROWS;
    case 128: return 64 * SplitShape<128>::ROWS;
    default: return 0;
  }
}

void launch_estep_wave(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  if (a.n == 0) return;
  switch (wave_kmax(a.k)) {
    case 64: launch_kmax<64>(s, a, stats, bound); break;
    case 104: launch_kmax<104>(s, a, stats, bound); break;
    case 128: launch_kmax<128>(s, a, stats, bound); break;
    default: throw Error(STC_ERR_INVALID_ARG, "wave E-step: k > 128");
  }
}

}  // namespace lda
}  // namespace stc
