// lda_wave.hip — K6 fast path: one 64-lane wavefront per document, the document block in VGPRs.
//
// Same fixed point as k_estep / [U] OnlineLDAOptimizer.variationalTopicInference (see lda.hip for
// the row-scaled numerics), specialised for fp32, k <= 128 and nnz <= 64·ROWS:
//   lane l holds rows n = l, l+64, … (ROWS of them) of B = expElogβ'[ids, :] — KMAX floats each,
//   so φ_n = B_n·eθ' is lane-local (eθ' broadcast from 512 B of LDS with ds_read_b128);
//   s = Bᵀr is a reduce-scatter across the 64 lanes: v_permlane32_swap / v_permlane16_swap halve
//   the topic set twice, then four DPP steps (row_mirror, row_half_mirror, two quad_perms) — every
//   lane ends owning ⌈KMAX/64⌉ topics, where γ, ψ(γ) and exp run with all 64 lanes busy.
// No workgroup barrier anywhere: the wave is the unit (LDS ops of one wave retire in order).
// Per inner iteration and lane: ROWS·KMAX FMAs for φ, ROWS·KMAX for Bᵀr, ~230 permute/add/select.
#include "lda_kernels.h"

namespace stc {
namespace lda {

namespace {

constexpr double kLogEps = -230.25850929940458;  // ln(1e-100): Spark's φ epsilon (see lda.hip)

template <int KMAX>
struct WaveShape;
template <>
struct WaveShape<64> {
  static constexpr int ROWS = 4;
};
template <>
struct WaveShape<100> {
  static constexpr int ROWS = 3;
};
template <>
struct WaveShape<128> {
  static constexpr int ROWS = 2;
};

constexpr int hup(int n) { return (n + 1) / 2; }

__device__ __forceinline__ unsigned fb(float x) { return __builtin_bit_cast(unsigned, x); }
__device__ __forceinline__ float bf(unsigned x) { return __builtin_bit_cast(float, x); }

// reduce-scatter step across lane distance 32 (or 16): lanes with the role bit clear keep topic
// set X, the others keep Y; after the swap x + y is the pair's total of the kept topic.
__device__ __forceinline__ float rs_swap32(float x, float y) { return swap32_pair(x, true, y); }
__device__ __forceinline__ float rs_swap16(float x, float y) { return swap16_pair(x, true, y); }
// reduce-scatter step through a DPP involution (row_mirror / row_half_mirror / quad_perm)
template <int CTRL>
__device__ __forceinline__ float rs_dpp(float x, float y, bool hi) {
  const float keep = hi ? y : x;
  const float send = hi ? x : y;
  return keep + bf((unsigned)__builtin_amdgcn_update_dpp(0, (int)fb(send), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_QP_3210 = 0x1B, DPP_QP_1032 = 0xB1;

template <int KMAX, bool STATS, bool BOUND>
__global__ __launch_bounds__(64) void k_estep_wave(EStepArgs<float> a) {
  constexpr int ROWS = WaveShape<KMAX>::ROWS;
  constexpr int C4 = KMAX / 4;
  constexpr int N1 = hup(KMAX), N2 = hup(N1), N3 = hup(N2), N4 = hup(N3), N5 = hup(N4), N6 = hup(N5);
  static_assert(KMAX % 4 == 0 && N6 >= 1, "shape");
  __shared__ __attribute__((aligned(16))) float s_eth[KMAX];

  if ((int64_t)blockIdx.x >= a.n) return;
  const int lane = threadIdx.x;
  const int64_t slot = a.slot0 + blockIdx.x;
  const int64_t mem = a.orig ? (int64_t)a.orig[slot] : slot;
  const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
  const int64_t s0 = a.indptr[row];
  const int nnz = (int)(a.indptr[row + 1] - s0);
  const int64_t e0 = a.bptr ? a.bptr[slot] : s0;
  const int k = a.k, kp = a.kp;

  // topics owned by this lane after the reduce-scatter: slot s ↦ t[s]; a slot is owned only if
  // its relative index stays inside every level's (odd-sized sets are padded by one zero)
  int tt[N6];
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
    v &= r < KMAX;
    tt[s] = r;
    own[s] = v;
  }

  // ---- load the document: ids, counts, ε-log-scales and the B rows (zero-padded)
  float B[ROWS][KMAX];
  float cts[ROWS], lse[ROWS], rr[ROWS];
  int ids[ROWS];
  bool any = false;
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    const int n = j * 64 + lane;
    const bool v = n < nnz;
    ids[j] = v ? a.indices[s0 + n] : 0;
    cts[j] = v ? a.values[s0 + n] : 0.f;
    lse[j] = v ? (float)(kLogEps - a.logscale[ids[j]]) : 0.f;
    any |= (cts[j] != 0.f);
    const float4* src = reinterpret_cast<const float4*>(a.Bp + (int64_t)ids[j] * kp);
#pragma unroll
    for (int c = 0; c < C4; ++c) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (v && 4 * c < kp) x = src[c];
      B[j][4 * c + 0] = x.x;
      B[j][4 * c + 1] = x.y;
      B[j][4 * c + 2] = x.z;
      B[j][4 * c + 3] = x.w;
    }
  }
  const bool nonempty = __any(any);
  if (!nonempty) {
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      const int t = tt[s];
      if (own[s] && t < k) {
        if (a.gamma) a.gamma[mem * k + t] = 0.f;
        if (STATS) a.elogth[slot * k + t] = 0.f;
      }
      if (STATS && own[s] && t < kp) a.eth[slot * kp + t] = 0.f;
    }
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
    return;
  }

  // ---- γ₀ for the owned topics, eθ' = exp(ψ(γ) − ψ(max γ))
  uint64_t stream = 0;
  if (!a.gamma0) {
    const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, mem) : (uint64_t)(a.doc_id_base + row);
    stream = doc_stream(a.seed, key);
  }
  float gam[N6], eth[N6], alp[N6];
  float gsum = 0.f, gmax = 0.f;
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    const int t = tt[s];
    const bool v = own[s] && t < k;
    gam[s] = v ? (a.gamma0 ? a.gamma0[mem * k + t] : (float)gamma_sample(stream, t, a.gamma_shape)) : 0.f;
    alp[s] = v ? (float)a.alpha[t] : 0.f;
    gsum += gam[s];
    gmax = fmaxf(gmax, gam[s]);
  }
  gsum = wave_sum_dpp(gsum);
  gmax = wave_max_dpp(gmax);
  float psimax = digamma_fast(gmax);
  float lmax = psimax - digamma_fast(gsum);
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    const int t = tt[s];
    eth[s] = (own[s] && t < k) ? __expf(digamma_fast(gam[s]) - psimax) : 0.f;
    if (own[s]) s_eth[t] = eth[s];
  }
  __builtin_amdgcn_wave_barrier();

  int it = 0;
  bool done = false;
  double b_tok = 0.0, c_tok = 0.0;
  float dot[ROWS];
  while (true) {
    // Phase A: φ_n = B_n·eθ' + ε'_n ; r_n = cts_n / φ_n   (lane-local)
#pragma unroll
    for (int j = 0; j < ROWS; ++j) dot[j] = 0.f;
#pragma unroll
    for (int c = 0; c < C4; ++c) {
      const float4 e = *reinterpret_cast<const float4*>(s_eth + 4 * c);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {  // rows past nnz are zero: no per-row branches
        dot[j] = fmaf(B[j][4 * c + 0], e.x, dot[j]);
        dot[j] = fmaf(B[j][4 * c + 1], e.y, dot[j]);
        dot[j] = fmaf(B[j][4 * c + 2], e.z, dot[j]);
        dot[j] = fmaf(B[j][4 * c + 3], e.w, dot[j]);
      }
    }
    const bool last = done || it >= a.max_iter;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const float phi = dot[j] + fmaxf(__expf(lse[j] - lmax), 1.17549435e-38f);
      rr[j] = __fdividef(cts[j], phi);
      if (BOUND && last && cts[j] != 0.f) {
        b_tok += (double)cts[j] * ((double)logf(fmaxf(dot[j], 1.17549435e-38f)) + a.logscale[ids[j]]);
        c_tok += (double)cts[j];
      }
    }
    if (last) break;

    // Phase B: s = Bᵀ r, reduce-scattered so lane owns s[off .. off+N6)
    float p1[N1];
#pragma unroll
    for (int q = 0; q < N1; ++q) {
      float x = 0.f, y = 0.f;
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        x = fmaf(B[j][q], rr[j], x);
        if (N1 + q < KMAX) y = fmaf(B[j][N1 + q], rr[j], y);
      }
      p1[q] = rs_swap32(x, y);
    }
    float p2[N2];
#pragma unroll
    for (int q = 0; q < N2; ++q) p2[q] = rs_swap16(p1[q], (N2 + q < N1) ? p1[N2 + q] : 0.f);
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

    // Phase C: γ ← eθ' ⊙ s + α on the owned topics; Σ|Δγ|, Σγ, max γ over the wave
    float dsum = 0.f;
    gsum = 0.f;
    gmax = 0.f;
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      if (own[s] && tt[s] < k) {
        const float g = fmaf(eth[s], p6[s], alp[s]);
        dsum += fabsf(g - gam[s]);
        gam[s] = g;
        gsum += g;
        gmax = fmaxf(gmax, g);
      }
    }
    dsum = wave_sum_dpp(dsum);
    gsum = wave_sum_dpp(gsum);
    gmax = wave_max_dpp(gmax);
    // Phase D: eθ' = exp(ψ(γ) − ψ(max γ)), broadcast through LDS
    psimax = digamma_fast(gmax);
    lmax = psimax - digamma_fast(gsum);
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      const int t = tt[s];
      eth[s] = (own[s] && t < k) ? __expf(digamma_fast(gam[s]) - psimax) : 0.f;
      if (own[s]) s_eth[t] = eth[s];
    }
    __builtin_amdgcn_wave_barrier();
    ++it;
    done = dsum <= 1e-3f * (float)k;
  }

  // ---- outputs
  const double psisum = digamma_t<double>((double)gsum);
#pragma unroll
  for (int s = 0; s < N6; ++s) {
    const int t = tt[s];
    if (own[s] && t < k) {
      if (a.gamma) a.gamma[mem * k + t] = gam[s];
      if (STATS) a.elogth[slot * k + t] = (float)(digamma_t<double>((double)gam[s]) - psisum);
    }
  }
  if (STATS)  // from the LDS copy φ was computed with (pads are zero)
    for (int t = lane; t < kp; t += 64) a.eth[slot * kp + t] = s_eth[t];
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
  if (BOUND) {
    const double elog_max = digamma_t<double>((double)gmax) - psisum;
    double topic = 0.0, asum = 0.0;
#pragma unroll
    for (int s = 0; s < N6; ++s) {
      const int t = tt[s];
      if (own[s] && t < k) {
        const double g = (double)gam[s], al = a.alpha[t];
        const double el = digamma_t<double>(g) - psisum;
        topic += (al - g) * el + (lgamma(g) - lgamma(al));
        asum += al;
      }
    }
    double tot = b_tok + c_tok * elog_max + topic;
    tot = wave_sum(tot);
    asum = wave_sum(asum);
    if (lane == 0) a.bound[mem] = tot + (lgamma(asum) - lgamma((double)gsum));
  }
}

template <int KMAX>
void launch_kmax(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  const dim3 grid((unsigned)a.n);
  if (stats) k_estep_wave<KMAX, true, false><<<grid, 64, 0, s>>>(a);
  else if (bound) k_estep_wave<KMAX, false, true><<<grid, 64, 0, s>>>(a);
  else k_estep_wave<KMAX, false, false><<<grid, 64, 0, s>>>(a);
  KERNEL_CHECK();
}

}  // namespace

int wave_kmax(int k) {
  if (k <= 64) return 64;
  if (k <= 100) return 100;
  if (k <= 128) return 128;
  return 0;
}

int wave_row_cap(int k) {
  switch (wave_kmax(k)) {
    case 64: return 64 * WaveShape<64>::ROWS;
    case 100: return 64 * WaveShape<100>::ROWS;
    case 128: return 64 * WaveShape<128>::ROWS;
    default: return 0;
  }
}

void launch_estep_wave(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound) {
  if (a.n == 0) return;
  switch (wave_kmax(a.k)) {
    case 64: launch_kmax<64>(s, a, stats, bound); break;
    case 100: launch_kmax<100>(s, a, stats, bound); break;
    case 128: launch_kmax<128>(s, a, stats, bound); break;
    default: throw Error(STC_ERR_INVALID_ARG, "wave E-step: k > 128");
  }
}

}  // namespace lda
}  // namespace stc
