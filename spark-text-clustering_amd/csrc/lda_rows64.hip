// lda_rows64.hip — K6 at Spark's precision: the ROWS-split fp64 E-step for k ≤ 104
// ([U] OnlineLDAOptimizer.variationalTopicInference in Breeze Double, called per document inside
// submitMiniBatch behind lda.run, TextClustering/src/main/scala/LDAClustering.scala:61).
//
// One document per workgroup of four waves.  Wave w holds rows n = 32·j + 8·w + rl (row set j < R,
// R = ⌈nnz/32⌉ chosen per document) for EVERY topic; inside a wave lane = tl + 8·rl, and topic lane
// tl holds topics [KL·tl, KL·tl + KL) of its R rows: R·KL doubles (k ≤ 104: KL = 13, 26·R VGPRs for
// R ≤ 5, a sixth row set in LDS; documents with 7–8 row sets run in a second launch with all eight
// sets in VGPRs at one workgroup per CU).
//   φ_n = B_n·eθ : KL lane-local FMAs per row; the eight topic lanes' partials go to the wave's own
//     LDS rows and worker lane q (one per wave row) adds them in a fixed order, forms r_q = cts/φ
//     once and publishes it to the wave.  The exchange never leaves the wave: no block barrier.
//   s = Bᵀr : R lane-local FMAs per topic, KL partials per lane to LDS, ONE block barrier; then the
//     ψ waves of this iteration read a topic's 32 partials per lane, update γ and compute
//     eθ = exp(ψ(γ) − ψ(Σγ')) for ⌈kp/2⌉ topics each (k > 64: two ψ waves, alternating between
//     waves {0,1} and {2,3} by iteration parity so every SIMD carries the transcendental chain every
//     other iteration; k ≤ 64: one, rotating over the four waves), publish eθ and γ, second barrier.
//   ψ(Σγ') from Σγ' = Σα + Σ_n cts_n − Σ_n r_n·ε'_n (exact in real arithmetic): a per-document
//     constant unless some row's ε' is visible at fp64 resolution (ε' ≥ 2^-53·φ).
//   Spark's stop rule Σ|Δγ|/k ≤ 1e-3 is one comparison against EStepArgs::stop_thr; the ψ waves'
//     Σ|Δγ| partials ride the second barrier.
// Against the round-2 topic split (lda_grid64.hip, since removed: each wave a 26-topic slice, the s
// reduction a 32-lane DPP / permlane reduce-scatter of 13 values in every wave, ψ/exp in all four
// waves) this removes ≈ 75
// cross-lane and ≈ 200 transcendental VALU instructions per document-iteration and the scratch
// reload the old loop carried; the cost is LDS traffic (13 8-byte stores per lane and iteration),
// which the LDS array absorbs beside the VALU (MI355X_MICROARCH.md §LDS).
// Numerics as lda.hip: Bp row-scaled by e^{-m_v}, Spark's 1e-100 carried as ε'_n = 1e-100·e^{-m_v}.
#include "estep_common.h"
#include "psi64.h"

#ifndef R64_LOAD_BATCH
#define R64_LOAD_BATCH 3  // row sets whose B loads are in flight together in the load phase (r03: 2 → 3, −2 %)
#endif
#ifndef R64_PRIO
#define R64_PRIO 2  // wave priority raised over the latency-critical phases (1: ψ; 2: ψ + r): −2 % E-step (r03)
#endif
#ifndef R64_RCP_NR
#define R64_RCP_NR 2  // Newton steps after v_rcp_f64 in that chain
#endif
#ifndef R64_MIRROR
#define R64_MIRROR 1  // 1 (k > 64): the idle wave of the ψ wave's topic set computes Σ|Δγ| off the ψ chain.
                      // r04 measured it +1.3 % (31.96 vs 31.54 ms, off then); after the in-wave s
                      // reduce-scatter and the resident grid it is −4 %: headline E-step 27.05 → 25.97 ms
#endif
#ifndef R64_LONG_OCC
#define R64_LONG_OCC 1  // long-document kernel workgroups per CU the register budget is cut for
#endif

namespace stc {
namespace lda {

namespace {

constexpr int kW = 4;          // waves per document
constexpr int kSbPitch = 4;   // s-partial row pitch (doubles): one sum per wave (rs_rows8), 16-B reads
constexpr int kPaPitch = 10;   // φ-partial row pitch (doubles): conflict-free 16-B worker reads
constexpr int kOnChipSets = 6; // row sets the common kernel holds (5 in VGPRs + 1 in LDS)
constexpr int kMaxSets = 8;    // one worker lane per wave row: 8 row lanes × 8 sets = 64 lanes

template <int KL_, int RREG_, int RMAX_>
struct RShape {
  static constexpr int KL = KL_;             // topics per topic lane (8 topic lanes: k ≤ 8·KL)
  static constexpr int KLP = (KL_ + 1) / 2 * 2;
  static constexpr int KT = 8 * KL_;
  static constexpr int RREG = RREG_;         // row sets in VGPRs
  static constexpr int RMAX = RMAX_;         // row sets handled (≤ kMaxSets)
  static constexpr int NOVF = RMAX_ > RREG_ ? RMAX_ - RREG_ : 0;  // row sets in LDS
};
template <int KL>
using RCommon = RShape<KL, 5, kOnChipSets>;
template <int KL>
using RLong = RShape<KL, kMaxSets, kMaxSets>;

template <class S>
struct RLds {
  double eth[8][S::KLP] __attribute__((aligned(16)));  // eθ, topic t at [t / KL][t % KL]
  double gam[S::KT];               // γ
  double rrow[kW][8 * S::RMAX];    // r = cts/φ per (wave, wave row)
  int rid[kW][8 * S::RMAX];        // term id per (wave, wave row): the coalesced entry outputs
  double dsum[2];                  // Σ|Δγ| of the last update per ψ wave
  double esum[kW] __attribute__((aligned(16)));  // Σ r·ε' over a wave's rows (0 unless an ε' is visible)
  double part[kW][4];              // per-wave partial sums (init: Σγ₀, Σα, Σcts; end: Σγ, bound terms)
  double cs;                       // ψ(Σγ') of the current eθ (the bound's scale)
  double apc[S::KT][2] __attribute__((aligned(16)));  // α_t, ψc_t of the ψ lanes' topics (not in VGPRs)
  double ac[4] __attribute__((aligned(16)));  // Σα, Σcts, ψ(Σα + Σcts) (the flat ψ(Σγ'))
  PsiK psik;                       // the exp() constants of the ψ chain (psi_expk_load)
  union {
    struct {
      double pa[kW][8 * S::RMAX][kPaPitch];  // φ partials (wave, wave row, topic lane)
      double sb[S::KT][kSbPitch];            // s partials (topic, row lane 8·w + rl)
    } l;
    double stage[kW][8][S::KT + 2];          // load phase: eight B rows per wave at a time
  } u __attribute__((aligned(16)));
  double ovf[S::NOVF > 0 ? S::NOVF * kW * S::KL * 64 : 1];  // row sets past RREG ([set][w][p][lane])
};

// Per-lane document context: set up once per document by rows64_open, outside the row-set
// specialisation, and read by the R-specialised loop (rows64_iterate) and by rows64_close.  Only the
// block loads and the loop are instantiated per R: the prologue (γ₀ from the counter RNG — fp64 log,
// sqrt, cos — and the first eθ) and the epilogue (digamma / lgamma of the outputs) exist once per
// kernel.  Per R they made the common kernel 170 KB of code, past the 64 KB instruction cache a CU
// pair shares, and documents that iterate a dozen times (the planted state) paid instruction-fetch
// misses for the whole prologue of every document.
struct RDoc {
  int64_t slot, row, mem, s0, e0;
  int nnz, rsets;
  int tid;                           // the resident long kernel's threadIdx.x, laundered per document
  int lane, w, tl, rl;
  int npsi, half, pw, tt, ttl, ttp;  // ψ-lane topic map
  bool tval, town;                   // γ / eθ slot (the fp64 pad column included); a real topic
  bool wv;                           // worker lane with a document row
  int qid;                           // worker: term id, count, m_v, 2^53·ε'
  double qc, qls, qe2;
#ifdef STC_STAMP
  unsigned long long st0;            // kernel entry (diagnostic build: the per-document prologue)
#endif
};

// threadIdx.x, or its per-document laundered copy in the resident long-document kernel (RES)
template <bool RES>
__device__ __forceinline__ int rows64_tid(const RDoc& d) { return RES ? d.tid : (int)threadIdx.x; }

// worker lanes, γ₀, α / ψc, Σγ₀ / Σα / Σcts, the first eθ; false (outputs written) for a document
// without a nonzero count
template <class S, bool STATS, bool BOUND, bool RES>
__device__ __forceinline__ bool rows64_open(const EStepArgs<double>& a, RLds<S>& sm, RDoc& d) {
  const int tid = rows64_tid<RES>(d);
  constexpr int KL = S::KL, KLP = S::KLP;
  const int k = a.k, kp = a.kp;
  // the wave index is wave-uniform: held in an SGPR, every per-wave role test (ψ wave, worker sets) is
  // scalar instead of a v_cmp / v_cndmask chain per iteration
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  d.lane = lane;
  d.w = w;
  d.tl = lane & 7;
  d.rl = lane >> 3;
  // ψ-lane topic map: k > 64 two ψ waves of `half` topics (t = (w & 1)·half + lane), else one
  d.npsi = kp > 64 ? 2 : 1;
  d.half = d.npsi == 2 ? (kp + 1) / 2 : kp;
  d.pw = d.npsi == 2 ? (w & 1) : 0;
  d.tt = d.pw * d.half + lane;
  d.tval = lane < d.half && d.tt < kp;
  d.town = lane < d.half && d.tt < k;
  d.ttl = d.tt / KL;
  d.ttp = d.tt - d.ttl * KL;
  const int npsi = d.npsi, tt = d.tt;

  // ---- worker lane: wave row q = lane (set q >> 3, row lane q & 7) → document row qn
  const int qn = 32 * (lane >> 3) + 8 * w + (lane & 7);
  d.wv = lane < 8 * d.rsets && qn < d.nnz;
  const int64_t qe = d.wv ? d.s0 + qn : 0;
  d.qid = d.wv ? a.indices[qe] : 0;
  d.qc = d.wv ? a.values[qe] : 0.0;
  // (m_v = logscale[id] and ε' are loaded in rows64_iterate beside the block's B rows: a third dependent
  // round trip here would sit on the prologue's chain)

  // ---- γ₀ / α partials (the first npsi waves hold the topics), Σcts, eθ pads, α and ψc to LDS
  double g0 = 0.0;
  const double alp = d.town ? a.alpha[tt] : 0.0;
  const double pc = d.town ? a.psic[tt] : 0.0;  // ψ(Σ_v λ_vt): expElogβ's per-topic factor, carried by eθ
  if (w < npsi) {
    if (d.tval) {
      sm.apc[tt][0] = alp;
      sm.apc[tt][1] = pc;
    }
    if (d.town) {
      if (a.gamma0) {
        g0 = a.gamma0[d.mem * k + tt];
      } else {
        const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, d.mem) : (uint64_t)(a.doc_id_base + d.row);
#ifdef R64_DIAG_NORNG  // diagnostic build only (tools/iter_sweep.py): the prologue without γ₀'s RNG
        g0 = 1.0 + 1e-3 * (double)(key & 1023) + 1e-4 * tt;
#else
        g0 = gamma_sample(doc_stream(a.seed, key), tt, a.gamma_shape);
#endif
      }
    }
    if (d.tval) sm.gam[tt] = g0;
  }
  for (int i = tid; i < 8 * KLP; i += 64 * kW) (&sm.eth[0][0])[i] = 0.0;
  psik_fill(sm.psik, tid, 64 * kW);  // (published by the barrier below)
  {
    const double gs = wave_sum_d(g0), as = wave_sum_d(alp), cts = wave_sum_d(d.qc);
    if (lane == 0) {
      sm.part[w][0] = w < npsi ? gs : 0.0;
      sm.part[w][1] = w < npsi ? as : 0.0;
      sm.part[w][2] = cts;
    }
  }
  const bool nonempty = __syncthreads_or(d.wv && d.qc != 0.0) != 0;  // (also publishes γ₀ and the partials)
  const double gsum0 = (sm.part[0][0] + sm.part[1][0]) + (sm.part[2][0] + sm.part[3][0]);
  if (tid == 0) {  // read back by the ψ phase and the bound (published by the next barrier)
    const double asum = (sm.part[0][1] + sm.part[1][1]) + (sm.part[2][1] + sm.part[3][1]);
    const double ctot = (sm.part[0][2] + sm.part[1][2]) + (sm.part[2][2] + sm.part[3][2]);
    sm.ac[0] = asum;
    sm.ac[1] = ctot;
    // inside the loop ψ(Σγ') comes from the Σα + Σcts − Σ r·ε' identity, so without a visible ε' it is
    // one constant per document
    sm.ac[2] = digamma_fast_d(asum + ctot);
  }

  if (!nonempty) {
    if (w < npsi) {
      if (d.town) {
        if (a.gamma) a.gamma[d.mem * k + tt] = 0.0;
        if (STATS) a.elogth[d.slot * k + tt] = 0.0;
      }
      if (STATS && d.tval) a.eth[d.slot * kp + tt] = 0.0;
    }
    if (tid == 0) {
      if (a.iters) a.iters[d.mem] = 0;
      if (a.nonempty) a.nonempty[d.mem] = 0;
      if (BOUND) a.bound[d.mem] = 0.0;
    }
    return false;
  }
  // eθ' = exp(ψ(γ) − ψ(Σγ) − ψc_t): Spark's exp(E[log θ]) times expElogβ's per-topic factor
  {
    const double cs0 = digamma_fast_d(gsum0);
    if (w < npsi && d.town) sm.eth[d.ttl][d.ttp] = exp_digamma_minus_v2<R64_RCP_NR>(g0, cs0 + pc);
    if (tid == 0) sm.cs = cs0;
  }
  return true;  // (the block loads' barrier publishes eθ)
}

// the document block (R row sets) and the fixed point; returns the iteration count, the worker's φ
// (without ε') in qdt; the final r sits in sm.rrow
template <class S, int R>
__device__ __forceinline__ int rows64_iterate(const EStepArgs<double>& a, RLds<S>& sm, RDoc& d, double& qdt) {
  constexpr int KL = S::KL, KLP = S::KLP;
  constexpr int RG = R < S::RREG ? R : S::RREG;  // row sets in VGPRs; [RG, R) in sm.ovf
  static_assert(R >= 1 && R <= S::RMAX && R - RG <= S::NOVF, "row sets");
  STAMP_DECL
#ifdef STC_STAMP
  st_acc[10] += st_last - d.st0;
#endif
  const int lane = d.lane, w = d.w, tl = d.tl, rl = d.rl;
  const int k = a.k, kp = a.kp, nnz = d.nnz, npsi = d.npsi, pw = d.pw, tt = d.tt, ttl = d.ttl, ttp = d.ttp;
  const bool town = d.town;
  const int qid = d.qid;
  const double qc = d.qc;
  // the worker row's m_v, issued before the B gather so the two round trips overlap
  d.qls = a.logscale[qid];
  // mirror mode (k > 64): the waves w and w ^ 2 share a topic set and take turns as its ψ wave and as
  // its Σ|Δγ| wave; each keeps γ / eθ of its lane's topic as it last computed them (read once below)
  const bool mir = R64_MIRROR && npsi == 2;
  double gm = 0.0, em = 0.0;

  // ---- B rows, coalesced: per row set the wave copies its eight rows (kp doubles each) with
  // 16-byte loads, stages them in LDS and every lane picks up its (row lane, topic lane) part
  double B[RG][KL];
  double* const ovf = sm.ovf + (size_t)w * KL * 64 + lane;  // set RG + i at ovf[i·kW·KL·64 + 64·p]
#define BV(j, p) ((j) < RG ? B[(j) < RG ? (j) : 0][p] : ovf[((j) - RG) * kW * KL * 64 + 64 * (p)])
  {
    const int C2 = kp >> 1;                     // double2 pieces per row
    constexpr int NP = (8 * (S::KT / 2) + 63) / 64;  // pieces per lane per row set (upper bound)
    double* const stg = &sm.u.stage[w][0][0];
    constexpr int SP = S::KT + 2;
#pragma unroll
    for (int j0 = 0; j0 < R; j0 += R64_LOAD_BATCH) {
      double2 pc[R64_LOAD_BATCH][NP];
#pragma unroll
      for (int jj = 0; jj < R64_LOAD_BATCH; ++jj) {
        const int j = j0 + jj;
        if (j >= R) break;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int c = lane + 64 * i;
          const int srow = c / C2, q = c - srow * C2;
          const int id = __builtin_amdgcn_ds_bpermute((8 * j + (srow & 7)) << 2, qid);  // its worker lane
          const bool keep = c < 8 * C2 && 32 * j + 8 * w + srow < nnz;
#ifdef R64_DIAG_NOGATHER  // diagnostic build only: the load phase without the B gather
          const double2 x = make_double2(1e-3 * (id & 7), 1e-3 * (q & 7));
#else
          const double2 x = *reinterpret_cast<const double2*>(a.Bp + (int64_t)(keep ? id : 0) * kp + 2 * (keep ? q : 0));
#endif
          pc[jj][i] = keep ? x : make_double2(0.0, 0.0);
        }
      }
#pragma unroll
      for (int jj = 0; jj < R64_LOAD_BATCH; ++jj) {
        const int j = j0 + jj;
        if (j >= R) break;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int c = lane + 64 * i;
          const int srow = c / C2, q = c - srow * C2;
          if (c < 8 * C2) *reinterpret_cast<double2*>(stg + srow * SP + 2 * q) = pc[jj][i];
        }
        __builtin_amdgcn_wave_barrier();  // one wave writes and reads its stage; LDS is in order per wave
#pragma unroll
        for (int p = 0; p < KL; ++p) {
          const int t = KL * tl + p;
          const double v = t < k ? stg[rl * SP + t] : 0.0;
          if (j < RG) B[j < RG ? j : 0][p] = v;
          else ovf[(j - RG) * kW * KL * 64 + 64 * p] = v;  // read back only by this lane
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
  }

  // ε'_q = 1e-100·e^{-m_v} held as 2^53·ε' (the test 2^53·ε' ≥ φ is then direct), capped at 1e300
  // where e^{-m_v} overflows (Spark's unscaled row is 0 there; r ≈ cts·1e-284 reproduces that).
  // Padding rows hold −2^53 (φ = −1, r = −0, never live).
  const double qe2 = d.wv ? fmin(0x1p53 * exp(kLogEps - d.qls), 1e300) : -0x1p53;
  d.qe2 = qe2;
  __syncthreads();  // the staging area is the loop's partial arrays; (also publishes the first eθ)
  if (mir && town) {  // γ₀ / eθ₀ of the lane's topic (no ψ phase has overwritten them before barrier 1)
    gm = sm.gam[tt];
    em = sm.eth[ttl][ttp];
  }

  double* const pa = &sm.u.l.pa[w][0][0];
  double* const sb = &sm.u.l.sb[0][0];
  const PsiExpK expk = psi_expk_load(sm.psik);
  double rr[R];
  double qr = 0.0;  // worker: r of its row (φ without ε' in qdt)
  qdt = 0.0;
  double dsum = 0.0;
  int it = 0;
  STAMP(0);  // block loads and their barrier
  while (true) {
    // Phase A: φ partials over the lane's KL topics; worker lane q (one per wave row) adds the eight
    // topic lanes' partials in a fixed order, forms r_q = cts/φ once and publishes it (wave-local LDS)
    {
      double acc[R];
#pragma unroll
      for (int j = 0; j < R; ++j) acc[j] = 0.0;
#pragma unroll
      for (int c = 0; c < KLP / 2; ++c) {
        const double2 e = *reinterpret_cast<const double2*>(&sm.eth[tl][2 * c]);
#pragma unroll
        for (int j = 0; j < R; ++j) {
          acc[j] = fma(BV(j, 2 * c), e.x, acc[j]);
          if (2 * c + 1 < KL) acc[j] = fma(BV(j, 2 * c + 1), e.y, acc[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < R; ++j) pa[(8 * j + rl) * kPaPitch + tl] = acc[j];
    }
    STAMP(1);  // eθ reads, φ FMAs, partial stores
    __builtin_amdgcn_wave_barrier();
    if (R64_PRIO >= 2) __builtin_amdgcn_s_setprio(3);
    bool live = false;
    if (lane < 8 * R) {
      const double2* const pr = reinterpret_cast<const double2*>(pa + lane * kPaPitch);
      const double2 x0 = pr[0], x1 = pr[1], x2 = pr[2], x3 = pr[3];
      qdt = ((x0.x + x0.y) + (x1.x + x1.y)) + ((x2.x + x2.y) + (x3.x + x3.y));
      const double ph = fma(qe2, 0x1p-53, qdt);
      qr = qc * rcp_nr(ph);
      live = qe2 >= ph;  // ε' visible at fp64 resolution
      sm.rrow[w][lane] = qr;
    }
    if (__builtin_amdgcn_ballot_w64(live) != 0) {
      const double e = wave_sum_d(lane < 8 * R ? qr * (qe2 * 0x1p-53) : 0.0);
      if (lane == 0) sm.esum[w] = e;
    } else if (lane == 0) {
      sm.esum[w] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < R; ++j) rr[j] = sm.rrow[w][8 * j + rl];
    if (R64_PRIO >= 2) __builtin_amdgcn_s_setprio(0);
    STAMP(2);  // worker sums, r, ε' ballot, r reads
    // Spark: while (meanGammaChange > 1e-3); dsum is block-uniform (every wave adds the same LDS
    // values in the same order)
    if ((it > 0 && dsum <= a.stop_thr) || it >= a.max_iter) break;

    // Phase B: s partials over the lane's R rows, one row lane's slot per topic
    {  // the eight row lanes summed inside the wave (estep_common.h rs_rows8): lane (tl, rl) stores the wave
       // sums of its topic lane's topics 2·rl, 2·rl + 1, so a ψ lane reads 4 partials instead of 32
      double x[16];
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        double acc = 0.0;
        if (p < KL) {
#pragma unroll
          for (int j = 0; j < R; ++j) acc = fma(BV(j, p < KL ? p : 0), rr[j], acc);
        }
        x[p] = acc;
      }
      double s0, s1;
      rs_rows8(x, lane, s0, s1);
      if (2 * rl < KL) sb[(KL * tl + 2 * rl) * kSbPitch + w] = s0;
      if (2 * rl + 1 < KL) sb[(KL * tl + 2 * rl + 1) * kSbPitch + w] = s1;
    }
    STAMP(3);  // s FMAs + partial stores
    __syncthreads();  // (1) s partials and esum published
    STAMP(4);  // barrier 1
    const bool psi = npsi == 2 ? ((w >> 1) == (it & 1)) : (w == (it & 3));
    if (psi) {
      if (R64_PRIO >= 1) __builtin_amdgcn_s_setprio(3);
      double dg = 0.0;
      if (town) {
        // every LDS read of the phase issued together: the partials, γ, eθ, the four ε' sums
        const double2* const sp = reinterpret_cast<const double2*>(sb + tt * kSbPitch);
        const double2 x0 = sp[0], x1 = sp[1];  // the four waves' sums
        const double g = mir ? gm : sm.gam[tt], eo = sm.eth[ttl][ttp];
        const double2 ap = *reinterpret_cast<const double2*>(&sm.apc[tt][0]);  // α_t, ψc_t
        const double2 e01 = *reinterpret_cast<const double2*>(&sm.esum[0]);
        const double2 e23 = *reinterpret_cast<const double2*>(&sm.esum[2]);
        const double s = (x0.x + x0.y) + (x1.x + x1.y);
        const double et = (e01.x + e01.y) + (e23.x + e23.y);
        const double csn = et != 0.0 ? digamma_fast_d(sm.ac[0] + sm.ac[1] - et) : sm.ac[2];
        const double gn = fma(eo, s, ap.x);  // γ ← eθ ⊙ s + α
        dg = fabs(gn - g);
        sm.gam[tt] = gn;
        const double en = exp_digamma_minus_v4<R64_RCP_NR>(gn, csn + ap.y, expk);
        sm.eth[ttl][ttp] = en;
        gm = gn;
        em = en;
        if (tt == 0) sm.cs = csn;
      }
      if (!mir) {
        const double d = wave_sum_d(dg);
        if (lane == 0) sm.dsum[pw] = d;
      }
      if (R64_PRIO >= 1) __builtin_amdgcn_s_setprio(0);
    } else if (mir) {
      // the other wave of this topic set: the same γ update from its own γ / eθ registers (bitwise the ψ
      // wave's: same partials, same order), and Σ|Δγ| — its six-step reduction no longer sits on the ψ chain
      double dg = 0.0;
      if (town) {
        const double2* const sp = reinterpret_cast<const double2*>(sb + tt * kSbPitch);
        const double al = sm.apc[tt][0];
        const double2 y0 = sp[0], y1 = sp[1];
        const double s = (y0.x + y0.y) + (y1.x + y1.y);
        const double gn = fma(em, s, al);
        dg = fabs(gn - gm);
        gm = gn;  // (its eθ: the ψ wave's, from LDS, when this wave is next the ψ wave)
      }
      const double d = wave_sum_d(dg);
      if (lane == 0) sm.dsum[pw] = d;
    }
    STAMP(psi ? 5 : 8);  // ψ phase (ψ waves; non-ψ waves: nothing)
    __syncthreads();  // (2) eθ, γ, Σ|Δγ| published
    dsum = npsi == 2 ? sm.dsum[0] + sm.dsum[1] : sm.dsum[0];
    STAMP(psi ? 6 : 9);  // barrier 2 (ψ waves / the others)
    ++it;
  }
#undef BV
  STAMP_FLUSH
  return it;
}

// outputs: γ, E[log θ], eθ, the entries' r / keys / vals, iteration count, the bound
template <class S, bool STATS, bool BOUND, bool RES>
__device__ __forceinline__ void rows64_close(const EStepArgs<double>& a, RLds<S>& sm, const RDoc& d, int it, double qdt) {
  const int tid = rows64_tid<RES>(d);
  const int lane = d.lane, w = d.w;
  const int k = a.k, kp = a.kp, nnz = d.nnz, npsi = d.npsi, tt = d.tt, ttl = d.ttl, ttp = d.ttp;
  const bool town = d.town, tval = d.tval, wv = d.wv;
  const int64_t slot = d.slot, mem = d.mem, e0 = d.e0;
  const int qid = d.qid;
  const double qc = d.qc, qls = d.qls;
#ifdef STC_STAMP
  const unsigned long long st_close = stamp_now();
#endif
  // ---- outputs.  Exact Σγ of the final γ (ψ(Σγ) of E[log θ] and the bound)
  const double gfin = (w < npsi && town) ? sm.gam[tt] : 0.0;
  {
    const double gs = wave_sum_d(gfin);
    double bt = 0.0, bc = 0.0;
    if (BOUND && wv && qc != 0.0) {
      bt = qc * (log(fmax(qdt, 0x1p-1074)) + qls);
      bc = qc;
    }
    if (BOUND) {
      bt = wave_sum_d(bt);
      bc = wave_sum_d(bc);
    }
    if (lane == 0) {
      sm.part[w][0] = w < npsi ? gs : 0.0;
      sm.part[w][1] = bt;
      sm.part[w][2] = bc;
    }
    if (wv) sm.rid[w][lane] = qid;  // (rrow holds the final r since the last worker phase)
  }
  __syncthreads();
  const double gsum = (sm.part[0][0] + sm.part[1][0]) + (sm.part[2][0] + sm.part[3][0]);
  const double psisum = digamma_t<double>(gsum);
  double topic = 0.0;
  if (w < npsi) {
    if (town) {
      const double el = digamma_t<double>(gfin) - psisum;
      if (a.gamma) a.gamma[mem * k + tt] = gfin;
      if (STATS) a.elogth[slot * k + tt] = el;
      if (BOUND) {
        const double alp = sm.apc[tt][0];
        topic = (alp - gfin) * el + (lgamma(gfin) - lgamma(alp));
      }
    }
    if (STATS && tval) a.eth[slot * kp + tt] = sm.eth[ttl][ttp];  // the eθ the final φ used
  }
  // entry outputs in row order, consecutive threads on consecutive entries (whole cache lines: a
  // wave's own eight rows per set would be 32–64-byte pieces of lines another wave also writes)
  for (int n = tid; n < nnz; n += 64 * kW) {
    const int ws = (n >> 3) & 3, q = 8 * (n >> 5) + (n & 7);  // row n = 32·set + 8·wave + row lane
    const double rv = sm.rrow[ws][q];
    a.r[e0 + n] = rv;
    if (STATS && a.keys) {  // (null: the pairs were built and sorted beside the E-step, api.hip presort)
      a.keys[e0 + n] = (uint32_t)sm.rid[ws][q];
      a.vals[e0 + n] = entry_val<double>(slot, e0 + n, rv);
    }
  }
  if (tid == 0) {
    if (a.iters) a.iters[mem] = it;
    if (a.nonempty) a.nonempty[mem] = 1;
  }
  if (BOUND) {
    topic = wave_sum_d(topic);
    if (lane == 0) sm.part[w][3] = topic;
    __syncthreads();
    if (tid == 0) {
      double tok = 0.0, ctk = 0.0, tp = 0.0;
#pragma unroll
      for (int v = 0; v < kW; ++v) {
        tok += sm.part[v][1];
        ctk += sm.part[v][2];
        tp += sm.part[v][3];
      }
      const double elog_max = sm.cs - psisum;  // log of the scale eθ carried (≈ 0)
      a.bound[mem] = tok + ctk * elog_max + tp + (lgamma(sm.ac[0]) - lgamma(gsum));
    }
  }
#ifdef STC_STAMP
  if (lane == 0) atomicAdd(&g_stamps[7], stamp_now() - st_close);
#endif
}

// one document (slot, row, member and extent set by the caller): open → iterate<R> → close
// LONG: the 7–8-row-set documents; RES: a resident kernel (d.tid laundered per document)
template <class S, bool STATS, bool BOUND, bool LONG, bool RES = LONG>
__device__ __forceinline__ void rows64_doc(const EStepArgs<double>& a, RLds<S>& sm, RDoc& d) {
  d.e0 = a.bptr ? a.bptr[d.slot] : d.s0;
  if (!rows64_open<S, STATS, BOUND, RES>(a, sm, d)) return;
  double qdt = 0.0;
  int it;
  if constexpr (LONG) {
    it = d.rsets == 7 ? rows64_iterate<S, 7>(a, sm, d, qdt) : rows64_iterate<S, 8>(a, sm, d, qdt);
  } else {
    switch (d.rsets) {
      case 1: it = rows64_iterate<S, 1>(a, sm, d, qdt); break;
      case 2: it = rows64_iterate<S, 2>(a, sm, d, qdt); break;
      case 3: it = rows64_iterate<S, 3>(a, sm, d, qdt); break;
      case 4: it = rows64_iterate<S, 4>(a, sm, d, qdt); break;
      case 5: it = rows64_iterate<S, 5>(a, sm, d, qdt); break;
      default: it = rows64_iterate<S, 6>(a, sm, d, qdt); break;
    }
  }
  rows64_close<S, STATS, BOUND, RES>(a, sm, d, it, qdt);
}

// the documents with ≤ kOnChipSets row sets: one workgroup per slot (the long documents exit at once)
template <class S, bool STATS, bool BOUND>
__global__ __launch_bounds__(64 * kW, 2) void k_estep_rows64(EStepArgs<double> a) {
  __shared__ RLds<S> sm;
  if ((int64_t)blockIdx.x >= a.n) return;
  RDoc d;
#ifdef STC_STAMP
  d.st0 = stamp_now();
#endif
  d.slot = a.slot0 + blockIdx.x;
  d.row = a.batch ? (int64_t)a.batch[d.slot] : d.slot;
  d.mem = a.orig ? (int64_t)a.orig[d.slot] : d.slot;
  d.s0 = a.indptr[d.row];
  d.nnz = (int)(a.indptr[d.row + 1] - d.s0);
  d.rsets = (d.nnz + 31) >> 5;
  if (d.rsets > kOnChipSets) return;  // the long-document kernel's
  rows64_doc<S, STATS, BOUND, false>(a, sm, d);
}

// The same documents on a resident grid: every workgroup takes the next slot from a ticket counter and
// walks until the tickets run out (no dependency between workgroups: any residency drains).  A workgroup
// per slot paid a dispatch and its own prologue start per document; here the next ticket is requested at
// the start of a document and read at its end, and the per-document lane maps are laundered (as in the
// long-document kernel) so they are not hoisted and held across the fixed point.
template <class S, bool STATS, bool BOUND>
__global__ __launch_bounds__(64 * kW, 2) void k_estep_rows64_pers(EStepArgs<double> a, int32_t* ticket) {
  __shared__ RLds<S> sm;
  __shared__ int s_tk;
  if (threadIdx.x == 0) s_tk = atomicAdd(ticket, 1);
  __syncthreads();
  int cur = s_tk;
  while (cur < a.n) {
    __syncthreads();  // every thread has read s_tk
    int nxt = 0;
    if (threadIdx.x == 0) nxt = atomicAdd(ticket, 1);  // the next document's ticket, stored after this one
    RDoc d;
#ifdef STC_STAMP
    d.st0 = stamp_now();
#endif
    d.tid = threadIdx.x;
    asm volatile("" : "+v"(d.tid));
    d.slot = a.slot0 + cur;
    d.row = a.batch ? (int64_t)a.batch[d.slot] : d.slot;
    d.mem = a.orig ? (int64_t)a.orig[d.slot] : d.slot;
    d.s0 = a.indptr[d.row];
    d.nnz = (int)(a.indptr[d.row + 1] - d.s0);
    d.rsets = (d.nnz + 31) >> 5;
    if (d.rsets <= kOnChipSets) rows64_doc<S, STATS, BOUND, false, true>(a, sm, d);
    if (threadIdx.x == 0) s_tk = nxt;
    __syncthreads();  // LDS is the next document's; s_tk published
    cur = s_tk;
  }
}

// the launch's 7–8-set documents into a.long_list: word 0 the count, then their slot offsets (in any
// order: every document's outputs are its own)
__global__ void k_rows64_long_list(EStepArgs<double> a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int64_t slot = a.slot0 + i;
  const int64_t row = a.batch ? (int64_t)a.batch[slot] : slot;
  const int nnz = (int)(a.indptr[row + 1] - a.indptr[row]);
  if (nnz > 32 * kOnChipSets) a.long_list[1 + atomicAdd(&a.long_list[0], 1)] = (int32_t)i;
}

// the 7–8-set documents at one workgroup per CU, a resident grid walking the list (a grid over every
// slot would dispatch ~n workgroups at that occupancy only to have most exit after two dependent loads)
template <class S, bool STATS, bool BOUND>
__global__ __launch_bounds__(64 * kW, R64_LONG_OCC) void k_estep_rows64_long(EStepArgs<double> a) {
  __shared__ RLds<S> sm;
  const int cnt = a.long_list[0];
  for (int j = blockIdx.x; j < cnt; j += gridDim.x) {
    RDoc d;
#ifdef STC_STAMP
    d.st0 = stamp_now();
#endif
    // every per-lane value derives from tid: laundered per document, so the compiler cannot hoist the
    // lane maps and the α / ψc loads out of the document loop and hold them across the fixed point
    d.tid = threadIdx.x;
    asm volatile("" : "+v"(d.tid));
    d.slot = a.slot0 + a.long_list[1 + j];
    d.row = a.batch ? (int64_t)a.batch[d.slot] : d.slot;
    d.mem = a.orig ? (int64_t)a.orig[d.slot] : d.slot;
    d.s0 = a.indptr[d.row];
    d.nnz = (int)(a.indptr[d.row + 1] - d.s0);
    d.rsets = (d.nnz + 31) >> 5;
    rows64_doc<S, STATS, BOUND, true>(a, sm, d);
    __syncthreads();  // LDS is the next document's
  }
}

template <class S>
bool launch_persist(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound) {
  if (!a.long_list || bound) return false;  // (the bound E-step keeps a workgroup per slot)
  int32_t* ticket = a.long_list + a.n + 1;  // the word past the long-document list (api.hip reserves it)
  auto go = [&](const void* kern) {
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kW, 0));
    if (per_cu < 1) return false;
    HIP_CHECK(hipMemsetAsync(ticket, 0, sizeof(int32_t), s));
    EStepArgs<double> aa = a;
    void* args[] = {&aa, &ticket};
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(a.n, (int64_t)per_cu * cus));
    HIP_CHECK(hipLaunchKernel(kern, dim3((unsigned)blocks), dim3(64 * kW), args, 0, s));
    return true;
  };
  if (stats) return go((const void*)k_estep_rows64_pers<S, true, false>);
  return go((const void*)k_estep_rows64_pers<S, false, false>);
}
template <class S>
void launch_common(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound) {
  if (launch_persist<S>(s, a, stats, bound)) return;
  const dim3 grid((unsigned)a.n);
  const int threads = 64 * kW;
  if (stats) k_estep_rows64<S, true, false><<<grid, threads, 0, s>>>(a);
  else if (bound) k_estep_rows64<S, false, true><<<grid, threads, 0, s>>>(a);
  else k_estep_rows64<S, false, false><<<grid, threads, 0, s>>>(a);
  KERNEL_CHECK();
}
template <class S>
void launch_long(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound) {
  if (!a.long_list) throw Error(STC_ERR_STATE, "fp64 rows E-step: no long-document list buffer");
  HIP_CHECK(hipMemsetAsync(a.long_list, 0, sizeof(int32_t), s));
  k_rows64_long_list<<<dim3((unsigned)((a.n + 255) / 256)), 256, 0, s>>>(a);
  KERNEL_CHECK();
  int dev = 0, cus = 0;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(a.n, (int64_t)cus * R64_LONG_OCC)));
  const int threads = 64 * kW;
  if (stats) k_estep_rows64_long<S, true, false><<<grid, threads, 0, s>>>(a);
  else if (bound) k_estep_rows64_long<S, false, true><<<grid, threads, 0, s>>>(a);
  else k_estep_rows64_long<S, false, false><<<grid, threads, 0, s>>>(a);
  KERNEL_CHECK();
}
// the 7–8-set documents first (`long_docs` = false when the caller knows there are none), then the rest
template <int KL>
void launch_r(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound, bool long_docs) {
  if (long_docs) launch_long<RLong<KL>>(s, a, stats, bound);
  launch_common<RCommon<KL>>(s, a, stats, bound);
}

}  // namespace

int rows64_row_cap(int k) { return k <= 104 ? 32 * kMaxSets : 0; }
int rows64_onchip_rows(int k) { return k <= 104 ? 32 * kOnChipSets : 0; }

void launch_estep_rows64(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound, bool long_docs) {
  if (a.n == 0) return;
  if (a.kp > 8 * 13 || a.kp < a.k || (a.kp & 1)) throw Error(STC_ERR_INVALID_ARG, "fp64 rows E-step: bad k / kp");
  if (a.k <= 32) launch_r<4>(s, a, stats, bound, long_docs);
  else if (a.k <= 56) launch_r<7>(s, a, stats, bound, long_docs);
  else launch_r<13>(s, a, stats, bound, long_docs);
}

STC_STAMP_READER(stc_debug_stamps_rows64)

}  // namespace lda
}  // namespace stc
