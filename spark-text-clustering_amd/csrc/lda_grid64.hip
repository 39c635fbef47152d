// lda_grid64.hip — K6 at Spark's precision: the row-lane × topic-group grid E-step of lda_grid.hip
// in fp64 ([U] OnlineLDAOptimizer.variationalTopicInference computes in Breeze Double).
//
// One document per workgroup of W wavefronts.  Inside a wave lane bit 3 picks a topic group g and the
// other five lane bits a row lane rl; wave w, group g own KL = 13 topics [(2w+g)·13, +13), so k ≤ 104
// takes W = 4 (k = 100: eight slices of 13).  A lane holds rows n = 32·j + rl (j < R, R = ⌈nnz/32⌉
// chosen per document) of its slice: R·13 doubles = 26·R VGPRs for R ≤ 5; a sixth row set (nnz ≤ 192)
// is read from LDS, which keeps the loop free of scratch spills at two waves per SIMD.  Documents with
// a seventh and eighth set (nnz ≤ 256: long documents, and 13 % of a planted-topic corpus at L = 200)
// run in a second launch with all eight sets in VGPRs at one wave per SIMD (the row-streaming path,
// expElogβ' re-read each pass, remains for a shape with fewer register sets than row sets).
//   φ_n = B_n·eθ : 13 lane-local fp64 FMAs per row, + the other group's partial through a 64-bit DPP
//     row_ror:8 (lane i ↔ i^8), then the W wave partials meet in LDS.  W = 4: row set j's total and
//     r = cts/φ are computed ONCE, by the (wave, group) pair 2·wave + group = j, and published behind
//     a second barrier (one rcp chain per row instead of eight; 459 → 408 VALU instructions per
//     iteration at R = 5).  W < 4: every wave adds the partials in the same order behind one barrier.
//     Either way every wave sees bit-identical φ and r.
//   s = Bᵀr : lane-local FMAs into 13 partials, reduce-scattered over the 32 row lanes (permlane32 /
//     permlane16 swaps of both dwords, then row_half_mirror / quad_perm DPP pairs, all keeping bit 3)
//     — each lane ends owning at most one topic of its group.
//   γ, ψ(γ), exp on the owned topic; eθ back into the group's LDS slice (read only by this wave).
//   ψ(Σγ') from Σγ' = Σα + Σ_n cts_n − Σ_n cts_n·ε'_n/φ_n (exact in real arithmetic): a per-document
//     constant unless a ballot finds a row whose ε' is visible at fp64 resolution (ε' ≥ 2^-53·φ).
// Numerics as lda.hip: Bp row-scaled by e^{-m_v}, Spark's 1e-100 carried as ε'_n = 1e-100·e^{-m_v}.
#include "estep_common.h"

#ifndef G64_LOAD_BATCH
#define G64_LOAD_BATCH 3  // row sets whose B loads are in flight together in the load phase
#endif

namespace stc {
namespace lda {

namespace {

// (waves per document, topics per lane group, max rows per lane, row sets in VGPRs)
template <int W_, int KL_, int RMAX_, int RREG_ = 5>
struct DShape {
  static constexpr int W = W_, KL = KL_, RMAX = RMAX_;
  static constexpr int RREG = RREG_;  // row sets per lane in VGPRs (26·5 = 130); the next goes to LDS
  static constexpr int RLDS = RREG + 1;  // row sets past this one are streamed from expElogβ'
  static constexpr int KLP = (KL + 1) / 2 * 2;  // LDS slice pitch (ds_read_b128 granules)
};
using D26 = DShape<1, 13, 8>;   // k <= 26
using D52 = DShape<2, 13, 8>;   // k <= 52
using D104 = DShape<4, 13, 8>;  // k <= 104 (k = 100: 8 slices of 13 topics)
constexpr int kOnChipSets = 6;   // row sets the common kernel holds on chip (5 in VGPRs + 1 in LDS)
// the long-document kernel's shape: all G64_LONG_RREG = 8 row sets in VGPRs at one workgroup per CU
// (G64_LONG_OCC; 346 VGPRs of the 512 a lone wave gets, no scratch, nothing streamed).  Measured on the
// planted-topic state (13 % of its documents have 193–256 rows): E-step 6.79 → 6.31 ms against five
// register sets at two workgroups per CU, which spilled and re-read two sets from expElogβ' per pass
// (four register sets: no fewer spills).
#ifndef G64_LONG_RREG
#define G64_LONG_RREG 8
#endif
#ifndef G64_LONG_OCC
#define G64_LONG_OCC 1  // long-document kernel workgroups per CU the register budget is cut for
#endif
template <class S>
using DLong = DShape<S::W, S::KL, S::RMAX, G64_LONG_RREG>;

template <class S>
struct DLds {
  double eth[S::W][2][S::KLP] __attribute__((aligned(16)));
  // the load stage (one 32-row step of the wave's 2·KL columns) is dead once the loop starts
  union {
    double phi[2][S::W][S::RMAX][32];   // W < 4: per row lane (both groups hold the same joined φ)
    double phig[2][S::W][2][S::RMAX][32];  // W = 4: per (wave, group) partial, joined by the set's worker
    double stage[S::W][32 * 2 * S::KL];
  } __attribute__((aligned(16)));
  double red[2][S::W][2];
  double bd[S::W][2];
  // W = 4: each row set's total φ and r, computed once by the (wave, group) that owns the set
  double rtot[S::RMAX][32], dtot[S::RMAX][32];
  int epsf[S::W];
  // per-row counts and 2^53·ε' (read each iteration from here rather than held in VGPRs)
  double rowc[32 * S::RMAX], rowe[32 * S::RMAX];
  // rows past RREG·32 (the sixth row set): their (wave, group) slice lives here, [p][row lane] with
  // the group stride padded by 16 doubles so the two groups of a ds_read_b64 half-wave hit disjoint banks
  double ovf[S::W * 2][S::KL * 32 + 16];
};

// cross-wave exchange of nd φ partials per lane + two wave-uniform scalars behind one barrier; every
// wave combines them in the same order ⇒ bit-identical results in every wave.  Double-buffered by
// parity: a buffer is reused only after every wave has passed the following barrier.
// The two lane groups hold the same joined φ (a + b == b + a), so a row's slot is indexed by the row
// lane: both groups store the same value to it.
template <class S>
__device__ __forceinline__ void xchg_d(DLds<S>& sm, int b, int wave, int lane, int rl, double* dot, int nd,
                                       double& x, double& y) {
  constexpr int W = S::W;
  if constexpr (W > 1) {
    double* const base = &sm.phi[0][0][0][0] + rl;
    constexpr int BS = S::W * S::RMAX * 32, WS = S::RMAX * 32;
    double* const mine = base + (b * BS + wave * WS);
#pragma unroll
    for (int j = 0; j < nd; ++j) mine[32 * j] = dot[j];
    if (lane == 0) {
      sm.red[b][wave][0] = x;
      sm.red[b][wave][1] = y;
    }
    __syncthreads();
    if constexpr (W == 2) {
      const int o = wave ^ 1;
      const double* const other = base + (b * BS + o * WS);
#pragma unroll
      for (int j = 0; j < nd; ++j) dot[j] += other[32 * j];  // a + b == b + a: identical in both waves
      x += sm.red[b][o][0];
      y += sm.red[b][o][1];
    } else {
      const double* const b0 = base + b * BS;
#pragma unroll
      for (int j = 0; j < nd; ++j) {
        double d = b0[32 * j];
#pragma unroll
        for (int w = 1; w < W; ++w) d += b0[w * WS + 32 * j];
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

struct DDoc {
  int lane, wave, g, rl, nnz, k, kp, t0, tl, t, it;
  bool ok, own;
  int64_t slot, row, mem, s0, e0;
  double gam, alp, eth, cs, gsum, asum;
  double b_tok, c_tok;
};

template <class S, int R, bool STATS, bool BOUND>
__device__ __forceinline__ bool grid64_core(const EStepArgs<double>& a, DLds<S>& sm, DDoc& d) {
  constexpr int W = S::W, KL = S::KL, KLP = S::KLP;
  constexpr int N1 = hup(KL), N2 = hup(N1), N3 = hup(N2), N4 = hup(N3), N5 = hup(N4);
  static_assert(N5 == 1 && R >= 1 && R <= S::RMAX, "shape");
  const int lane = d.lane, wave = d.wave, rl = d.rl, nnz = d.nnz, kp = d.kp;
  const int64_t s0 = d.s0, e0 = d.e0;
  double* const my_eth = sm.eth[d.wave][d.g];

  // ---- load in two dependent rounds with every address valid: (1) ids and counts; (2) m_v and the
  // B rows.  Rows past nnz read entry 0 / term 0 and are zeroed; columns past kp are clamped + zeroed.
  constexpr int RG = R < S::RREG ? R : S::RREG;  // row sets held in VGPRs; the next in sm.ovf
  constexpr int RL = R < S::RLDS ? R : S::RLDS;  // row sets held on chip; [RL, R) are streamed
  double B[RG][KL];
  double* const ovf = sm.ovf[2 * wave + d.g] + rl;
  // B_{32j+rl, p} of this lane's slice, from registers or (j >= RG) from LDS
#define BV(j, p) ((j) < RG ? B[(j) < RG ? (j) : 0][p] : ovf[32 * (p)])
  double rr[R];
  int ids[R];
  int any = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int n = 32 * j + rl;
    const bool v = n < nnz;
    const int64_t e = v ? s0 + n : 0;
    const int id = a.indices[e];
    const double c = a.values[e];
    ids[j] = v ? id : 0;
    any |= (v && c != 0.0);
    if (wave == 0 && d.g == 0) sm.rowc[n] = v ? c : 0.0;
    rr[j] = 0.0;
  }
  double ls[R];
#pragma unroll
  for (int j = 0; j < R; ++j) ls[j] = a.logscale[ids[j]];
  // B rows, coalesced: per 32-row step the wave copies its 2·KL columns of the 32 rows with 16-byte
  // loads (consecutive lanes → consecutive pieces of one row), stages them in LDS, and every lane
  // picks up its (row, group) part
  constexpr int C2 = KL;                          // double2 pieces per staged row (2·KL doubles)
  constexpr int NP = (32 * C2 + 63) / 64;         // pieces per lane per step
  const int wcol = wave * 2 * KL;                 // the wave's first column (even)
  double* const stg = sm.stage[wave];
  // the loads of LB row sets are issued together (one memory latency per batch rather than per row
  // set), then staged one row set at a time through the wave's stage buffer
#pragma unroll
  for (int j0 = 0; j0 < RL; j0 += G64_LOAD_BATCH) {
    double2 pc[G64_LOAD_BATCH][NP];
#pragma unroll
    for (int jj = 0; jj < G64_LOAD_BATCH; ++jj) {
      const int j = j0 + jj;
      if (j >= RL) break;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int c = lane + 64 * i;
        const int srow = c / C2, q = c - srow * C2;
        const int src_lane = (srow & 7) | ((srow >> 3) << 4);  // the group-0 lane holding row srow
        const int id = __builtin_amdgcn_ds_bpermute(src_lane << 2, ids[j]);
        const int col = wcol + 2 * q;
        const double2 x = *reinterpret_cast<const double2*>(a.Bp + (int64_t)id * kp + min(col, kp - 2));
        const bool keep = c < 32 * C2 && 32 * j + srow < nnz && col < kp;
        pc[jj][i] = keep ? x : make_double2(0.0, 0.0);
      }
    }
#pragma unroll
    for (int jj = 0; jj < G64_LOAD_BATCH; ++jj) {
      const int j = j0 + jj;
      if (j >= RL) break;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int c = lane + 64 * i;
        if (c < 32 * C2) *reinterpret_cast<double2*>(stg + 2 * c) = pc[jj][i];  // row c / C2, piece c % C2
      }
      __builtin_amdgcn_wave_barrier();  // one wave writes and reads its stage; LDS is in order per wave
      const double* mine = stg + rl * 2 * KL + d.g * KL;
#pragma unroll
      for (int p = 0; p < KL; ++p) {
        if (j < RG) B[j < RG ? j : 0][p] = mine[p];
        else ovf[32 * p] = mine[p];  // read back only by this lane
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  // ε'_n = 1e-100·e^{-m_v} held as 2^53·ε'_n (the ballot below asks 2^53·ε' ≥ φ directly), capped at
  // 1e300 where e^{-m_v} overflows (Spark's unscaled expElogβ row is then 0 and the row contributes
  // nothing; r ≈ cts·1e-284 reproduces that without an ∞ in the Newton reciprocal).  Padding rows
  // hold −2^53 (φ = −1, r = −0, never live).
  // streamed row sets: the lane's KL entries of row 32·j + rl, zero past nnz and past kp.  The offset
  // goes through an empty asm each pass so the loads stay inside the loop (hoisted, they would spill)
  const int64_t col0 = d.t0;
  auto stream_row = [&](int j, double* y) {
    int64_t off = (int64_t)ids[j] * kp;
    asm volatile("" : "+v"(off));
    const bool v = 32 * j + rl < nnz;
#pragma unroll
    for (int p = 0; p < KL; ++p) {
      const double x = a.Bp[off + min(col0 + p, (int64_t)kp - 1)];
      y[p] = (v && col0 + p < kp) ? x : 0.0;
    }
  };
  if (wave == 0 && d.g == 0) {
#pragma unroll
    for (int j = 0; j < R; ++j)
      sm.rowe[32 * j + rl] = (32 * j + rl < nnz) ? fmin(0x1p53 * exp(kLogEps - ls[j]), 1e300) : -0x1p53;
  }
  bool nonempty;  // (the block barrier below also publishes rowc / rowe)
  if constexpr (W > 1) nonempty = __syncthreads_or(any) != 0;
  else nonempty = __any(any);

  if (nonempty) {
    double gsum = d.gsum, asum = d.asum, dsum = 0.0, dummy = 0.0;
    xchg_d<S>(sm, 1, wave, lane, rl, nullptr, 0, gsum, asum);
    d.asum = asum;
    // eθ = exp(ψ(γ) − ψ(Σγ)): Spark's unscaled exp(E[log θ]); inside the loop ψ(Σγ') comes from the
    // Σα + Σcts − Σ cts·ε'/φ identity, so without live ε' it is one constant per document
    double cs = digamma_fast_d(gsum);
    double ct = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) ct += sm.rowc[32 * j + rl];
    const double ctot = 0.5 * wave_sum_d(ct);  // Σ_n cts_n (each row is held by both groups)
    const double cs_flat = digamma_fast_d(asum + ctot);
    double gam = d.gam, eth = d.own ? exp_digamma_minus_d(gam, cs) : 0.0;
    const double alp = d.alp;
    if (d.own) my_eth[d.tl] = eth;
    __builtin_amdgcn_wave_barrier();  // the slices are read back only by this wave
    int it = 0;
    double dg = 0.0;  // |Δγ| of the owned topic in the last update
    while (true) {
      // Phase A: φ_n = B_n·eθ (+ ε'_n below) ; r_n = cts_n / φ_n
      double dot[R];
      {
        double acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = 0.0;
#pragma unroll
        for (int c = 0; c < KLP / 2; ++c) {
          const double2 e = *reinterpret_cast<const double2*>(my_eth + 2 * c);
#pragma unroll
          for (int j = 0; j < RL; ++j) {
            acc[j] = fma(BV(j, 2 * c), e.x, acc[j]);
            if (2 * c + 1 < KL) acc[j] = fma(BV(j, 2 * c + 1), e.y, acc[j]);
          }
        }
#pragma unroll
        for (int j = RL; j < R; ++j) {
          double y[KL];
          stream_row(j, y);
#pragma unroll
          for (int c = 0; c < KLP / 2; ++c) {
            const double2 e = *reinterpret_cast<const double2*>(my_eth + 2 * c);
            acc[j] = fma(y[2 * c], e.x, acc[j]);
            if (2 * c + 1 < KL) acc[j] = fma(y[2 * c + 1], e.y, acc[j]);
          }
        }
        if constexpr (W == 4) {  // the groups' partials are joined by the set's worker (LDS)
#pragma unroll
          for (int j = 0; j < R; ++j) dot[j] = acc[j];
        } else {
#pragma unroll
          for (int j = 0; j < R; ++j) dot[j] = acc[j] + dpp_d<DPP_ROW_ROR8>(acc[j]);  // + the other group
        }
      }
      // Σ|Δγ| of the last update rides along with the φ exchange
      dsum = wave_sum_d(dg);
      bool last;
      uint64_t eps_live = 0;
      if constexpr (W == 4) {
        // the partials of the four waves meet in LDS; row set j's total φ and r are then computed ONCE,
        // by worker (wave, group) = ((j mod 8) / 2, j mod 2) — the same sum order as every wave used
        // before, so the same bits — and published for every wave behind a second barrier
        double* const base = &sm.phig[0][0][0][0][0] + rl;
        constexpr int GS = S::RMAX * 32, WS = 2 * GS, BS = S::W * WS;
        const int b = it & 1;
#pragma unroll
        for (int j = 0; j < R; ++j) base[b * BS + wave * WS + d.g * GS + 32 * j] = dot[j];
        if (lane == 0) sm.red[b][wave][0] = dsum;
        __syncthreads();  // (A) partials published
        dsum = sm.red[b][0][0];
#pragma unroll
        for (int w = 1; w < W; ++w) dsum += sm.red[b][w][0];
        last = __builtin_amdgcn_readfirstlane((int)((it > 0 && dsum <= a.stop_thr) || it >= a.max_iter)) != 0;
        const int j = 2 * wave + d.g;  // this worker's row set (R ≤ 8 = workers)
        bool live = false;
        if (j < R) {
          const double* const b0 = base + b * BS + 32 * j;
          double dt = b0[0] + b0[GS];  // (wave 0, group 0) + (wave 0, group 1), then waves 1..3 alike
#pragma unroll
          for (int w = 1; w < W; ++w) dt += b0[w * WS] + b0[w * WS + GS];
          const double cj = sm.rowc[32 * j + rl], ej = sm.rowe[32 * j + rl];
          const double ph = fma(ej, 0x1p-53, dt);
          sm.rtot[j][rl] = cj * rcp_nr(ph);
          sm.dtot[j][rl] = dt;
          live = ej >= ph;  // ε' visible at fp64 resolution
        }
        const uint64_t lv = __builtin_amdgcn_ballot_w64(live);
        if (lane == 0) sm.epsf[wave] = lv != 0;
        __syncthreads();  // (B) r and φ totals published
#pragma unroll
        for (int jj = 0; jj < R; ++jj) {
          rr[jj] = sm.rtot[jj][rl];
          dot[jj] = sm.dtot[jj][rl];
        }
        eps_live = (sm.epsf[0] | sm.epsf[1] | sm.epsf[2] | sm.epsf[3]) != 0;
        if (BOUND && last && d.g == 0) {
#pragma unroll
          for (int jj = 0; jj < R; ++jj) {
            const double cj = sm.rowc[32 * jj + rl];
            if (cj != 0.0) {
              d.b_tok += cj * (log(fmax(dot[jj], 0x1p-1074)) + a.logscale[a.indices[s0 + 32 * jj + rl]]);
              d.c_tok += cj;
            }
          }
        }
      } else {
        xchg_d<S>(sm, it & 1, wave, lane, rl, dot, R, dsum, dummy);
        // Spark: while (meanGammaChange > 1e-3), meanGammaChange = Σ|Δγ| / k.  Wave-uniform by
        // construction; readfirstlane makes the loop a scalar loop
        last = __builtin_amdgcn_readfirstlane((int)((it > 0 && dsum <= a.stop_thr) || it >= a.max_iter)) != 0;
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const double cj = sm.rowc[32 * j + rl], ej = sm.rowe[32 * j + rl];
          const double ph = fma(ej, 0x1p-53, dot[j]);
          rr[j] = cj * rcp_nr(ph);
          eps_live |= __builtin_amdgcn_ballot_w64(ej >= ph);  // ε' visible at fp64 resolution
          if (BOUND && last && d.g == 0 && cj != 0.0) {
            d.b_tok += cj * (log(fmax(dot[j], 0x1p-1074)) + a.logscale[a.indices[s0 + 32 * j + rl]]);
            d.c_tok += cj;
          }
        }
      }
      if (last) break;
      // ψ(Σγ') for the next eθ (see the header); the ε' part only when the ballot saw one
      double cs_next = cs_flat;
      if (eps_live) {
        double e = 0.0;
#pragma unroll
        for (int j = 0; j < R; ++j)  // cts·ε'/φ as cts·(1 − dot/φ): 0 for padding, cts when ε' = ∞
          e = fma(sm.rowc[32 * j + rl], 1.0 - dot[j] * rcp_nr(fma(sm.rowe[32 * j + rl], 0x1p-53, dot[j])), e);
        cs_next = digamma_fast_d(asum + ctot - 0.5 * wave_sum_d(e));  // each row is held twice
      }

      // Phase B: s = Bᵀr over the group's KL topics, then reduce-scatter over the 32 row lanes
      double flat[KL];
#pragma unroll
      for (int p = 0; p < KL; ++p) {
        double x = 0.0;
#pragma unroll
        for (int j = 0; j < RL; ++j) x = fma(BV(j, p), rr[j], x);
        flat[p] = x;
      }
#pragma unroll
      for (int j = RL; j < R; ++j) {
        double y[KL];
        stream_row(j, y);
#pragma unroll
        for (int p = 0; p < KL; ++p) flat[p] = fma(y[p], rr[j], flat[p]);
      }
      double ys1[N1];
#pragma unroll
      for (int q = 0; q < N1; ++q) ys1[q] = (N1 + q < KL) ? flat[N1 + q] : 0.0;
      double p1[N1];
      swap_add_nd<true, N1>(flat, ys1, p1);  // bit 5
      double ys2[N2];
#pragma unroll
      for (int q = 0; q < N2; ++q) ys2[q] = (N2 + q < N1) ? p1[N2 + q] : 0.0;
      double p2[N2];
      swap_add_nd<false, N2>(p1, ys2, p2);  // bit 4
      double p3[N3];
#pragma unroll
      for (int q = 0; q < N3; ++q)
        p3[q] = rs_dpp_d<DPP_ROW_HALF_MIRROR>(p2[q], (N3 + q < N2) ? p2[N3 + q] : 0.0, lane & 4);
      double p4[N4];
#pragma unroll
      for (int q = 0; q < N4; ++q)
        p4[q] = rs_dpp_d<DPP_QP_3210>(p3[q], (N4 + q < N3) ? p3[N4 + q] : 0.0, lane & 2);
      double y5 = 0.0;
      if constexpr (N5 < N4) y5 = p4[N5];
      const double s_own = rs_dpp_d<DPP_QP_1032>(p4[0], y5, lane & 1);

      // Phase C: γ ← eθ ⊙ s + α on the owned topic (lanes without one keep γ = 0 and dg = 0)
      {
        const double gn = fma(eth, s_own, alp);
        dg = d.own ? fabs(gn - gam) : 0.0;
        gam = d.own ? gn : gam;
      }
      // Phase D: eθ = exp(ψ(γ) − ψ(Σγ)) into the group's LDS slice (computed in every lane, stored
      // by the owners)
      cs = cs_next;
      eth = d.own ? exp_digamma_minus_d(d.own ? gam : 1.0, cs) : 0.0;
      if (d.own) my_eth[d.tl] = eth;
      __builtin_amdgcn_wave_barrier();
      ++it;
    }
#undef BV
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
          a.keys[e0 + n] = (uint32_t)a.indices[s0 + n];
          a.vals[e0 + n] = entry_val<double>(d.slot, e0 + n, rr[j]);
        }
      }
    }
  }
  return nonempty;
}

// LONG = false: documents with ≤ RLDS row sets; LONG = true: the streamed ones (nnz > 32·RLDS).  Both
// kernels run over the same slots and each skips the other's documents, so the streamed variants'
// register pressure stays out of the common kernel.
template <class S, bool STATS, bool BOUND, bool LONG>
__global__ __launch_bounds__(64 * S::W, LONG ? G64_LONG_OCC : 2) void k_estep_grid64(EStepArgs<double> a) {
  constexpr int W = S::W, KL = S::KL;
  constexpr int N1 = hup(KL), N2 = hup(N1), N3 = hup(N2), N4 = hup(N3), N5 = hup(N4);
  __shared__ DLds<S> sm;
  if ((int64_t)blockIdx.x >= a.n) return;
  DDoc d;
  d.lane = threadIdx.x & 63;
  d.wave = threadIdx.x >> 6;
  d.g = (d.lane >> 3) & 1;
  d.rl = (d.lane & 7) | ((d.lane >> 4) << 3);
  d.slot = a.slot0 + blockIdx.x;
  d.row = a.batch ? (int64_t)a.batch[d.slot] : d.slot;
  d.mem = a.orig ? (int64_t)a.orig[d.slot] : d.slot;
  d.s0 = a.indptr[d.row];
  d.nnz = (int)(a.indptr[d.row + 1] - d.s0);
  const int rsets = (d.nnz + 31) >> 5;
  if (LONG ? rsets <= kOnChipSets : rsets > kOnChipSets) return;  // the other kernel's document
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
  d.gam = d.own ? (a.gamma0 ? a.gamma0[mem * k + t] : gamma_sample(stream, t, a.gamma_shape)) : 0.0;
  d.alp = d.own ? a.alpha[t] : 0.0;
  d.gsum = wave_sum_d(d.gam);
  d.asum = wave_sum_d(d.alp);
  for (int i = lane; i < 2 * S::KLP; i += 64) (&sm.eth[d.wave][0][0])[i] = 0.0;  // pads stay zero
  d.eth = 0.0;
  d.cs = 0.0;
  d.it = 0;
  d.b_tok = 0.0;
  d.c_tok = 0.0;

  // rows per lane for this document (block-uniform); the partition guarantees nnz <= 32·RMAX
  bool nonempty = false;
  static_assert(kOnChipSets == 6 && S::RMAX == 8 && (LONG || S::RLDS == kOnChipSets), "row-set cases below");
  if constexpr (LONG) {
    if (rsets == 7) nonempty = grid64_core<S, 7, STATS, BOUND>(a, sm, d);
    else nonempty = grid64_core<S, 8, STATS, BOUND>(a, sm, d);
  } else {
    switch (rsets) {
      case 0:
      case 1: nonempty = grid64_core<S, 1, STATS, BOUND>(a, sm, d); break;
      case 2: nonempty = grid64_core<S, 2, STATS, BOUND>(a, sm, d); break;
      case 3: nonempty = grid64_core<S, 3, STATS, BOUND>(a, sm, d); break;
      case 4: nonempty = grid64_core<S, 4, STATS, BOUND>(a, sm, d); break;
      case 5: nonempty = grid64_core<S, 5, STATS, BOUND>(a, sm, d); break;
      default: nonempty = grid64_core<S, 6, STATS, BOUND>(a, sm, d); break;
    }
  }

  // ---- topic-level outputs, once per kernel
  const int wave = d.wave;
  if (!nonempty) {
    if (d.own) {
      if (a.gamma) a.gamma[mem * k + t] = 0.0;
      if (STATS) a.elogth[slot * k + t] = 0.0;
    }
    if (STATS && d.ok && t < kp) a.eth[slot * kp + t] = 0.0;
    if (wave == 0 && lane == 0) {
      if (a.iters) a.iters[mem] = 0;
      if (a.nonempty) a.nonempty[mem] = 0;
      if (BOUND) a.bound[mem] = 0.0;
    }
    return;
  }
  // exact Σγ of the final γ (outputs and bound); the loop's last barrier used buffer it & 1
  double gsum = wave_sum_d(d.own ? d.gam : 0.0), dummy = 0.0;
  xchg_d<S>(sm, (d.it + 1) & 1, wave, lane, d.rl, nullptr, 0, gsum, dummy);
  const double psisum = digamma_t<double>(gsum);
  if (d.own) {
    if (a.gamma) a.gamma[mem * k + t] = d.gam;
    if (STATS) a.elogth[slot * k + t] = digamma_t<double>(d.gam) - psisum;
  }
  if (STATS && d.ok && t < kp) a.eth[slot * kp + t] = sm.eth[wave][d.g][d.tl];  // the eθ φ used
  if (wave == 0 && lane == 0) {
    if (a.iters) a.iters[mem] = d.it;
    if (a.nonempty) a.nonempty[mem] = 1;
  }
  if (BOUND) {
    // token terms from the group-0 lanes of wave 0 (each row once); topic terms summed over waves
    double topic = 0.0, as = 0.0;
    if (d.own) {
      const double gd = d.gam, al = a.alpha[t];
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
      const double elog_max = d.cs - psisum;  // log of the scale eθ carried (≈ 0)
      a.bound[mem] = tok + ct * elog_max + tp + (lgamma(asw) - lgamma(gsum));
    }
  }
}

template <class S, bool LONG>
void launch_d1(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound) {
  const dim3 grid((unsigned)a.n);
  const int threads = 64 * S::W;
  if (stats) k_estep_grid64<S, true, false, LONG><<<grid, threads, 0, s>>>(a);
  else if (bound) k_estep_grid64<S, false, true, LONG><<<grid, threads, 0, s>>>(a);
  else k_estep_grid64<S, false, false, LONG><<<grid, threads, 0, s>>>(a);
  KERNEL_CHECK();
}
// the streamed-row documents first (longest first), then the rest; `long_docs` = false when the
// caller knows no document has more than 32·RLDS rows
template <class S>
void launch_d(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound, bool long_docs) {
  if (long_docs) launch_d1<DLong<S>, true>(s, a, stats, bound);
  launch_d1<S, false>(s, a, stats, bound);
}

}  // namespace

int grid64_row_cap(int k) {
  if (k <= 104) return 32 * D104::RMAX;
  return 0;
}
int grid64_onchip_rows(int k) { return k <= 104 ? 32 * kOnChipSets : 0; }

void launch_estep_grid64(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound, bool long_docs) {
  if (a.n == 0) return;
  if (a.k <= 26) launch_d<D26>(s, a, stats, bound, long_docs);
  else if (a.k <= 52) launch_d<D52>(s, a, stats, bound, long_docs);
  else if (a.k <= 104) launch_d<D104>(s, a, stats, bound, long_docs);
  else throw Error(STC_ERR_INVALID_ARG, "fp64 grid E-step: k > 104");
}

}  // namespace lda
}  // namespace stc
