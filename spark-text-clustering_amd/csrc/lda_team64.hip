// lda_team64.hip — K6 at Spark's precision for many topics (fp64, k > 104: BASELINE config 4's k = 500):
// one document per TEAM of P workgroups (P CUs), the TOPICS split over the members, and inside a member
// the rows64 grid ([U] OnlineLDAOptimizer.variationalTopicInference in Breeze Double, called per document
// inside submitMiniBatch behind lda.run, TextClustering/src/main/scala/LDAClustering.scala:61).
//
// Member m owns the KT = 8·KL topics [m·KT, m·KT + KT) of every row (config 4: P = 5 members of 104
// topics).  Its eight waves hold the rows n = 64·j + 8·w + rl of row set j < R (R = ⌈nnz/64⌉ ≤ 7); inside a
// wave lane = tl + 8·rl and topic lane tl holds the member's topics [KL·tl, KL·tl + KL) of its R rows:
// KL·R doubles per lane (six row sets in VGPRs, a seventh in LDS).  Per inner iteration:
//   φ_n = B_n·eθ : KL lane-local FMAs per row, the eight topic lanes' partials summed by worker lane q
//     (one per wave row) in a fixed order → the member's partial of φ_n;
//   exchange     : every member publishes its nnz partials (and its Σ|Δγ| partial) as epoch granules and
//     sums the P partials of its rows in member order, so φ, r = cts/φ, the ψ(Σγ') identity and the stop
//     rule are bit-identical in every member and the team leaves the loop together;
//   s = Bᵀr      : R lane-local FMAs per topic, the eight row lanes' partials reduce-scattered inside the
//     wave, eight partials per topic (one per wave) to LDS, one block barrier;
//   ψ phase      : four waves (one per SIMD, alternating wave sets by iteration parity) add a topic's 8
//     partials, update γ and eθ = exp(ψ(γ) − ψ(Σγ') − ψc) for their KT/4 topics, second barrier.
// Against k_estep_wide_mc (the rows split: one topic per lane, every row's φ a 512-lane reduction, the
// s partials of all k topics exchanged, ψ of all k topics in every member, registers spilled in the loop)
// a member's block is KT columns × nnz rows in registers, φ needs an eight-lane sum, the exchange carries
// nnz + 1 values, and each member evaluates ψ for its own KT topics only.
// Numerics as lda_rows64.hip: Bp row-scaled by e^{-m_v}, Spark's 1e-100 carried as ε'_n = 1e-100·e^{-m_v};
// the ψ/exp chain is psi64.h's.  Persistent grid, granules, bounded spins: as k_estep_wide_mc.
#include "estep_common.h"
#include "psi64.h"
#include "team_exchange.h"

namespace stc {
namespace lda {

namespace {

constexpr int kTW = 8;                  // waves per member (one 512-thread workgroup per CU)
constexpr int kTThreads = 64 * kTW;
constexpr int kTSets = 7;               // row sets of 64 rows (8 waves × 8 row lanes): nnz ≤ 448
constexpr int kTReg = 6;                // row sets in VGPRs (the seventh in LDS)
constexpr int kTKL = 13;                // topics per topic lane: KT = 104 per member
constexpr int kTPaPitch = 10;           // φ-partial row pitch (doubles): conflict-free 16-B worker reads
constexpr int kTSbPitch = 10;           // s-partial row pitch (doubles): one per wave + pad, 16-B aligned rows
constexpr int kTSlotD = 64 * kTSets;    // granule slot of a member's Σ|Δγ| partial (rows: [0, nnz))
constexpr int kTSlotG = kTSlotD + 1;    // … of its final Σγ partial
constexpr int kTXStride = kTSlotG + 1;  // granules per member and parity
constexpr int kTMaxP = 8;               // members at most (k ≤ 832)
#ifndef TG_MIRROR
#define TG_MIRROR 1  // the ψ wave's Σ|Δγ| reduction moved to the idle wave of its topic set (0: on the ψ wave)
#endif
// s_sleep units (64 cycles) between the exchange's poll rounds (config 4, 8-step A/B: 1 → E-step 147.5 ms,
// 3 → 148.8 ms)
constexpr int kTPollSleep = 1;
#ifndef TG_LOAD_BATCH
#define TG_LOAD_BATCH 2                 // row sets whose block loads are in flight together
#endif

template <int KL>
struct TLds {
  static constexpr int KT = 8 * KL;
  static constexpr int KLP = (KL + 1) / 2 * 2;
  double eth[8][KLP] __attribute__((aligned(16)));  // the member's eθ: topic t at [t / KL][t % KL]
  double gam[KT];                                   // the member's γ
  double apc[KT][2] __attribute__((aligned(16)));   // α_t, ψc_t of the member's topics
  double rrow[kTW][8 * kTSets];                     // r = cts/φ per (wave, worker row)
  int rid[kTW][8 * kTSets];                         // term id per (wave, worker row): the entry outputs
  double esum[kTW] __attribute__((aligned(16)));    // Σ r·ε' over a wave's rows (0 unless an ε' is visible)
  double dpart[4];                                  // Σ|Δγ| per ψ wave of the last update
  double part[kTW][4];                              // per-wave sums (init: Σγ₀, Σα, Σcts; end: Σγ)
  double ac[4];                                     // Σα, Σcts, ψ(Σα + Σcts) (the flat ψ(Σγ')), ψ(Σγ) at the end
  union {
    struct {
      double pa[kTW][8 * kTSets][kTPaPitch];        // φ partials (wave, worker row, topic lane)
      double sb[KT][kTSbPitch];                     // s partials (topic, wave): each wave's eight row lanes summed
    } l;
    double stage[kTW][8][KT + 2];                   // block loads: eight rows per wave at a time
  } u __attribute__((aligned(16)));
  double ovf[kTW][KL][64];                          // row set kTReg (read back only by its own lane)
};

// per-document per-lane state, set by tg_open and read by the R-specialised loop and tg_close
struct TDoc {
  int64_t slot, row, mem, s0, e0;
  int nnz, rsets;
  bool wv;     // worker lane with a document row
  int qn, qid;  // worker: its row, term id, count, m_v, 2^53·ε'
  double qc, qls, qe2;
};

struct TTeam {
  int P, member, m0;        // members, this member, its first topic
  int lane, w, tl, rl;
  int tt, ttl, ttp;         // ψ-lane topic map (member-local topic tt, held by lane tt % PSIL of wave tt / PSIL)
  bool tval, town;          // an eθ slot of the member (pad columns included); a real topic
  bool pub_ok;              // debug (STC_TEAM_FAULT): false for the member that never publishes
  __amdgpu_buffer_rsrc_t rs;  // the team's granules
  int xstride;
  unsigned* tmo;
  unsigned spin_limit;
};

// the P partials of granule slot `idx` summed in member order (this member contributes `mine`); a lane
// with need = false reads nothing.  A wave whose partners never publish gives up (bounded spin): it sets
// the timeout word and s_abort, and its sums are garbage (the caller leaves at the next barrier).
__device__ __forceinline__ double team_sum(const TTeam& t, unsigned epoch, int idx, double mine, bool need, int* s_abort) {
  const int base = (int)(epoch & 1) * t.P * t.xstride;
  double sum = 0.0;
  for (int m = 0; m < t.P; ++m) {
    double v = 0.0;
    if (m == t.member) {
      v = mine;
    } else {
      for (unsigned spins = 0;; ++spins) {
        const bool ok = !need || get_granule<double>(t.rs, base + m * t.xstride + idx, epoch, v);
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spin_give_up(spins, t.tmo, t.spin_limit)) {
          *s_abort = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    sum += need ? v : 0.0;
  }
  return sum;
}

// worker lanes, γ₀ / α / ψc of the member's topics, Σγ₀ / Σα over all k topics, Σcts, the first eθ;
// false (outputs written) for a document without a nonzero count
template <int KL, bool STATS>
__device__ __forceinline__ bool tg_open(const EStepArgs<double>& a, TLds<KL>& sm, const TTeam& t, TDoc& d) {
  constexpr int KLP = TLds<KL>::KLP;
  const int tid = (int)threadIdx.x, lane = t.lane, w = t.w;
  const int k = a.k;
  // ---- worker lane q = lane: wave row q → document row qn = 64·(q >> 3) + 8·w + (q & 7)
  d.qn = 64 * (lane >> 3) + 8 * w + (lane & 7);
  d.wv = lane < 8 * d.rsets && d.qn < d.nnz;
  const int64_t qe = d.wv ? d.s0 + d.qn : 0;
  d.qid = d.wv ? a.indices[qe] : 0;
  d.qc = d.wv ? a.values[qe] : 0.0;
  d.qls = a.logscale[d.qid];
  d.qe2 = d.wv ? fmin(0x1p53 * exp(kLogEps - d.qls), 1e300) : -0x1p53;  // padding rows: φ = −1, r = −0

  // ---- γ₀ of ALL k topics for Σγ₀ (every member alike), Σα, Σcts
  uint64_t stream = 0;
  if (!a.gamma0) {
    const uint64_t key = a.key_mode == 0 ? train_doc_key(a.iteration, a.rank, d.mem) : (uint64_t)(a.doc_id_base + d.row);
    stream = doc_stream(a.seed, key);
  }
  double gs = 0.0, as = 0.0;
  for (int tg = tid; tg < k; tg += kTThreads) {
    gs += a.gamma0 ? a.gamma0[d.mem * k + tg] : gamma_sample(stream, tg, a.gamma_shape);
    as += a.alpha[tg];
  }
  // the member's own topics (ψ lanes: both wave sets hold the same map; set 0 initialises the LDS)
  double g0 = 0.0, pc = 0.0;
  if (w < 4 && t.town) {
    const int tg = t.m0 + t.tt;
    g0 = a.gamma0 ? a.gamma0[d.mem * k + tg] : gamma_sample(stream, tg, a.gamma_shape);
    pc = a.psic[tg];
    sm.apc[t.tt][0] = a.alpha[tg];
    sm.apc[t.tt][1] = pc;
  }
  if (w < 4 && t.tval) sm.gam[t.tt] = g0;
  for (int i = tid; i < 8 * KLP; i += kTThreads) (&sm.eth[0][0])[i] = 0.0;
  {
    const double gsw = wave_sum_d(gs), asw = wave_sum_d(as), cw = wave_sum_d(d.qc);
    if (lane == 0) {
      sm.part[w][0] = gsw;
      sm.part[w][1] = asw;
      sm.part[w][2] = cw;
    }
  }
  const bool nonempty = __syncthreads_or(d.wv && d.qc != 0.0) != 0;
  double gsum0 = 0.0, asum = 0.0, ctot = 0.0;
#pragma unroll
  for (int v = 0; v < kTW; ++v) {  // fixed order: identical in every member
    gsum0 += sm.part[v][0];
    asum += sm.part[v][1];
    ctot += sm.part[v][2];
  }
  if (tid == 0) {
    sm.ac[0] = asum;
    sm.ac[1] = ctot;
    sm.ac[2] = digamma_fast_d(asum + ctot);
  }
  if (!nonempty) {
    if (w < 4 && t.town) {
      const int tg = t.m0 + t.tt;
      if (a.gamma) a.gamma[d.mem * k + tg] = 0.0;
      if (STATS) a.elogth[d.slot * k + tg] = 0.0;
    }
    if (STATS && w < 4 && t.tval) a.eth[d.slot * a.kp + t.m0 + t.tt] = 0.0;
    if (t.member == 0) {
      for (int n = tid; n < d.nnz; n += kTThreads) {
        a.r[d.e0 + n] = 0.0;
        if (STATS) {
          a.keys[d.e0 + n] = (uint32_t)a.indices[d.s0 + n];
          a.vals[d.e0 + n] = entry_val<double>(d.slot, d.e0 + n, 0.0);
        }
      }
      if (tid == 0) {
        if (a.iters) a.iters[d.mem] = 0;
        if (a.nonempty) a.nonempty[d.mem] = 0;
      }
    }
    return false;
  }
  // eθ' = exp(ψ(γ) − ψ(Σγ) − ψc_t) of the member's topics
  const double cs0 = digamma_fast_d(gsum0);
  if (w < 4 && t.town) sm.eth[t.ttl][t.ttp] = exp_digamma_minus_v2<2>(g0, cs0 + pc);
  return true;  // (the block loads' barrier publishes eθ, γ, α/ψc)
}

// the block (R row sets of the member's KT columns) and the fixed point; returns the iteration count
// (−1: the team timed out); the final r sits in sm.rrow
template <int KL, int R>
__device__ __forceinline__ int tg_iterate(const EStepArgs<double>& a, TLds<KL>& sm, const TTeam& t, const TDoc& d,
                                          unsigned& epoch, int* s_abort) {
  constexpr int KT = TLds<KL>::KT, KLP = TLds<KL>::KLP;
  constexpr int RG = R < kTReg ? R : kTReg;  // row sets in VGPRs; [RG, R) in sm.ovf
  static_assert(R >= 1 && R <= kTSets && R - RG <= 1, "row sets");
  STAMP_DECL
  // the lane index laundered per document: every lane-derived index below (the block loads' piece
  // offsets and worker-lane permutes, the LDS addresses) is then computed per document instead of being
  // hoisted out of the persistent document loop and held — spilled — across every fixed point
  int lane = t.lane;
  asm volatile("" : "+v"(lane));
  const int w = t.w, tl = lane & 7, rl = lane >> 3;
  const int kp = a.kp, nnz = d.nnz, m0 = t.m0;
  const int qn = d.qn;
  const bool wv = d.wv;
  const double qc = d.qc, qe2 = d.qe2;

  // ---- B, coalesced: per row set the wave copies its eight rows' KT member columns with 16-byte loads,
  // stages them in LDS and every lane picks up its (row lane, topic lane) part
  double B[RG][KL];
  double* const ovf = &sm.ovf[w][0][lane];  // set RG at ovf[64·p]
#define BV(j, p) ((j) < RG ? B[(j) < RG ? (j) : 0][p] : ovf[64 * (p)])
  {
    constexpr int C2 = KT / 2;                 // double2 pieces per member row
    constexpr int NP = (8 * C2 + 63) / 64;     // pieces per lane per row set
    const int c2v = (kp - m0) < KT ? (kp - m0) / 2 : C2;  // pieces inside the matrix (the last member's tail is 0)
    double* const stg = &sm.u.stage[w][0][0];
    constexpr int SP = KT + 2;
#pragma unroll
    for (int j0 = 0; j0 < R; j0 += TG_LOAD_BATCH) {
      // TG_LOAD_BATCH row sets' loads in flight together; the scheduling barriers keep the compiler from
      // hoisting every set's loads to the top (all in flight at once they took 168 VGPRs and spilled B)
      __builtin_amdgcn_sched_barrier(0);
      double2 pcs[TG_LOAD_BATCH][NP];
#pragma unroll
      for (int jj = 0; jj < TG_LOAD_BATCH; ++jj) {
        const int j = j0 + jj;
        if (j >= R) break;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int c = lane + 64 * i;
          const int srow = c / C2, q = c - srow * C2;
          const int id = __builtin_amdgcn_ds_bpermute((8 * j + (srow & 7)) << 2, d.qid);  // its worker lane
          const bool keep = c < 8 * C2 && q < c2v && 64 * j + 8 * w + srow < nnz;
          const double2 x = *reinterpret_cast<const double2*>(a.Bp + (int64_t)(keep ? id : 0) * kp + (keep ? m0 + 2 * q : 0));
          pcs[jj][i] = keep ? x : make_double2(0.0, 0.0);
        }
      }
#pragma unroll
      for (int jj = 0; jj < TG_LOAD_BATCH; ++jj) {
        const int j = j0 + jj;
        if (j >= R) break;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int c = lane + 64 * i;
          const int srow = c / C2, q = c - srow * C2;
          if (c < 8 * C2) *reinterpret_cast<double2*>(stg + srow * SP + 2 * q) = pcs[jj][i];
        }
        __builtin_amdgcn_wave_barrier();  // one wave writes and reads its stage; LDS is in order per wave
#pragma unroll
        for (int p = 0; p < KL; ++p) {
          const double v = stg[rl * SP + KL * tl + p];
          if (j < RG) B[j < RG ? j : 0][p] = v;
          else ovf[64 * p] = v;
        }
        __builtin_amdgcn_wave_barrier();
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();  // the staging area is the loop's partial arrays; (also publishes the first eθ, γ, α/ψc)
  STAMP(0);  // block loads and their barrier
  // mirror mode (as lda_rows64.hip): waves w and w ^ 4 share a topic set and take turns as its ψ wave and
  // as its Σ|Δγ| wave; each keeps γ / eθ of its lane's topic as it last computed them
  double gm = 0.0, em = 0.0;
  if (TG_MIRROR && t.town) {
    gm = sm.gam[t.tt];
    em = sm.eth[t.ttl][t.ttp];
  }

  double* const pa = &sm.u.l.pa[w][0][0];
  double* const sb = &sm.u.l.sb[0][0];
  double rr[R];
  double qr = 0.0;
  double dmine = 0.0;  // this member's Σ|Δγ| partial of the last update (0 before the first)
  int it = 0;
  while (true) {
    // Phase A: the member's φ partials over the lane's KL topics; worker lane q adds the eight topic
    // lanes' partials in a fixed order
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
      for (int j = 0; j < R; ++j) pa[(8 * j + rl) * kTPaPitch + tl] = acc[j];
    }
    __builtin_amdgcn_wave_barrier();
    double part = 0.0;
    if (lane < 8 * R) {
      const double2* const pr = reinterpret_cast<const double2*>(pa + lane * kTPaPitch);
      const double2 x0 = pr[0], x1 = pr[1], x2 = pr[2], x3 = pr[3];
      part = ((x0.x + x0.y) + (x1.x + x1.y)) + ((x2.x + x2.y) + (x3.x + x3.y));
    }
    STAMP(1);  // eθ reads, φ FMAs, partial stores, worker sums
    // ---- exchange: the member's φ partials and Σ|Δγ| partial out, the team's sums in member order
    ++epoch;
    {
      const int base = (int)(epoch & 1) * t.P * t.xstride + t.member * t.xstride;
      if (t.pub_ok && wv) put_granule<double>(t.rs, base + qn, epoch, part);
      if (t.pub_ok && threadIdx.x == 0) put_granule<double>(t.rs, base + kTSlotD, epoch, dmine);
    }
    // every partner's row partial and Σ|Δγ| partial requested together (one L2 round trip per poll, not
    // one per member and value), then summed in member order
    double phi = 0.0, dsum = 0.0;
    {
      const int base = (int)(epoch & 1) * t.P * t.xstride;
      // rows: each worker lane polls its row's granule of every partner; the Σ|Δγ| granules: lane m polls
      // partner m's only and the wave takes the values by readlane (every lane polling every partner's D
      // granule was most of the poll traffic queued at this CU — the hand-off's price, MI355X_MICROARCH.md
      // handoff-1to1 — for values that are the same in every lane)
      // A granule already received is not requested again (got: one bit per partner, and bit kTMaxP for the
      // lane's D granule): every poll round re-requesting the partners that had arrived kept the queue full.
      double vr[kTMaxP], vdl = 0.0;
      const bool dl = lane < t.P && lane != t.member;
      unsigned need = dl ? 1u << kTMaxP : 0u;
#pragma unroll
      for (int m = 0; m < kTMaxP; ++m) {
        vr[m] = 0.0;
        if (m < t.P && m != t.member && wv) need |= 1u << m;
      }
      for (unsigned spins = 0;; ++spins) {
#pragma unroll
        for (int m = 0; m < kTMaxP; ++m)
          if (need & (1u << m)) {
            if (get_granule<double>(t.rs, base + m * t.xstride + qn, epoch, vr[m])) need &= ~(1u << m);
          }
        if (need & (1u << kTMaxP)) {
          if (get_granule<double>(t.rs, base + lane * t.xstride + kTSlotD, epoch, vdl)) need &= ~(1u << kTMaxP);
        }
        if (__builtin_amdgcn_ballot_w64(need != 0) == 0) break;
        if (spin_give_up(spins, t.tmo, t.spin_limit)) {
          *s_abort = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(kTPollSleep);
      }
#pragma unroll
      for (int m = 0; m < kTMaxP; ++m) {
        if (m < t.P) {
          phi += m == t.member ? part : vr[m];
          dsum += m == t.member ? dmine : readlane_t(vdl, m);
        }
      }
      if (!wv) phi = 0.0;
    }
    STAMP(2);  // exchange: publish, poll, member-order sums
    bool live = false;
    if (lane < 8 * R) {
      const double ph = fma(qe2, 0x1p-53, phi);
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
    // Spark: while (meanGammaChange > 1e-3); dsum is identical in every wave of every member unless a
    // wave timed out, which every wave sees after the barrier below
    const bool stop = (it > 0 && dsum <= a.stop_thr) || it >= a.max_iter;
    STAMP(3);  // r, ε' ballot, r reads

    // Phase B: s partials over the lane's R rows, summed over the wave's eight row lanes by a
    // reduce-scatter (lane bits 5, 4, 3: permlane32 / permlane16 swaps, then row_ror:8), so each lane
    // stores two topics' wave sums and a ψ lane reads eight partials (one per wave) instead of 64
    if (!stop) {
      static_assert(KL == 13, "the reduce-scatter below is laid out for 13 topics per topic lane");
      double x[14];
#pragma unroll
      for (int p = 0; p < KL; ++p) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < R; ++j) acc = fma(BV(j, p), rr[j], acc);
        x[p] = acc;
      }
      x[13] = 0.0;
      double a7[7], b4[4];
      swap_add_nd<true, 7>(x, x + 7, a7);           // bit 5: p [0, 7) | [7, 14)
      const double a8[8] = {a7[0], a7[1], a7[2], a7[3], a7[4], a7[5], a7[6], 0.0};
      swap_add_nd<false, 4>(a8, a8 + 4, b4);        // bit 4: entries [0, 4) | [4, 8)
      const bool h3 = (lane & 8) != 0;
      const double c0 = rs_dpp_d<DPP_ROW_ROR8>(b4[0], b4[2], h3);  // bit 3: entries {0, 1} | {2, 3}
      const double c1 = rs_dpp_d<DPP_ROW_ROR8>(b4[1], b4[3], h3);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int jb = ((lane & 16) ? 4 : 0) + (h3 ? 2 : 0) + i;  // entry of the bit-5 list
        const int p = ((lane & 32) ? 7 : 0) + jb;
        if (jb < 7 && p < KL) sb[(KL * tl + p) * kTSbPitch + w] = i == 0 ? c0 : c1;
      }
    }
    STAMP(4);  // s FMAs + partial stores
    __syncthreads();  // (1) s partials, esum and any give-up published
    STAMP(5);  // barrier 1
    if (*s_abort) return -1;
    if (stop) break;
    const bool psi = (w >> 2) == (it & 1);
    if (psi) {
      __builtin_amdgcn_s_setprio(3);
      double dg = 0.0;
      if (t.town) {
        const double2* const sp = reinterpret_cast<const double2*>(sb + t.tt * kTSbPitch);
        const double2 x0 = sp[0], x1 = sp[1], x2 = sp[2], x3 = sp[3];  // the eight waves' sums, fixed order
        const double s = ((x0.x + x0.y) + (x1.x + x1.y)) + ((x2.x + x2.y) + (x3.x + x3.y));
        const double g = TG_MIRROR ? gm : sm.gam[t.tt], eo = sm.eth[t.ttl][t.ttp];
        const double2 ap = *reinterpret_cast<const double2*>(&sm.apc[t.tt][0]);  // α_t, ψc_t
        const double2 e01 = *reinterpret_cast<const double2*>(&sm.esum[0]);
        const double2 e23 = *reinterpret_cast<const double2*>(&sm.esum[2]);
        const double2 e45 = *reinterpret_cast<const double2*>(&sm.esum[4]);
        const double2 e67 = *reinterpret_cast<const double2*>(&sm.esum[6]);
        const double et = ((e01.x + e01.y) + (e23.x + e23.y)) + ((e45.x + e45.y) + (e67.x + e67.y));
        const double csn = et != 0.0 ? digamma_fast_d(sm.ac[0] + sm.ac[1] - et) : sm.ac[2];
        const double gn = fma(eo, s, ap.x);  // γ ← eθ ⊙ s + α
        dg = fabs(gn - g);
        sm.gam[t.tt] = gn;
        const double en = exp_digamma_minus_v2<2>(gn, csn + ap.y);
        sm.eth[t.ttl][t.ttp] = en;
        gm = gn;
        em = en;
      }
      if (!TG_MIRROR) {
        const double dw = wave_sum_d(dg);
        if (lane == 0) sm.dpart[w & 3] = dw;
      }
      __builtin_amdgcn_s_setprio(0);
    } else if (TG_MIRROR) {
      // the topic set's other wave: the same γ update from its own γ / eθ registers (bitwise the ψ wave's:
      // same partials, same order) and Σ|Δγ|, off the ψ chain
      double dg = 0.0;
      if (t.town) {
        const double2* const sp = reinterpret_cast<const double2*>(sb + t.tt * kTSbPitch);
        const double2 x0 = sp[0], x1 = sp[1], x2 = sp[2], x3 = sp[3];
        const double s = ((x0.x + x0.y) + (x1.x + x1.y)) + ((x2.x + x2.y) + (x3.x + x3.y));
        const double gn = fma(em, s, sm.apc[t.tt][0]);
        dg = fabs(gn - gm);
        gm = gn;  // (its eθ: the ψ wave's, from LDS, when this wave is next the ψ wave)
      }
      const double dw = wave_sum_d(dg);
      if (lane == 0) sm.dpart[w & 3] = dw;
    }
    STAMP(psi ? 6 : 8);  // ψ phase (ψ waves; the others: nothing)
    __syncthreads();  // (2) eθ, γ, Σ|Δγ| partials published
    STAMP(psi ? 7 : 9);  // barrier 2 (ψ waves / the others)
    dmine = (sm.dpart[0] + sm.dpart[1]) + (sm.dpart[2] + sm.dpart[3]);
    ++it;
  }
#undef BV
  STAMP_FLUSH
  return it;
}

// outputs: the team's exact Σγ (one more exchange), γ, E[log θ], eθ of the member's topics; member 0: the
// entries' r / keys / vals, the iteration count.  false: the team timed out
template <int KL, bool STATS>
__device__ __forceinline__ bool tg_close(const EStepArgs<double>& a, TLds<KL>& sm, const TTeam& t, const TDoc& d, int it,
                                         unsigned& epoch, int* s_abort) {
  constexpr int KT = TLds<KL>::KT;
  const int tid = (int)threadIdx.x, lane = t.lane, w = t.w;
  const int k = a.k;
  if (d.wv) sm.rid[w][lane] = d.qid;  // (rrow holds the final r since the last worker phase)
  // the member's Σγ over its topics in a fixed order (wave 0), then the team's in member order
  ++epoch;
  if (w == 0) {
    double gp = 0.0;
    for (int i = lane; i < KT; i += 64)
      if (t.m0 + i < k) gp += sm.gam[i];
    gp = wave_sum_d(gp);
    if (t.pub_ok && lane == 0) {
      const int base = (int)(epoch & 1) * t.P * t.xstride + t.member * t.xstride;
      put_granule<double>(t.rs, base + kTSlotG, epoch, gp);
    }
    const double gsum = team_sum(t, epoch, kTSlotG, gp, true, s_abort);
    if (lane == 0) sm.ac[3] = digamma_t<double>(gsum);
  }
  __syncthreads();
  if (*s_abort) return false;
  const double psisum = sm.ac[3];
  if (w < 4) {
    const int tg = t.m0 + t.tt;
    if (t.town) {
      const double gfin = sm.gam[t.tt];
      if (a.gamma) a.gamma[d.mem * k + tg] = gfin;
      if (STATS) a.elogth[d.slot * k + tg] = digamma_t<double>(gfin) - psisum;
    }
    if (STATS && t.tval) a.eth[d.slot * a.kp + tg] = sm.eth[t.ttl][t.ttp];  // the eθ the final φ used
  }
  if (t.member == 0) {
    // entry outputs in row order, consecutive threads on consecutive entries (row n = 64·set + 8·wave + row lane)
    for (int n = tid; n < d.nnz; n += kTThreads) {
      const int ws = (n >> 3) & 7, q = 8 * (n >> 6) + (n & 7);
      const double rv = sm.rrow[ws][q];
      a.r[d.e0 + n] = rv;
      if (STATS) {
        a.keys[d.e0 + n] = (uint32_t)sm.rid[ws][q];
        a.vals[d.e0 + n] = entry_val<double>(d.slot, d.e0 + n, rv);
      }
    }
    if (tid == 0) {
      if (a.iters) a.iters[d.mem] = it;
      if (a.nonempty) a.nonempty[d.mem] = 1;
    }
  }
  return true;
}

// Persistent grid of G = 8·P·⌊CUs/(8P)⌋ blocks; team members share blockIdx % 8 (one XCD: the granule
// lines stay in its L2); team t takes slots t, t + T, ….  Every document of the launch has ≤ 64·kTSets rows
// (the host routes longer ones elsewhere).
template <int KL, bool STATS>
__global__ __launch_bounds__(kTThreads, 1) void k_estep_tgrid64(EStepArgs<double> a, WideTeam wt) {
  __shared__ TLds<KL> sm;
  __shared__ int s_abort;
  constexpr int KT = TLds<KL>::KT;
  TTeam t;
  t.P = wt.P;
  const int b = (int)blockIdx.x, il = b / 8;
  t.member = il % t.P;
  const int team = (il / t.P) * 8 + (b % 8), nteams = (int)gridDim.x / t.P;
  t.m0 = t.member * KT;
  t.lane = threadIdx.x & 63;
  t.w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);  // wave-uniform: scalar role tests
  t.tl = t.lane & 7;
  t.rl = t.lane >> 3;
  constexpr int PSIL = (KT + 3) / 4;
  t.tt = (t.w & 3) * PSIL + t.lane;
  t.tval = t.lane < PSIL && t.tt < KT && t.m0 + t.tt < a.kp;
  t.town = t.lane < PSIL && t.tt < KT && t.m0 + t.tt < a.k;
  t.ttl = t.tt / KL;
  t.ttp = t.tt - t.ttl * KL;
  if (t.tt >= KT) {  // lanes past the member's topics: a harmless in-bounds map
    t.ttl = 0;
    t.ttp = 0;
  }
  t.pub_ok = !(team == 0 && t.member == wt.fault_member);
  t.xstride = (int)wt.xstride;
  const int team_granules = 2 * t.P * t.xstride;
  unsigned char* const xb = reinterpret_cast<unsigned char*>(wt.xbuf) + (int64_t)team * team_granules * 16;
  t.rs = __builtin_amdgcn_make_buffer_rsrc(xb, 0, team_granules * 16, 0x00020000);
  t.tmo = wt.tmo;
  t.spin_limit = wt.spin_limit;
  if (threadIdx.x == 0) s_abort = 0;
  unsigned epoch = 0;
  for (int64_t j = team; j < a.n; j += nteams) {
    TDoc d;
    d.slot = a.slot0 + j;
    d.row = a.batch ? (int64_t)a.batch[d.slot] : d.slot;
    d.mem = a.orig ? (int64_t)a.orig[d.slot] : d.slot;
    d.s0 = a.indptr[d.row];
    d.nnz = (int)(a.indptr[d.row + 1] - d.s0);
    d.rsets = (d.nnz + 63) >> 6;
    d.e0 = a.bptr ? a.bptr[d.slot] : d.s0;
    if (tg_open<KL, STATS>(a, sm, t, d)) {
      int it;
      switch (d.rsets) {
        case 1: it = tg_iterate<KL, 1>(a, sm, t, d, epoch, &s_abort); break;
        case 2: it = tg_iterate<KL, 2>(a, sm, t, d, epoch, &s_abort); break;
        case 3: it = tg_iterate<KL, 3>(a, sm, t, d, epoch, &s_abort); break;
        case 4: it = tg_iterate<KL, 4>(a, sm, t, d, epoch, &s_abort); break;
        case 5: it = tg_iterate<KL, 5>(a, sm, t, d, epoch, &s_abort); break;
        case 6: it = tg_iterate<KL, 6>(a, sm, t, d, epoch, &s_abort); break;
        default: it = tg_iterate<KL, 7>(a, sm, t, d, epoch, &s_abort); break;
      }
      if (it < 0) return;  // a team timed out: every block leaves (the host re-runs the one-CU kernel)
      if (!tg_close<KL, STATS>(a, sm, t, d, it, epoch, &s_abort)) return;
    }
    __syncthreads();  // LDS is the next document's
  }
}

}  // namespace

STC_STAMP_READER(stc_debug_stamps_team64)

int tgrid64_row_cap() { return 64 * kTSets; }
int tgrid64_members(int kp) { return (kp + 8 * kTKL - 1) / (8 * kTKL); }
int64_t tgrid64_xstride() { return kTXStride; }

// false: the grid could not be resident at once (nothing launched; the caller runs another kernel)
bool launch_estep_tgrid64(hipStream_t s, const EStepArgs<double>& a, bool stats, const WideTeam& wt) {
  if (a.n == 0) return true;
  if (wt.P != tgrid64_members(a.kp) || wt.xstride < kTXStride)
    throw Error(STC_ERR_INVALID_ARG, "fp64 team-grid E-step: members / granule stride do not match k");
  auto go = [&](const void* kern) {
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kTThreads, 0));
    if ((int64_t)per_cu * cus < wt.blocks) return false;
    EStepArgs<double> aa = a;
    WideTeam ww = wt;
    void* args[] = {&aa, &ww};
    HIP_CHECK(hipLaunchKernel(kern, dim3((unsigned)wt.blocks), dim3(kTThreads), args, 0, s));
    return true;
  };
  return stats ? go((const void*)k_estep_tgrid64<kTKL, true>) : go((const void*)k_estep_tgrid64<kTKL, false>);
}

}  // namespace lda
}  // namespace stc
