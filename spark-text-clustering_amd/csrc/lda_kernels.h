// lda_kernels.h — host-side launch API of the online-LDA kernels (lda.hip).
#pragma once

#include <cmath>

#include "stc_internal.h"

namespace stc {
namespace lda {

constexpr int kBlock = 256;           // threads per E-step workgroup (4 waves of 64)
constexpr int kLdsBudget = 80 * 1024; // dynamic LDS per E-step workgroup → 2 workgroups / CU
constexpr int kChunk = 256;           // sorted entries per wave in the sstats segmented SpMM
constexpr int kRowsPerBlock = 64;     // terms per workgroup in the λ update

// An entry's sort value for the term-sorted sstats SpMM: its member slot in the high word and, in
// the low word, r itself for fp32 (so the SpMM reads (slot, r) with the sorted keys instead of
// gathering them per entry) or the entry index for fp64 (r is gathered from r[e]).
template <typename T>
__device__ __forceinline__ uint64_t entry_val(int64_t slot, int64_t e, T r) {
  if constexpr (sizeof(T) == 4)
    return ((uint64_t)(uint32_t)slot << 32) | __builtin_bit_cast(uint32_t, r);
  else
    return ((uint64_t)(uint32_t)slot << 32) | (uint32_t)e;
}

// Everything the E-step kernel reads/writes.  T = the E-step arithmetic type (float/double).
template <typename T>
struct EStepArgs {
  int k = 0, kp = 0, P = 0;            // topics, global row pitch of Bp, LDS row pitch
  int lds_rows = 0;                    // docs with nnz <= lds_rows keep their block in LDS
  const int64_t* indptr = nullptr;     // documents (CSR rows)
  const int32_t* indices = nullptr;
  const T* values = nullptr;
  // A launch covers slots [slot0, slot0 + n).  slot → row via `batch` (nullptr: row = slot);
  // slot → caller's member index via `orig` (nullptr: member = slot) — γ₀, γ, iters, nonempty,
  // bound and the RNG key are per MEMBER; eth / elogth / entry slots are per SLOT.
  const int32_t* batch = nullptr;
  const int32_t* orig = nullptr;
  int64_t slot0 = 0;
  int64_t n = 0;                       // slots in this launch
  const int64_t* bptr = nullptr;       // slot → first entry slot (nullptr: the row's CSR offset)
  // per CSR entry: the in-row position of the row's n-th E-step row (lda_wide.hip: the corpus's
  // rarest terms first, so the register / LDS rows are the cold ones and the streamed rows the hot
  // ones the MALL holds for every CU); nullptr: CSR order
  const int32_t* order = nullptr;
  const T* Bp = nullptr;               // V×kp  row-scaled expElogβ': exp(ψ(λ_vt) − m_v)
  const double* psic = nullptr;        // 2k    ψ(Σ_v λ_vt), then exp(−ψ(Σ_v λ_vt)): eθ' = exp(ψ(γ_t) − ψ(Σγ) − psic_t)
  const double* logscale = nullptr;    // V     m_v (BOUND)
  const double* alpha = nullptr;       // k
  const T* gamma0 = nullptr;           // n×k or nullptr (counter RNG)
  uint64_t seed = 0;
  int64_t iteration = 0;
  int rank = 0;
  int key_mode = 0;                    // 0: train_doc_key(iteration, rank, i); 1: doc_id_base + row
  int64_t doc_id_base = 0;
  double gamma_shape = 100.0;
  int max_iter = 100000;
  // Spark's stop rule Σ|Δγ|/k ≤ 1e-3 as one comparison: the largest double T with fl(T / k) ≤ 1e-3
  // (fl(x / k) is monotone in x, so x ≤ T ⇔ fl(x / k) ≤ 1e-3 exactly; stop_threshold() below)
  double stop_thr = 0.0;
  // outputs
  T* gamma = nullptr;                  // n×k (optional)
  T* eth = nullptr;                    // n×kp scaled exp(E[log θ]) (STATS)
  T* elogth = nullptr;                 // n×k  E[log θ] (STATS: logphat)
  T* r = nullptr;                      // entry slots: cts/φ' (always)
  uint32_t* keys = nullptr;            // entry slots: term id (STATS)
  uint64_t* vals = nullptr;            // entry slots: entry_val(slot, entry, r) (STATS)
  int32_t* iters = nullptr;            // n (optional)
  int32_t* nonempty = nullptr;         // n (optional)
  double* bound = nullptr;             // n (BOUND)
  // fp64 rows / fp32 grid kernels: scratch for the list of this launch's long documents (capacity n
  // slots + one count word), filled on the device before the long-document launch walks it (last, so
  // the other kernels' argument layout is unchanged)
  int32_t* long_list = nullptr;
};

// the largest double x with fl(x / k) ≤ 1e-3 (host; see EStepArgs::stop_thr)
inline double stop_threshold(int k) {
  const double kd = (double)k;
  double x = 1e-3 * kd;
  while (x / kd > 1e-3) x = std::nextafter(x, 0.0);
  while (std::nextafter(x, INFINITY) / kd <= 1e-3) x = std::nextafter(x, INFINITY);
  return x;
}

template <typename T>
size_t estep_lds_bytes(int kp, int lds_rows, int P);
template <typename T>
int estep_lds_rows(int k, int kp, int P);
template <typename T>
void launch_estep(hipStream_t s, const EStepArgs<T>& a, bool stats, bool bound);

// fp32 row-lane × topic-group grid E-step (lda_grid.hip): k <= 128, nnz <= grid_row_cap(k) (0 if n/a)
int grid_row_cap(int k);
// documents past grid_onchip_rows(k) run in a second, resident launch (`long_docs`; a.long_list set)
int grid_onchip_rows(int k);
void launch_estep_grid(hipStream_t s, const EStepArgs<float>& a, bool stats, bool bound, bool long_docs);
// fp64 rows-split E-step (lda_rows64.hip): k <= 104, nnz <= rows64_row_cap(k) (0 if n/a); documents
// past rows64_onchip_rows(k) run in a second launch (`long_docs`)
int rows64_row_cap(int k);
int rows64_onchip_rows(int k);
void launch_estep_rows64(hipStream_t s, const EStepArgs<double>& a, bool stats, bool bound, bool long_docs);
// many-topic E-step (lda_wide.hip): topics across a 512-thread workgroup, k <= 2048, nnz <= wide_row_cap(k)
int wide_row_cap(int k);
// a team of P CUs per document for the many-topic E-step (lda_wide.hip k_estep_wide_mc)
struct WideTeam {
  int P = 1;                 // workgroups (CUs) per document
  int blocks = 0;            // persistent grid: a multiple of 8·P, ≤ the CU count
  unsigned* tmo = nullptr;   // timeout word (zeroed before each launch)
  void* xbuf = nullptr;      // [teams][2][P][xstride] 16-byte {epoch, value} granules (zeroed before each launch)
  int64_t xstride = 0;       // granules per member: rows split kp + 1 (s partials, Σ r·φ); topics split
                             // 512 + 2 (φ partials, Σ|Δγ|, Σγ)
  unsigned spin_limit = 1u << 22;  // polls before a member gives up (a few seconds)
  int fault_member = -1;     // debug (STC_TEAM_FAULT): this member of team 0 never publishes
  int max_row = -1;          // the launch's longest document (< 0: unknown) — k_estep_wide_tc sizes its
                             // per-row LDS arrays by it, so the rest of the CU's LDS holds block rows
  int xrows = 0;             // (set by the tc launcher) rows of those arrays
};
// after the E-step's logphat: a timed-out team poisons the non-empty count (small[k] = −1e300, negative
// after any all-reduce over ranks), which gates the λ / colsum / expElogβ' / α updates off
template <typename T>
int wide_resident_rows(int k);
// false: the grid could not be resident at once (nothing launched; the caller runs the one-CU kernel)
template <typename T>
bool launch_estep_wide_mc(hipStream_t s, const EStepArgs<T>& a, bool stats, const WideTeam& wt);
// the same with the TOPICS split over the team (k > 512; lda_wide.hip k_estep_wide_tc)
template <typename T>
bool launch_estep_wide_tc(hipStream_t s, const EStepArgs<T>& a, bool stats, const WideTeam& wt);
template <typename T>
void launch_estep_wide(hipStream_t s, const EStepArgs<T>& a, bool stats, bool bound);
// fp64 many-topic team E-step with the TOPICS split over P = tgrid64_members(kp) CUs and the rows64 grid
// inside a member (lda_team64.hip k_estep_tgrid64): nnz ≤ tgrid64_row_cap(); wt.xstride ≥ tgrid64_xstride();
// false: the grid could not be resident at once (nothing launched)
int tgrid64_row_cap();
int tgrid64_members(int kp);
int64_t tgrid64_xstride();
bool launch_estep_tgrid64(hipStream_t s, const EStepArgs<double>& a, bool stats, const WideTeam& wt);

// Batch partition: slots [0, n_short) = members with nnz <= cap (wave kernel), then the rest.
void launch_part_flags(hipStream_t s, const int64_t* indptr, const int32_t* batch, int64_t n,
                       int64_t cap, int64_t* nnz_out, int32_t* short_flag);
void launch_part_scatter(hipStream_t s, const int32_t* batch, const int64_t* nnz, int64_t n,
                         const int32_t* short_flag, const int32_t* short_incl, int32_t* batch_p,
                         int32_t* orig_p, int64_t* nnz_p);

// The multi-GPU stat layout for a reduce-scatter per vocabulary sub-chunk (api.hip train_tail): rank
// r's slice [r·vs, (r+1)·vs) is cut into nsub sub-chunks of vsj rows (the last one the rest), and
// sub-chunk j of every slice is stored together, in rank order, at physical rows [n·j·vsj, …) — so
// sub-chunk j is ONE contiguous reduce-scatter of n pieces.  sub ≥ 0 restricts an sstats launch to the
// terms of sub-chunk j (the entries, their sort order and the chunk grid are the whole launch's, so
// every row's fp64 sum associates exactly as in the single launch); sub < 0: canonical rows, every term.
struct StatMap {
  uint32_t vs = 0, vsj = 0;
  int n = 1, nsub = 1, sub = -1;
};
__host__ __device__ __forceinline__ int stat_sub(const StatMap& m, uint32_t v) {
  const uint32_t j = (v % m.vs) / m.vsj;
  return j < (uint32_t)(m.nsub - 1) ? (int)j : m.nsub - 1;
}
// (rank, sub-chunk) group of a term: the groups are contiguous term ranges, in term order
__host__ __device__ __forceinline__ uint32_t stat_group(const StatMap& m, uint32_t v) {
  return (v / m.vs) * (uint32_t)m.nsub + (uint32_t)stat_sub(m, v);
}
__host__ __device__ __forceinline__ int64_t stat_row(const StatMap& m, uint32_t v) {
  if (m.sub < 0) return (int64_t)v;
  const uint32_t r = v / m.vs, rem = v - r * m.vs;
  const int j = stat_sub(m, v);
  const int64_t w = j < m.nsub - 1 ? (int64_t)m.vsj : (int64_t)m.vs - (int64_t)(m.nsub - 1) * m.vsj;
  return (int64_t)m.n * j * m.vsj + (int64_t)r * w + (rem - (int64_t)j * m.vsj);
}

// stamp (one rank, canonical rows only; may be null): stamp[v] = sid for every row v this launch writes, so
// the M-step can tell this step's rows from stale ones and stat needs no clearing (launch_lambda_eeb)
template <typename T>
void launch_sstats(hipStream_t s, const uint32_t* skeys, const uint64_t* svals, int64_t E,
                   const T* r, const T* eth, int kp, T* stat, T* headbuf, T* tailbuf,
                   const StatMap& map = StatMap{}, int32_t* stamp = nullptr, int32_t sid = 0);

// γ₀ of n slots' members (gamma_sample, keyed as the E-step kernels key it) into out[member·k + t]
template <typename T>
void launch_gamma0(hipStream_t s, const int32_t* batch, const int32_t* orig, int64_t n, int k, uint64_t seed,
                   int64_t iteration, int rank, int key_mode, int64_t doc_id_base, double shape, T* out);

// the fused M-step pass (update = true: λ update; both: expElogβ' rows, logscale, colsum partials)
// Bp64 (STC_MIXED, T = float only; may be null): the same rows in fp64 at the same m_v, for the re-solve.
// stamp (may be null): rows with stamp[v] ≠ sid take stat = 0 without reading stat / Bp (launch_sstats)
template <typename T>
void launch_lambda_eeb(hipStream_t s, bool update, double* lam, const T* stat, T* Bp, double* logscale,
                       int64_t V, int k, int kp, double rho, double scale, double eta, const double* gate,
                       double* colpart, int64_t nblocks, double* Bp64 = nullptr, const int32_t* stamp = nullptr,
                       int32_t sid = 0);
// colsum (block order), psic[0, k) = ψ(colsum), psic[k, 2k) = exp(−ψ(colsum))
void launch_colsum_reduce(hipStream_t s, const double* colpart, int64_t nblocks, int k,
                          const double* gate, double* colsum, double* psic);
template <typename T>
void launch_logphat(hipStream_t s, const T* elogth, const int32_t* nonempty, int64_t n, int k,
                    double* small /* k+1 */, double* part /* kLogphatBlocks × (k+1) scratch */);
constexpr int kLogphatBlocks = 2048;
void launch_update_alpha(hipStream_t s, double* alpha, const double* small, int k, double rho);
void launch_init_lambda(hipStream_t s, double* lam, int64_t V, int k, uint64_t seed, double shape);
template <typename T>
void launch_topics_bound(hipStream_t s, const double* lam, const double* colsum, int64_t V, int k,
                         double eta, double* partials, int64_t nblocks);
void launch_sum_f64(hipStream_t s, const double* x, int64_t n, double* out);
template <typename T>
void launch_sum_vals(hipStream_t s, const T* x, int64_t n, double* out);
void launch_iter_stats(hipStream_t s, const int32_t* iters, const int32_t* nonempty, int64_t n,
                       int max_iter, int64_t* out4 /* sum, max, caphits, nonempty */,
                       int64_t* cum2 /* += Σiters, caphits; may be null */);
void launch_batch_nnz(hipStream_t s, const int64_t* indptr, const int32_t* batch, int64_t n,
                      int64_t* nnz_out);
void launch_sample(hipStream_t s, const int64_t* indptr, int64_t D, double fraction, int with_repl,
                   uint64_t seed, int64_t iteration, int rank, int64_t cap, int32_t* counts,
                   int64_t* weights, int32_t* short_counts);
// writes partitioned slots: batch_p (row), orig_p (raw member position), nnz_p
// out[0..2] = {*a, *b, *c} (the inclusive scans' totals for one readback)
void launch_last3(hipStream_t s, const int32_t* a, const int64_t* b, const int32_t* c, int64_t* out);
void launch_permute_slots(hipStream_t s, const int32_t* idx, int64_t n, const int32_t* batch, const int32_t* orig,
                          const int64_t* nnz, int32_t* batch2, int32_t* orig2, int64_t* nnz2);
void launch_iota(hipStream_t s, int32_t* x, int64_t n);
void launch_entry_pairs(hipStream_t s, const int64_t* indptr, const int32_t* indices, const int32_t* batch,
                        const int64_t* bptr, int64_t n, uint32_t* keys, uint64_t* vals);
void launch_fill_batch(hipStream_t s, const int64_t* indptr, int64_t D, int64_t cap,
                       const int32_t* counts, const int32_t* count_incl,
                       const int32_t* short_incl, int64_t n_short, int32_t* batch_p,
                       int32_t* orig_p, int64_t* nnz_p);
// STC_MIXED (api.hip mixed_resolve): the fp32 E-step's documents past `thr` iterations, listed for the fp64
// re-solve (nnz ≤ cap64 from position 0 up, cnt[0]; the rest from n − 1 down, cnt[1]) ...
void launch_mixed_list(hipStream_t s, const int64_t* indptr, const int32_t* batch, const int32_t* orig,
                       const int64_t* bptr, const int32_t* iters, const int32_t* nonempty, int64_t n, int thr,
                       int64_t cap64, int32_t* lbatch, int32_t* lorig, int64_t* lbptr, int32_t* lslot, int32_t* cnt);
// ... and their fp64 outputs written back into the fp32 step buffers (γ when gamma is given)
void launch_mixed_fixup(hipStream_t s, const int64_t* indptr, const int32_t* lbatch, const int32_t* lorig,
                        const int64_t* lbptr, const int32_t* lslot, int64_t n, int ms, int ml, int k, int kp,
                        const double* eth64, const double* elogth64, const double* r64, const double* gamma64,
                        float* eth, float* elogth, float* r, uint64_t* vals, float* gamma);
void launch_to_f32(hipStream_t s, const double* in, float* out, int64_t n);
void launch_transpose_kv(hipStream_t s, const double* lam, int64_t V, int k, double* out_kv,
                         int32_t* idx_kv);
template <typename T>
void launch_unscale_stat(hipStream_t s, const T* stat, const double* logscale, const double* psic, int64_t V,
                         int k, int kp, double* out_vk);

}  // namespace lda
}  // namespace stc
