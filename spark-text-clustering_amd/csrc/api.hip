// api.hip — the C ABI of libstc.so (include/stc.h): contexts, device CSR, HashingTF/IDF entry
// points, and the online-LDA driver (one submitMiniBatch per stc_lda_step / stc_lda_next).
//
// Host-side control flow mirrors [U] OnlineLDAOptimizer.submitMiniBatch (spark-mllib 2.4.3):
//   iteration += 1 → E-step over the batch (K6) → stat (K sstats) → treeReduce ≙ RCCL all-reduce
//   → batchResult = stat ⊙ expElogβ, updateLambda (K7) → expElogβ (K8) → updateAlpha.
// One host sync per step (to size the sort for the batch's entry count); everything else is
// stream-ordered on the context's HIP stream.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>
#include <type_traits>
#include <unordered_set>

#include "lda_kernels.h"

namespace stc {

static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }

}  // namespace stc

using namespace stc;

struct stc_ctx : Ctx {};

// the contexts that exist (stc_dcsr_free hands a matrix's buffers back only to a live one)
static std::mutex g_live_mu;
static std::unordered_set<stc_ctx*> g_live;
struct stc_dcsr : DCsr {};
struct stc_dtok {
  Ctx* ctx = nullptr;  // the context it was uploaded on; only it may read the buffers
  int device = -1;     // for stc_tokens_free, which may run after that context is gone
  DevBuf utf8, tok_off, doc_off;
  int64_t n_bytes = 0, n_tok = 0, n_docs = 0;
  int64_t max_doc = -1;  // the longest document's token count (from the upload's offsets)
  bool off32 = false;    // tok_off holds u32 offsets (blob + padding < 4 GiB), else int64
};

// ---------------------------------------------------------------------------------------
// LDA state
// ---------------------------------------------------------------------------------------
struct stc_lda {
  Ctx* ctx = nullptr;
  stc_lda_config cfg{};
  int k = 0, kp = 0, P = 0, lds_rows = 0;
  int64_t V = 0;
  int dtype = STC_F32;
  size_t tsize = 4;
  double eta = 0.0;
  int64_t iteration = 0;
  const DCsr* corpus = nullptr;
  int64_t corpus_total = 0;
  bool has_topics = false;
  int64_t nblocks_m = 0;

  DevBuf lam, Bp, logscale, colsum, psic, colpart, alpha, small, scal;
  DevBuf batch_raw, batch, orig, flags, sincl, bptr, bnnz, nnzp, g0, gamma, eth, elogth, iters,
      nonempty, r, keys, vals, skeys, svals, stat, headbuf, tailbuf, sort_tmp, scan_tmp,
      stats4, cum2, bound, dtmp, lpart;
  DevBuf g0gen;  // γ₀ drawn ahead of the E-step (lda::launch_gamma0) when the caller injects none
  // STC_MIXED (dtype reported STC_F32 inside the library; `mixed` set): the fp32 E-step, then the documents past
  // mixed_thr fp32 iterations re-solved in fp64 (mixed_resolve) from Bp64, the fp64 expElogβ' rows the M-step
  // writes beside Bp, and the corpus's fp64 values; vals32 is the fp32 copy the fp32 E-step reads
  bool mixed = false;
  int mixed_thr = 500;
  int P64 = 0, lds_rows64 = 0;  // the fp64 workgroup kernel's LDS pitch / rows at this kp
  int64_t cap64 = 0;            // the fp64 fast kernels' row capacity (longer documents: the workgroup kernel)
  DevBuf Bp64, vals32, m_batch, m_orig, m_bptr, m_slot, m_cnt, eth64, elogth64, r64, keys64, vals64, gamma64, g0_64;
  const DCsr* vals32_for = nullptr;
  int32_t* hmcnt = nullptr;     // pinned: the two list counts
  DevBuf s_counts, s_weights, s_short, s_cincl, s_wincl, s_sincl;
  // the next draw is sampled on a side stream, concurrently with this step's E-step (it reads only
  // indptr and writes only the s_* buffers, which this step's fill_batch has consumed)
  hipStream_t side = nullptr;
  hipEvent_t ev_fill = nullptr, ev_samp = nullptr;
  bool samp_pending = false;
  // next(): the prefetched draw's batch (fill, slot order, offsets) is built on the side stream once the
  // previous step's E-step has read the batch buffers (ev_est), under that step's M-step and all-gathers.
  // prep_side: the last user of the batch buffers was next() (any other call's ensure_batch clears it).
  hipEvent_t ev_est = nullptr;
  bool prep_side = false;
  DevBuf side_scan_tmp;
  DevBuf long_list;  // rows / grid kernels: the launch's long documents (count word + slot offsets)
  DevBuf o_keys, o_keys2, o_idx, o_idx2, o_batch, o_orig, o_nnz, o_tmp;  // slot ordering (order_slots)
  bool sort_docs = true;  // STC_SORT_DOCS=0 keeps sampling order
  // fp64 rows kernels: the sstats pairs built and radix-sorted on a low-priority stream beside the E-step
  // (estep_and_stats); STC_PRESORT=0 sorts them after the E-step
  int presort = 1;
  hipStream_t sort_stream = nullptr;
  hipEvent_t ev_ps0 = nullptr, ev_sorted = nullptr;
  // many-topic kernel: per-entry row order, rarest terms first (lda_wide.hip), for `order_for`
  DevBuf order, order_df;
  const DCsr* order_for = nullptr;
  bool hot_order = true;  // STC_HOT_ORDER=0: CSR order
  int64_t wave_cap = 0;  // docs with nnz <= wave_cap run the wave-per-document E-step
  // many-topic documents larger than one CU: a team of P CUs per document (lda_wide.hip
  // k_estep_wide_mc); STC_WIDE_TEAM=n forces P = n (1: the one-CU kernel)
  int team_force = 0;
  bool tgrid = true;  // fp64 many-topic documents: the topic-split grid team kernel when they fit (STC_TGRID=0: off)
  bool tgrid_require = false;  // STC_TGRID=2 (tests): a many-topic fp64 launch that cannot take it is an error
  DevBuf team_words, team_x;
  unsigned* htmo = nullptr;  // pinned copy of the team kernel's timeout word
  int64_t team_fallbacks = 0;  // team launches re-run on the one-CU kernel after a timeout
  int64_t kcount[STC_KC_N] = {};  // E-step launches per kernel family (stc_lda_kernel_counts)

  // M-step sharding over the vocabulary (multi-GPU): rank r owns λ / expElogβ rows [r·Vs, (r+1)·Vs);
  // Vs is a multiple of the λ-update block so the per-block colsum partials (and hence colsum) are
  // bit-identical to the one-GPU reduction.  virt > 1 runs the same slices on one GPU without
  // collectives (STC_VIRTUAL_SHARDS, for testing the slicing).
  int shards = 1, virt = 1;
  int tail_fault = 0;  // test knob (STC_GROUP_STEP_FAULT): the tail_fault-th next step throws before its reduce-scatter
  bool force_coll = false;  // STC_COLLECTIVE_MSTEP=1: the RCCL slice path even on a 1-rank communicator (tests)
  // sharded steps: stat reduce-scattered in rs_chunks vocabulary sub-chunks on cstream, each as soon as
  // its sstats launch is done, and the M-step of sub-chunk j under the reduce-scatter of j+1
  // (STC_RS_CHUNKS, 1: one reduce-scatter after the whole stat)
  int rs_chunks = 4;
  hipStream_t cstream = nullptr;
  hipEvent_t ev_ss[16] = {}, ev_rs[16] = {};
  int64_t Vs = 0, vpad = 0;
  // one rank: sstats stamps the rows it writes (rowstamp[v] = the step's id) and the M-step reads the other
  // rows as zero, so stat is not cleared every step (V·kp·T bytes: 4.2 GB at config 5)
  DevBuf rowstamp;
  int32_t stamp_seq = 0, step_sid = 0;
  bool step_stamped = false;
  bool lam_stale = false;  // rows outside this rank's slice are out of date (sharded M-step)

  // minibatch draws: Spark's next() advances its generator on every call, empty batches included
  int64_t draws = 0;
  // prefetch: the next draw's membership is sampled during this step and its global size rides on
  // this step's collective, so the next call waits on an event instead of draining the stream
  bool pre_valid = false, pre_inflight = false;
  int64_t pre_draw = 0;
  hipEvent_t ev_pre = nullptr;
  int64_t* hpre = nullptr;

  bool timing = false;
  hipEvent_t ev[3][6] = {};
  int ev_set = 0;
  bool ev_pending[3] = {false, false, false};
  double acc_ms[5] = {0, 0, 0, 0, 0};
  int64_t timed_steps = 0;
  int64_t cum_docs = 0, cum_entries = 0;

  int64_t* hcnt = nullptr;  // pinned host words for the per-step count readback (one small copy)
  DevBuf dcnt;

  ~stc_lda() {
    for (auto& s : ev)
      for (auto& e : s)
        if (e) (void)hipEventDestroy(e);
    if (hcnt) (void)hipHostFree(hcnt);
    if (hmcnt) (void)hipHostFree(hmcnt);
    if (hpre) (void)hipHostFree(hpre);
    if (htmo) (void)hipHostFree(htmo);
    if (ev_pre) (void)hipEventDestroy(ev_pre);
    if (ev_fill) (void)hipEventDestroy(ev_fill);
    if (ev_samp) (void)hipEventDestroy(ev_samp);
    if (ev_est) (void)hipEventDestroy(ev_est);
    if (side) (void)hipStreamDestroy(side);
    for (int j = 0; j < 16; ++j) {
      if (ev_ss[j]) (void)hipEventDestroy(ev_ss[j]);
      if (ev_rs[j]) (void)hipEventDestroy(ev_rs[j]);
    }
    if (cstream) (void)hipStreamDestroy(cstream);
    if (ev_ps0) (void)hipEventDestroy(ev_ps0);
    if (ev_sorted) (void)hipEventDestroy(ev_sorted);
    if (sort_stream) (void)hipStreamDestroy(sort_stream);
  }
};

namespace {

template <typename T>
struct RcclType;
template <>
struct RcclType<float> {
  static constexpr ncclDataType_t v = ncclFloat32;
};
template <>
struct RcclType<double> {
  static constexpr ncclDataType_t v = ncclFloat64;
};

// ---------------------------------------------------------------------------------------
// Collectives.  RCCL over the context's communicator — or, for the members of one stc_group that share a
// device (a group of N handles on one GPU: the multi-GPU decomposition exercised on one device), an
// in-process transport: every member runs on its own host thread, the members exchange device pointers
// under a barrier and sum / copy with the kernels below, in member order (so every member's result is
// bit-identical).  Same call sequence on every member, as with RCCL.
// ---------------------------------------------------------------------------------------
}  // namespace

struct stc::LocalColl {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<void*> ptr;
  explicit LocalColl(int members) : n(members), ptr((size_t)members, nullptr) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (broken) throw Error(STC_ERR_STATE, "another member of the group failed");
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    cv.wait(lk, [&] { return gen != g || broken; });
    if (broken && gen == g) throw Error(STC_ERR_STATE, "another member of the group failed");
  }
  void fail() {
    std::lock_guard<std::mutex> lk(m);
    broken = true;
    cv.notify_all();
  }
};

namespace {

constexpr int kMaxMembers = 16;
struct MemberPtrs {
  const void* p[kMaxMembers];
};
template <typename T>
__global__ void k_sum_members(T* __restrict__ out, MemberPtrs src, int n, int64_t off, int64_t count) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    T acc = static_cast<const T*>(src.p[0])[off + i];
    for (int m = 1; m < n; ++m) acc += static_cast<const T*>(src.p[m])[off + i];
    out[i] = acc;
  }
}
size_t dt_size(ncclDataType_t t) { return t == ncclFloat32 ? 4 : 8; }
void launch_sum_members(hipStream_t s, ncclDataType_t t, void* out, const MemberPtrs& src, int n, int64_t off,
                        int64_t count) {
  if (count == 0) return;
  const int grid = (int)std::min<int64_t>(ceil_div(count, 256), 4096);
  if (t == ncclFloat64) k_sum_members<double><<<grid, 256, 0, s>>>(static_cast<double*>(out), src, n, off, count);
  else if (t == ncclFloat32) k_sum_members<float><<<grid, 256, 0, s>>>(static_cast<float*>(out), src, n, off, count);
  else if (t == ncclInt64) k_sum_members<int64_t><<<grid, 256, 0, s>>>(static_cast<int64_t*>(out), src, n, off, count);
  else throw Error(STC_ERR_STATE, "in-process collective: unsupported type");
  KERNEL_CHECK();
}
MemberPtrs published(const LocalColl& L) {
  MemberPtrs p{};
  for (int m = 0; m < L.n; ++m) p.p[m] = L.ptr[(size_t)m];
  return p;
}

// ---------------------------------------------------------------------------------------
// Waiting on work that may hold RCCL collectives.  A collective whose peer never arrives (a member
// thread or a rank that failed before enqueuing its side) never completes, and hipStreamSynchronize
// would block for ever behind it.  So on a context with a communicator every wait polls — the stream or
// event, the group's abort flag, ncclCommGetAsyncError — against a deadline (STC_COLL_TIMEOUT_MS,
// default 120 s).  A timeout or an asynchronous RCCL error aborts this context's communicator
// (ncclCommAbort releases its queued kernels) and throws STC_ERR_RCCL; a failed peer throws STC_ERR_STATE
// (stc_group's for_members then aborts every member's communicator).  Without a communicator: plain
// blocking waits, as before.
// ---------------------------------------------------------------------------------------
void abort_comm(Ctx& c) {
  if (!c.comm || c.comm_aborted.exchange(true)) return;
  (void)ncclCommAbort(c.comm);  // (c.comm stays set: the context keeps counting as collective, and refuses)
}
void check_comm(const Ctx& c) {
  if (c.comm_aborted.load())
    throw Error(STC_ERR_STATE, "the RCCL communicator was aborted after a failure: destroy this context / group");
  if (c.abort_flag && c.abort_flag->load())
    throw Error(STC_ERR_STATE, "another member of the group failed; its collectives were abandoned");
}
template <class Query, class Block>
void poll_wait(Ctx& c, Query query, Block block, const char* what) {
  if (!c.comm || !c.coll_enqueued) {  // nothing can be stuck behind a collective (e.g. the corpus upload)
    HIP_CHECK(block());
    return;
  }
  check_comm(c);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = query();
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    check_comm(c);
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(c.comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      abort_comm(c);
      throw Error(STC_ERR_RCCL, std::string("RCCL asynchronous error while waiting for ") + what + ": " +
                                    ncclGetErrorString(ae) + " (communicator aborted)");
    }
    const int64_t ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (ms > c.coll_timeout_ms) {
      abort_comm(c);
      throw Error(STC_ERR_RCCL, std::string("waiting for ") + what + ": not complete after " + std::to_string(ms) +
                                    " ms (STC_COLL_TIMEOUT_MS = " + std::to_string(c.coll_timeout_ms) +
                                    "): a collective's peer never arrived; communicator aborted");
    }
    // yield for the first 20 ms (a step's wait is milliseconds, and a sleep costs its timer slack — ≈ 50 µs
    // on Linux — per wait), then sleep in 100 µs steps
    if (ms < 20) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}
void wait_stream(Ctx& c, hipStream_t s) {
  poll_wait(c, [&] { return hipStreamQuery(s); }, [&] { return hipStreamSynchronize(s); }, "a stream");
}
void wait_event(Ctx& c, hipEvent_t e) {
  poll_wait(c, [&] { return hipEventQuery(e); }, [&] { return hipEventSynchronize(e); }, "an event");
}

void coll_group_start(Ctx& c) {
  if (!c.comm) return;
  check_comm(c);
  RCCL_CHECK(ncclGroupStart());
  c.in_group = true;
  c.coll_enqueued = true;
}
void coll_group_end(Ctx& c) {
  if (!c.comm) return;
  c.in_group = false;
  RCCL_CHECK(ncclGroupEnd());
}
// in place: buf ← Σ over members
void coll_all_reduce(Ctx& c, void* buf, size_t count, ncclDataType_t t, hipStream_t s) {
  if (c.comm) {
    if (!c.in_group) check_comm(c);
    c.coll_enqueued = true;
    RCCL_CHECK(ncclAllReduce(buf, buf, count, t, ncclSum, c.comm, s));
    return;
  }
  LocalColl& L = *c.local;
  HIP_CHECK(hipStreamSynchronize(s));
  L.ptr[(size_t)c.rank] = buf;
  L.barrier();
  c.coll_tmp.reserve(dt_size(t) * std::max<size_t>(count, 1));
  launch_sum_members(s, t, c.coll_tmp.p, published(L), L.n, 0, (int64_t)count);
  HIP_CHECK(hipStreamSynchronize(s));
  L.barrier();  // every member has read every buffer
  HIP_CHECK(hipMemcpyAsync(buf, c.coll_tmp.p, dt_size(t) * count, hipMemcpyDeviceToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
}
// recv (recvcount elements) ← Σ over members of their send[rank·recvcount, +recvcount); recv may be
// the member's own slice of send
void coll_reduce_scatter(Ctx& c, const void* send, void* recv, size_t recvcount, ncclDataType_t t, hipStream_t s) {
  if (c.comm) {
    if (!c.in_group) check_comm(c);
    c.coll_enqueued = true;
    RCCL_CHECK(ncclReduceScatter(send, recv, recvcount, t, ncclSum, c.comm, s));
    return;
  }
  LocalColl& L = *c.local;
  HIP_CHECK(hipStreamSynchronize(s));
  L.ptr[(size_t)c.rank] = const_cast<void*>(send);
  L.barrier();
  launch_sum_members(s, t, recv, published(L), L.n, (int64_t)(c.rank * recvcount), (int64_t)recvcount);
  HIP_CHECK(hipStreamSynchronize(s));
  L.barrier();
}
// recv[q·sendcount, +sendcount) ← member q's send, on every member (send may be its own slice of recv)
void coll_all_gather(Ctx& c, const void* send, void* recv, size_t sendcount, ncclDataType_t t, hipStream_t s) {
  if (c.comm) {
    if (!c.in_group) check_comm(c);
    c.coll_enqueued = true;
    RCCL_CHECK(ncclAllGather(send, recv, sendcount, t, c.comm, s));
    return;
  }
  LocalColl& L = *c.local;
  const size_t bytes = dt_size(t) * sendcount;
  HIP_CHECK(hipStreamSynchronize(s));
  L.ptr[(size_t)c.rank] = recv;
  L.barrier();
  for (int q = 0; q < L.n; ++q) {
    char* dst = static_cast<char*>(L.ptr[(size_t)q]) + (size_t)c.rank * bytes;
    if (dst != send && bytes) HIP_CHECK(hipMemcpyAsync(dst, send, bytes, hipMemcpyDeviceToDevice, s));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  L.barrier();
}

// The sstats pairs' radix sort by term (u32 keys, u64 values): rocprim's onesweep at STC_SORT_BITS bits (11: slower)
// per pass (gfx950's tuned block shape, 1024 threads × 8 items)
#ifndef STC_SORT_BITS
#define STC_SORT_BITS 9  // 18-bit term ids (V = 2^18) in two passes: sstats phase −75 µs headline, −90 µs planted vs 8
#endif
using TermSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, STC_SORT_BITS,
                                        rocprim::block_radix_rank_algorithm::match>>;
hipError_t term_sort(void* tmp, size_t& bytes, const uint32_t* kin, uint32_t* kout, const uint64_t* vin, uint64_t* vout,
                     int64_t n, int bits, hipStream_t s) {
  return rocprim::radix_sort_pairs<TermSortConfig>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, s);
}

inline int bits_for(int64_t n) {
  int b = 1;
  while ((int64_t(1) << b) < n) ++b;
  return b;
}

void record(stc_lda& L, int slot) {
  if (L.timing) HIP_CHECK(hipEventRecord(L.ev[L.ev_set][slot], L.ctx->stream));
}

// add the phase times of an event set whose step has completed (left pending otherwise)
void harvest(stc_lda& L, int set) {
  if (!L.ev_pending[set]) return;
  if (hipEventQuery(L.ev[set][5]) != hipSuccess) return;
  for (int p = 0; p < 5; ++p) {
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, L.ev[set][p], L.ev[set][p + 1]));
    L.acc_ms[p] += ms;
  }
  L.timed_steps += 1;
  L.ev_pending[set] = false;
}
void harvest_all(stc_lda& L) {
  for (int set = 0; set < 3; ++set) harvest(L, set);
}
// before a step records into the current set: a set is reused three steps later, long complete
void claim_event_set(stc_lda& L) {
  if (!L.timing || !L.ev_pending[L.ev_set]) return;
  wait_event(*L.ctx, L.ev[L.ev_set][5]);
  harvest(L, L.ev_set);
}

// the vocabulary slices of the M-step: shards = the RCCL ranks (or STC_VIRTUAL_SHARDS on one GPU).
// λ, expElogβ', logscale and stat are padded to shards·Vs rows (the RCCL reduce-scatter / all-gather
// chunks); the padded rows of stat are zero, those of λ / Bp never read.  Called before a step; a
// change of shard count (comm initialised after the handle) keeps λ and recomputes the rest.
void ensure_layout(stc_lda& L) {
  const int want = L.ctx->coll() && (L.ctx->n_ranks > 1 || L.force_coll) ? L.ctx->n_ranks : L.virt;
  if (want == L.shards && L.Vs > 0) return;
  if (L.lam_stale) throw Error(STC_ERR_STATE, "the shard count changed after sharded steps");
  const int64_t RB = lda::kRowsPerBlock;
  const int64_t Vs = ceil_div(ceil_div(L.V, (int64_t)want), RB) * RB;
  const int64_t vpad = Vs * want;
  if ((size_t)(8 * vpad * L.k) > L.lam.bytes) {  // grow λ, keeping its V·k prefix
    DevBuf tmp;
    tmp.reserve(8 * vpad * L.k);
    if (L.lam.p) {
      HIP_CHECK(hipMemcpyAsync(tmp.p, L.lam.p, 8 * L.V * L.k, hipMemcpyDeviceToDevice, L.ctx->stream));
      wait_stream(*L.ctx, L.ctx->stream);
    }
    std::swap(tmp.p, L.lam.p);
    std::swap(tmp.bytes, L.lam.bytes);
  }
  L.Bp.reserve(L.tsize * vpad * L.kp);
  if (L.mixed) L.Bp64.reserve(8 * vpad * L.kp);
  L.stat.reserve(L.tsize * vpad * L.kp);
  L.logscale.reserve(8 * vpad);
  L.colpart.reserve(8 * (vpad / RB) * L.k);
  if ((size_t)(4 * vpad) > L.rowstamp.bytes) {  // a new stamp array: no row is this step's
    L.rowstamp.reserve(4 * vpad);
    HIP_CHECK(hipMemsetAsync(L.rowstamp.p, 0xFF, L.rowstamp.bytes, L.ctx->stream));
    L.stamp_seq = 0;
  }
  L.shards = want;
  L.Vs = Vs;
  L.vpad = vpad;
  L.lam_stale = false;
}
void refresh(stc_lda& L);
void relayout(stc_lda& L) {
  const int old = L.shards;
  const int64_t vs = L.Vs;
  ensure_layout(L);
  if ((old != L.shards || vs != L.Vs) && L.has_topics) refresh(L);
}

template <typename T>
void refresh_model(stc_lda& L) {
  hipStream_t s = L.ctx->stream;
  lda::launch_lambda_eeb<T>(s, false, L.lam.as<double>(), nullptr, L.Bp.as<T>(), L.logscale.as<double>(), L.V,
                            L.k, L.kp, 0.0, 0.0, 0.0, nullptr, L.colpart.as<double>(), L.nblocks_m,
                            L.mixed ? L.Bp64.as<double>() : nullptr);
  lda::launch_colsum_reduce(s, L.colpart.as<double>(), L.nblocks_m, L.k, nullptr, L.colsum.as<double>(),
                            L.psic.as<double>());
  L.has_topics = true;
}

void refresh(stc_lda& L) {
  if (L.dtype == STC_F32) refresh_model<float>(L);
  else refresh_model<double>(L);
}

template <typename T>
void ensure_batch(stc_lda& L, int64_t n, int64_t E, bool from_next = false) {
  if (!from_next) L.prep_side = false;
  const size_t ts = sizeof(T);
  L.batch_raw.reserve(4 * (n + 1));
  L.batch.reserve(4 * (n + 1));
  L.orig.reserve(4 * (n + 1));
  L.flags.reserve(4 * (n + 1));
  L.sincl.reserve(4 * (n + 1));
  L.bptr.reserve(8 * (n + 1));
  L.bnnz.reserve(8 * (n + 1));
  L.nnzp.reserve(8 * (n + 1));
  L.gamma.reserve(ts * n * L.k);
  L.eth.reserve(ts * n * L.kp);
  L.elogth.reserve(ts * n * L.k);
  L.iters.reserve(4 * n);
  L.nonempty.reserve(4 * n);
  L.r.reserve(ts * E);
  L.keys.reserve(4 * E);
  L.vals.reserve(8 * E);
  L.skeys.reserve(4 * E);
  L.svals.reserve(8 * E);
  const int64_t nchunks = ceil_div(E, lda::kChunk) + 1;
  L.headbuf.reserve(ts * nchunks * L.kp);
  L.tailbuf.reserve(ts * nchunks * L.kp);
  L.lpart.reserve(sizeof(double) * lda::kLogphatBlocks * (L.k + 1));
  size_t tb = 0;
  HIP_CHECK(term_sort(nullptr, tb, L.keys.as<uint32_t>(), L.skeys.as<uint32_t>(), L.vals.as<uint64_t>(),
                      L.svals.as<uint64_t>(), std::max<int64_t>(E, 1), bits_for(L.V), L.ctx->stream));
  L.sort_tmp.reserve(tb);
}

template <typename X>
void incl_scan(stc_lda& L, const X* in, X* out, int64_t n, hipStream_t s = nullptr, DevBuf* tmp = nullptr) {
  if (n <= 0) return;
  if (!s) s = L.ctx->stream;
  if (!tmp) tmp = &L.scan_tmp;
  size_t sb = 0;
  HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, sb, in, out, (int)n, s));
  tmp->reserve(sb);
  HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp->p, sb, in, out, (int)n, s));
}

// bptr[0] = 0, bptr[i+1] = Σ_{j<=i} nnz_p[j]  (entry offsets of the partitioned slots)
void slot_offsets(stc_lda& L, int64_t n, hipStream_t s = nullptr, DevBuf* tmp = nullptr) {
  if (!s) s = L.ctx->stream;
  HIP_CHECK(hipMemsetAsync(L.bptr.p, 0, sizeof(int64_t), s));
  incl_scan<int64_t>(L, L.nnzp.as<int64_t>(), L.bptr.as<int64_t>() + 1, n, s, tmp);
}

struct Part {
  int64_t E = 0, n_short = 0;
};

// Partition members (raw = row ids on device, or nullptr for identity rows) into
// [nnz <= wave cap | rest] slots: fills L.batch, L.orig, L.nnzp.  One host sync (E, n_short).
Part partition(stc_lda& L, const int64_t* indptr, const int32_t* raw, int64_t n) {
  hipStream_t s = L.ctx->stream;
  Part p;
  if (n == 0) return p;
  lda::launch_part_flags(s, indptr, raw, n, L.wave_cap, L.bnnz.as<int64_t>(), L.flags.as<int32_t>());
  incl_scan<int64_t>(L, L.bnnz.as<int64_t>(), L.bptr.as<int64_t>() + 1, n);  // temp: total E
  incl_scan<int32_t>(L, L.flags.as<int32_t>(), L.sincl.as<int32_t>(), n);
  int32_t ns = 0;
  HIP_CHECK(hipMemcpyAsync(&p.E, L.bptr.as<int64_t>() + n, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(&ns, L.sincl.as<int32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, s));
  wait_stream(*L.ctx, s);
  p.n_short = ns;
  lda::launch_part_scatter(s, raw, L.bnnz.as<int64_t>(), n, L.flags.as<int32_t>(), L.sincl.as<int32_t>(),
                           L.batch.as<int32_t>(), L.orig.as<int32_t>(), L.nnzp.as<int64_t>());
  return p;
}

template <typename T>
lda::EStepArgs<T> estep_args(stc_lda& L) {
  lda::EStepArgs<T> a;
  a.k = L.k;
  a.kp = L.kp;
  a.P = L.P;
  a.lds_rows = L.lds_rows;
  a.Bp = L.Bp.as<T>();
  if constexpr (std::is_same<T, double>::value) {
    if (L.mixed) {  // the fp64 re-solve / inference of a mixed handle: the fp64 rows and workgroup shape
      a.Bp = L.Bp64.as<double>();
      a.P = L.P64;
      a.lds_rows = L.lds_rows64;
    }
  }
  a.logscale = L.logscale.as<double>();
  a.psic = L.psic.as<double>();
  a.alpha = L.alpha.as<double>();
  a.seed = L.cfg.seed;
  a.rank = L.ctx->rank;
  a.gamma_shape = L.cfg.gamma_shape;
  a.max_iter = L.cfg.max_inner_iter;
  a.stop_thr = lda::stop_threshold(L.k);
  return a;
}

// the register-resident kernel for the (k, dtype): the grid kernels up to k = 128 (fp32) / 104 (fp64),
// the topics-across-lanes kernel (lda_wide.hip) beyond
bool use_wide(int k, int dtype) { return dtype == STC_F32 ? lda::grid_row_cap(k) == 0 : lda::rows64_row_cap(k) == 0; }

// the fast kernel's slots [0, n_short) in descending nnz: the longest documents start first, so the
// launch does not end on a few long documents started late (longest-processing-time-first).  Each
// slot keeps its member index (orig: γ₀ keys, outputs), so results only change in the summation
// order of sstats within a term.
void order_slots(stc_lda& L, int64_t n_short, hipStream_t s = nullptr) {
  // measured: no gain at 50k docs per launch (≈ 100 documents per workgroup slot, the tail is
  // short), +0.13 ms of sorting; kept for small per-rank minibatches (strong scaling), where a
  // launch is only a few documents deep
  if (!L.sort_docs || n_short < 2 || n_short > 16384) return;
  if (!s) s = L.ctx->stream;
  L.o_keys.reserve(8 * n_short);
  L.o_keys2.reserve(8 * n_short);
  L.o_idx.reserve(4 * n_short);
  L.o_idx2.reserve(4 * n_short);
  L.o_batch.reserve(4 * n_short);
  L.o_orig.reserve(4 * n_short);
  L.o_nnz.reserve(8 * n_short);
  HIP_CHECK(hipMemcpyAsync(L.o_keys.p, L.nnzp.p, 8 * n_short, hipMemcpyDeviceToDevice, s));
  lda::launch_iota(s, L.o_idx.as<int32_t>(), n_short);
  size_t tb = 0;
  HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, L.o_keys.as<int64_t>(), L.o_keys2.as<int64_t>(),
                                                         L.o_idx.as<int32_t>(), L.o_idx2.as<int32_t>(), (int)n_short,
                                                         0, 16, s));
  L.o_tmp.reserve(tb);
  HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(L.o_tmp.p, tb, L.o_keys.as<int64_t>(), L.o_keys2.as<int64_t>(),
                                                         L.o_idx.as<int32_t>(), L.o_idx2.as<int32_t>(), (int)n_short,
                                                         0, 16, s));
  lda::launch_permute_slots(s, L.o_idx2.as<int32_t>(), n_short, L.batch.as<int32_t>(), L.orig.as<int32_t>(),
                            L.nnzp.as<int64_t>(), L.o_batch.as<int32_t>(), L.o_orig.as<int32_t>(),
                            L.o_nnz.as<int64_t>());
  HIP_CHECK(hipMemcpyAsync(L.batch.p, L.o_batch.p, 4 * n_short, hipMemcpyDeviceToDevice, s));
  HIP_CHECK(hipMemcpyAsync(L.orig.p, L.o_orig.p, 4 * n_short, hipMemcpyDeviceToDevice, s));
  HIP_CHECK(hipMemcpyAsync(L.nnzp.p, L.o_nnz.p, 8 * n_short, hipMemcpyDeviceToDevice, s));
}

// the many-topic kernel's row order for the training corpus: the corpus's document frequencies,
// then each row's entries by ascending df (once per set_corpus)
void ensure_order(stc_lda& L) {
  if (!L.hot_order || L.wave_cap <= 0 || !use_wide(L.k, L.dtype) || L.order_for == L.corpus) return;
  const DCsr& m = *L.corpus;
  L.order.reserve(4 * std::max<int64_t>(m.nnz, 1));
  L.order_df.reserve(8 * m.cols);
  idf::doc_freq(*L.ctx, m, L.order_df.as<int64_t>());
  hashing::row_order_by_df(*L.ctx, m, L.order_df.as<int64_t>(), L.order.as<int32_t>());
  L.order_for = L.corpus;
}

// team size for the many-topic kernel: enough CUs that a document of `mean_rows` rows is resident
// team for the many-topic kernel: enough CUs that a document of `mean_rows` rows stays resident.
// k ≤ 512: rows split (k_estep_wide_mc), P = ⌈1.05·rows / resident rows⌉ ≤ 4 (config 4, k = 500:
// fp64 P = 4, fp32 P = 2).  k > 512: topics split (k_estep_wide_tc), members of up to 1024 topics, when
// the one-CU kernel cannot keep the rows resident (config 5, k = 2000: fp64 P = 2; fp32 stays one CU).
// P = 1: the one-CU kernel.  STC_WIDE_TEAM=n forces P = n.
struct TeamChoice {
  int P = 1;
  bool topics = false;
  bool grid = false;  // the fp64 topic-split grid kernel (lda_team64.hip k_estep_tgrid64)
};
template <typename T>
TeamChoice team_choice(const stc_lda& L, double mean_rows, int64_t max_row) {
  const double need = 1.05 * mean_rows;
  if (L.team_force == 1) return {1, false};
  // fp64: the topic-split team with the rows64 grid in every member (members of 104 topics) when every
  // document of the corpus fits its 448 rows (config 4: k = 500, P = 5, 371 ± 10 rows); STC_TGRID=0: off
  if constexpr (std::is_same<T, double>::value) {
    const int P = lda::tgrid64_members(L.kp);
    if (L.tgrid && L.team_force == 0 && P >= 2 && P <= 8 && max_row >= 0 && max_row <= lda::tgrid64_row_cap())
      return {P, true, true};
    if (L.tgrid_require)
      throw Error(STC_ERR_STATE, "STC_TGRID=2: the fp64 grid team kernel cannot take this launch (k " + std::to_string(L.k) +
                                     ", longest document " + std::to_string(max_row) + " rows)");
  }
  if (L.k <= 512) {
    if (L.team_force > 1) return {L.team_force, false};
    const int P = (int)std::ceil(need / std::max(lda::wide_resident_rows<T>(L.k), 1));
    return {std::max(1, std::min(P, 4)), false};
  }
  if (L.team_force > 1) return {std::max(L.team_force, (L.k + 2047) / 2048), true};
  // only when a quarter or more of the rows would be re-streamed: a few streamed rows cost the one-CU
  // kernel less than a member's exchange (config 5 planted state, fp32: 47 resident of ≈ 47 rows, one
  // CU 2.2× faster than P = 2 at 3 inner iterations)
  if (lda::wide_resident_rows<T>(L.k) >= 0.75 * mean_rows) return {1, false};
  // two members of up to 1024 topics: measured at config 5 (k = 2000, fp64, E-step per minibatch) P = 2
  // 44.0 ms, one CU 53.7, P = 3 (a member without topics) 71.2, P = 4 61.9 — a member's exchange
  // latency is fixed, so the fewest members that hold the block win
  return {std::max(2, std::min(4, (L.k + 1023) / 1024)), true};
}

// The team kernel's timeout word: a member whose partner never arrived (a block that was not
// co-resident after all, e.g. another process holding CUs) gave up instead of hanging, and so did its
// team.  launch_split() reads the word right after the launch and, when it is set, runs the same slots
// again on the one-CU kernel inside the same call: the step completes with the one-CU kernel's results
// (which every member of a group or every rank gets on its own, so no rank's state can diverge).
// debug knob STC_TEAM_FAULT=m: member m of team 0 never publishes (its partners time out quickly)
int team_fault_member() {
  const char* e = getenv("STC_TEAM_FAULT");
  return e ? atoi(e) : -1;
}

template <typename T>
bool launch_wide_team(stc_lda& L, const lda::EStepArgs<T>& w, bool stats, TeamChoice tc, int64_t max_row) {
  const int P = tc.P;
  Ctx& c = *L.ctx;
  hipStream_t s = c.stream;
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device));
  lda::WideTeam wt;
  wt.P = P;
  wt.blocks = 8 * P * (cus / (8 * P));
  if (wt.blocks <= 0) return false;  // fewer CUs than one team per XCD group: the one-CU kernel
  const int teams = wt.blocks / P;
  // granules per member: rows split, the s partials + Σ r·φ; topics split, the φ partials + Σ|Δγ| + Σγ
  wt.xstride = tc.grid ? lda::tgrid64_xstride() : std::max<int64_t>(L.kp + 1, 512 + 2);
  const size_t xbytes = 16 * (size_t)teams * 2 * P * (size_t)wt.xstride;
  L.team_words.reserve(16);
  L.team_x.reserve(xbytes);
  if (!L.htmo) {
    HIP_CHECK(hipHostMalloc((void**)&L.htmo, sizeof(unsigned), hipHostMallocDefault));
    *L.htmo = 0;
  }
  wt.tmo = L.team_words.as<unsigned>();
  wt.xbuf = L.team_x.p;
  wt.fault_member = team_fault_member();
  wt.max_row = max_row <= INT32_MAX ? (int)max_row : -1;
  if (wt.fault_member >= 0) wt.spin_limit = 1u << 14;
  // every polled word zeroed before every launch: the timeout word, and the granules' epoch tags
  // (a tag left by an earlier launch could equal an epoch this launch waits for)
  HIP_CHECK(hipMemsetAsync(L.team_words.p, 0, 16, s));
  HIP_CHECK(hipMemsetAsync(L.team_x.p, 0, xbytes, s));
  bool ok;
  if constexpr (std::is_same<T, double>::value) {
    ok = tc.grid ? lda::launch_estep_tgrid64(s, w, stats, wt)
                 : tc.topics ? lda::launch_estep_wide_tc<T>(s, w, stats, wt) : lda::launch_estep_wide_mc<T>(s, w, stats, wt);
  } else {
    ok = tc.topics ? lda::launch_estep_wide_tc<T>(s, w, stats, wt) : lda::launch_estep_wide_mc<T>(s, w, stats, wt);
  }
  if (ok) HIP_CHECK(hipMemcpyAsync(L.htmo, wt.tmo, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  if (!ok && tc.grid && L.tgrid_require) throw Error(STC_ERR_STATE, "STC_TGRID=2: the grid team could not be resident");
  return ok;
}


// fast kernel on slots [0, n_short), workgroup kernel on [n_short, n); mean_rows = the launch's mean
// entries per document (the many-topic kernel's team size)
template <typename T>
void launch_split(stc_lda& L, const DCsr& m, lda::EStepArgs<T> a, int64_t n, int64_t n_short, bool stats,
                  bool bound, double mean_rows) {
  hipStream_t s = L.ctx->stream;
  if (n_short > 0) {
    lda::EStepArgs<T> w = a;
    w.slot0 = 0;
    w.n = n_short;
    const int dt = std::is_same<T, float>::value ? STC_F32 : STC_F64;  // (a mixed handle runs both)
    const TeamChoice tc = use_wide(L.k, dt) && !bound ? team_choice<T>(L, mean_rows, m.max_row) : TeamChoice{};
    const bool team = tc.P > 1 && launch_wide_team<T>(L, w, stats, tc, m.max_row);
    if (team) {  // launched (a grid that could not be resident falls through to the one-CU kernel)
      L.kcount[tc.grid ? STC_KC_TGRID64 : tc.topics ? STC_KC_WIDE_TC : STC_KC_WIDE_MC] += 1;
      wait_stream(*L.ctx, s);
      if (*L.htmo) {  // a team gave up: the same slots on the one-CU kernel (it rewrites every output)
        *L.htmo = 0;
        L.team_fallbacks += 1;
        L.kcount[STC_KC_TEAM_FALLBACK] += 1;
        L.kcount[STC_KC_WIDE] += 1;
        lda::launch_estep_wide<T>(s, w, stats, bound);
      }
    } else if (use_wide(L.k, dt)) {
      L.kcount[STC_KC_WIDE] += 1;
      lda::launch_estep_wide<T>(s, w, stats, bound);
    } else if constexpr (std::is_same<T, float>::value) {
      const bool long_docs = m.max_row < 0 || m.max_row > lda::grid_onchip_rows(L.k);
      // the long-document list (count word + slots) and, past it, the resident grid's ticket word
      L.long_list.reserve(4 * (size_t)(n_short + 2));
      w.long_list = L.long_list.as<int32_t>();
      L.kcount[STC_KC_GRID] += 1;
      lda::launch_estep_grid(s, w, stats, bound, long_docs);
    } else {
      const bool long_docs = m.max_row < 0 || m.max_row > lda::rows64_onchip_rows(L.k);
      // the long-document list (count word + slots) and, past it, the resident grid's ticket word
      L.long_list.reserve(4 * (size_t)(n_short + 2));
      w.long_list = L.long_list.as<int32_t>();
      L.kcount[STC_KC_ROWS64] += 1;
      if (long_docs) L.kcount[STC_KC_ROWS64_LONG] += 1;
      lda::launch_estep_rows64(s, w, stats, bound, long_docs);
    }
  }
  if (n > n_short) {
    a.slot0 = n_short;
    a.n = n - n_short;
    L.kcount[STC_KC_WORKGROUP] += 1;
    lda::launch_estep<T>(s, a, stats, bound);
  }
}

template <typename T>
const T* upload_gamma0(stc_lda& L, const double* gamma0, int64_t n) {
  if (!gamma0 || n == 0) return nullptr;
  std::vector<T> h((size_t)(n * L.k));
  for (size_t j = 0; j < h.size(); ++j) {
    STC_REQUIRE(gamma0[j] > 0.0, "gamma0 entries must be > 0");
    h[j] = (T)gamma0[j];
  }
  L.g0.reserve(sizeof(T) * h.size());
  HIP_CHECK(hipMemcpyAsync(L.g0.p, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice, L.ctx->stream));
  wait_stream(*L.ctx, L.ctx->stream);  // h dies at scope exit
  return L.g0.as<T>();
}

// the CSR value dtype a handle reads (a mixed handle: the fp64 values, and an fp32 copy it makes itself)
int corpus_dtype(const stc_lda& L) { return L.mixed ? STC_F64 : L.dtype; }

// STC_MIXED with an injected γ₀: its fp64 copy for the re-solve (the fp32 E-step reads the rounded one)
const double* mixed_gamma0(stc_lda& L, const double* gamma0, int64_t n) {
  if (!L.mixed || !gamma0 || n == 0) return nullptr;
  L.g0_64.reserve(sizeof(double) * n * L.k);
  HIP_CHECK(hipMemcpyAsync(L.g0_64.p, gamma0, sizeof(double) * n * L.k, hipMemcpyHostToDevice, L.ctx->stream));
  wait_stream(*L.ctx, L.ctx->stream);  // (the caller's buffer)
  return L.g0_64.as<double>();
}

// a step's M-step is sharded over the ranks (reduce-scatter, slice update, all-gather)
bool sharded(const stc_lda& L) { return L.ctx->coll() && (L.ctx->n_ranks > 1 || L.force_coll); }

// the stat sub-chunk layout of a sharded step (lda_kernels.h StatMap; nsub = 1: one reduce-scatter):
// at most rs_chunks sub-chunks of whole λ-update blocks, the last one the rest of the slice
lda::StatMap stat_layout(const stc_lda& L) {
  lda::StatMap m;
  const int64_t nb = L.Vs / lda::kRowsPerBlock;
  if (!sharded(L) || L.rs_chunks <= 1 || nb < 2) return m;
  const int64_t per = ceil_div(nb, (int64_t)L.rs_chunks);
  m.vs = (uint32_t)L.Vs;
  m.vsj = (uint32_t)(per * lda::kRowsPerBlock);
  m.n = L.shards;
  m.nsub = (int)ceil_div(nb, per);
  return m;
}
// sub-chunk j: (first canonical row within a slice, rows)
std::pair<int64_t, int64_t> stat_sub_rows(const lda::StatMap& m, int j) {
  const int64_t w = j < m.nsub - 1 ? (int64_t)m.vsj : (int64_t)m.vs - (int64_t)(m.nsub - 1) * m.vsj;
  return {(int64_t)j * m.vsj, w};
}

// γ₀ of the n partitioned slots' members from the counter RNG, keyed as the E-step kernels key it
// (key_mode 0: train_doc_key(iteration, rank, member); 1: doc_id_base + row), into L.g0gen
template <typename T>
const T* gen_gamma0(stc_lda& L, hipStream_t s, int64_t n, uint64_t seed, int64_t iteration, int key_mode,
                    int64_t base) {
  if (n == 0) return nullptr;
  L.g0gen.reserve(sizeof(T) * n * L.k);
  lda::launch_gamma0<T>(s, L.batch.as<int32_t>(), L.orig.as<int32_t>(), n, L.k, seed, iteration, L.ctx->rank,
                        key_mode, base, L.cfg.gamma_shape, L.g0gen.as<T>());
  return L.g0gen.as<T>();
}

// E-step over the n partitioned slots (L.batch / L.orig / L.bptr), then logphat / non-empty count into
// L.small and the term-sorted sstats SpMM into L.stat (V×kp, row-scaled).  split: a training step of a
// sharded handle — stat in the sub-chunk layout, one sstats launch per sub-chunk (ev_ss[j] after each).
template <typename T>
void launch_split(stc_lda& L, const DCsr& m, lda::EStepArgs<T> a, int64_t n, int64_t n_short, bool stats,
                  bool bound, double mean_rows);

// STC_MIXED: after the fp32 E-step over the n slots, the documents whose fp32 fixed point took more than
// mixed_thr iterations are re-solved in fp64 — the same γ₀ (the training key drawn in the kernel, or the
// injected fp64 γ₀ g0_64), the fp64 expElogβ' rows (Bp64) and the corpus's fp64 values — and their eθ',
// E[log θ], r, sstats sort values, iteration counts (and γ) replace the fp32 ones before logphat and
// sstats read them.  One host readback (the two list counts) sizes the fp64 launches.  Why the fp32
// iteration count selects them: DESIGN.md §4 (mixed mode).
void mixed_resolve(stc_lda& L, int64_t n, int64_t E, int64_t iteration, const double* g0_64, bool want_gamma) {
  if (n == 0) return;
  const DCsr& m = *L.corpus;
  hipStream_t s = L.ctx->stream;
  L.m_batch.reserve(4 * n);
  L.m_orig.reserve(4 * n);
  L.m_slot.reserve(4 * n);
  L.m_bptr.reserve(8 * n);
  L.m_cnt.reserve(2 * sizeof(int32_t));
  if (!L.hmcnt) HIP_CHECK(hipHostMalloc((void**)&L.hmcnt, 2 * sizeof(int32_t), hipHostMallocDefault));
  lda::launch_mixed_list(s, m.indptr.as<int64_t>(), L.batch.as<int32_t>(), L.orig.as<int32_t>(), L.bptr.as<int64_t>(),
                         L.iters.as<int32_t>(), L.nonempty.as<int32_t>(), n, L.mixed_thr, L.cap64,
                         L.m_batch.as<int32_t>(), L.m_orig.as<int32_t>(), L.m_bptr.as<int64_t>(), L.m_slot.as<int32_t>(),
                         L.m_cnt.as<int32_t>());
  HIP_CHECK(hipMemcpyAsync(L.hmcnt, L.m_cnt.p, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  wait_stream(*L.ctx, s);
  const int ms = L.hmcnt[0], ml = L.hmcnt[1];
  if (ms + ml == 0) return;
  L.kcount[STC_KC_MIXED_RESOLVES] += 1;
  L.kcount[STC_KC_MIXED_DOCS] += ms + ml;
  L.eth64.reserve(8 * n * L.kp);
  L.elogth64.reserve(8 * n * L.k);
  L.r64.reserve(8 * std::max<int64_t>(E, 1));
  L.keys64.reserve(4 * std::max<int64_t>(E, 1));
  L.vals64.reserve(8 * std::max<int64_t>(E, 1));
  if (want_gamma) L.gamma64.reserve(8 * n * L.k);
  lda::EStepArgs<double> a = estep_args<double>(L);  // Bp64 and the fp64 workgroup shape
  a.indptr = m.indptr.as<int64_t>();
  a.indices = m.indices.as<int32_t>();
  a.values = m.values.as<double>();
  a.gamma0 = g0_64;
  a.iteration = iteration;
  a.key_mode = 0;
  a.gamma = want_gamma ? L.gamma64.as<double>() : nullptr;
  a.r = L.r64.as<double>();
  a.keys = L.keys64.as<uint32_t>();  // (the fp64 sort values are the fp64 layout's: scratch, rewritten by the fixup)
  a.vals = L.vals64.as<uint64_t>();
  a.iters = L.iters.as<int32_t>();
  a.nonempty = L.nonempty.as<int32_t>();
  const double mean_rows = (double)E / (double)n;
  if (ms > 0) {  // the documents the fp64 fast kernels hold
    lda::EStepArgs<double> w = a;
    w.batch = L.m_batch.as<int32_t>();
    w.orig = L.m_orig.as<int32_t>();
    w.bptr = L.m_bptr.as<int64_t>();
    w.eth = L.eth64.as<double>();
    w.elogth = L.elogth64.as<double>();
    launch_split<double>(L, m, w, ms, ms, true, false, mean_rows);
  }
  if (ml > 0) {  // the longer ones: the workgroup kernel
    const int64_t off = n - ml;
    lda::EStepArgs<double> w = a;
    w.batch = L.m_batch.as<int32_t>() + off;
    w.orig = L.m_orig.as<int32_t>() + off;
    w.bptr = L.m_bptr.as<int64_t>() + off;
    w.eth = L.eth64.as<double>() + off * L.kp;
    w.elogth = L.elogth64.as<double>() + off * L.k;
    launch_split<double>(L, m, w, ml, 0, true, false, mean_rows);
  }
  lda::launch_mixed_fixup(s, m.indptr.as<int64_t>(), L.m_batch.as<int32_t>(), L.m_orig.as<int32_t>(),
                          L.m_bptr.as<int64_t>(), L.m_slot.as<int32_t>(), n, ms, ml, L.k, L.kp, L.eth64.as<double>(),
                          L.elogth64.as<double>(), L.r64.as<double>(), want_gamma ? L.gamma64.as<double>() : nullptr,
                          L.eth.as<float>(), L.elogth.as<float>(), L.r.as<float>(), L.vals.as<uint64_t>(),
                          want_gamma ? L.gamma.as<float>() : nullptr);
}

template <typename T>
void estep_and_stats(stc_lda& L, int64_t n, int64_t n_short, int64_t E, const T* g0, int64_t iteration,
                     bool split = false, const double* g0_64 = nullptr, bool want_gamma = false) {
  hipStream_t s = L.ctx->stream;
  lda::EStepArgs<T> a = estep_args<T>(L);
  a.indptr = L.corpus->indptr.as<int64_t>();
  a.indices = L.corpus->indices.as<int32_t>();
  a.values = L.mixed ? L.vals32.as<T>() : L.corpus->values.as<T>();
  // mixed: the fp32 pass stops a document at mixed_thr + 1 iterations — it is re-solved in fp64 anyway, so the
  // fp32 iterations past the threshold (up to ≈ 300 per such document at the bench state) are not spent
  if (L.mixed) a.max_iter = std::min(a.max_iter, L.mixed_thr + 1);
  a.batch = L.batch.as<int32_t>();
  a.orig = L.orig.as<int32_t>();
  a.bptr = L.bptr.as<int64_t>();
  a.order = L.order_for == L.corpus ? L.order.as<int32_t>() : nullptr;
  a.gamma0 = g0;
  a.iteration = iteration;
  a.key_mode = 0;
  a.gamma = L.gamma.as<T>();
  a.eth = L.eth.as<T>();
  a.elogth = L.elogth.as<T>();
  a.r = L.r.as<T>();
  a.keys = L.keys.as<uint32_t>();
  a.vals = L.vals.as<uint64_t>();
  a.iters = L.iters.as<int32_t>();
  a.nonempty = L.nonempty.as<int32_t>();
  record(L, 1);
  // fp64 on the rows kernels (k ≤ 104, every slot on them): an entry's sort value carries its index, not r, so
  // the (term, slot) pairs and their radix sort depend on the batch alone — they run on a low-priority stream
  // beside the E-step, whose blocks take the CU slots the resident grid frees as it drains, instead of after it
  bool presort = false;
  if constexpr (std::is_same<T, double>::value)
    presort = L.presort && !L.mixed && !use_wide(L.k, STC_F64) && n_short == n && E > 0;
  hipStream_t ss = nullptr;  // the handle's side stream when it has one (no extra hardware queue), else its own
  auto enqueue_presort = [&] {
    lda::launch_entry_pairs(ss, L.corpus->indptr.as<int64_t>(), L.corpus->indices.as<int32_t>(),
                            L.batch.as<int32_t>(), L.bptr.as<int64_t>(), n, L.keys.as<uint32_t>(), L.vals.as<uint64_t>());
    size_t tb = L.sort_tmp.bytes;
    HIP_CHECK(term_sort(L.sort_tmp.p, tb, L.keys.as<uint32_t>(), L.skeys.as<uint32_t>(), L.vals.as<uint64_t>(),
                        L.svals.as<uint64_t>(), E, bits_for(L.V), ss));
    HIP_CHECK(hipEventRecord(L.ev_sorted, ss));
  };
  if (presort) {
    if (!L.ev_ps0) {
      HIP_CHECK(hipEventCreateWithFlags(&L.ev_ps0, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&L.ev_sorted, hipEventDisableTiming));
    }
    // a process with several handles runs past the device's hardware queues (GPU_MAX_HW_QUEUES) when each adds
    // a stream, and a stream sharing a queue waits behind unrelated work: the side stream (next()'s draws,
    // which then queue behind the sort) is used when it exists
    if (!L.side && !L.sort_stream) {
      int least = 0, greatest = 0;
      HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIP_CHECK(hipStreamCreateWithPriority(&L.sort_stream, hipStreamNonBlocking, least));
    }
    ss = L.side ? L.side : L.sort_stream;
    HIP_CHECK(hipEventRecord(L.ev_ps0, s));  // the batch and its entry offsets are built; skeys / svals free
    HIP_CHECK(hipStreamWaitEvent(ss, L.ev_ps0, 0));
    // STC_PRESORT=2: the pairs and the sort enqueued before the E-step launch (their blocks then compete with
    // the grid's first workgroups); default: after it, so the resident grid is dispatched first
    if (L.presort == 2) enqueue_presort();
    a.keys = nullptr;  // (the E-step kernels leave the pairs alone)
    a.vals = nullptr;
  }
  launch_split<T>(L, *L.corpus, a, n, n_short, true, false, n > 0 ? (double)E / (double)n : 0.0);
  if (presort && L.presort != 2) enqueue_presort();
  if constexpr (std::is_same<T, float>::value) {
    if (L.mixed) mixed_resolve(L, n, E, iteration, g0_64, want_gamma);
  }
  if (L.ev_est) HIP_CHECK(hipEventRecord(L.ev_est, s));  // the batch buffers are free (next_impl)
  record(L, 2);
  // logphat first: its all-reduce rides with the first stat sub-chunk of a sharded step
  if (n > 0) {
    lda::launch_logphat<T>(s, L.elogth.as<T>(), L.nonempty.as<int32_t>(), n, L.k, L.small.as<double>(),
                             L.lpart.as<double>());
    lda::launch_iter_stats(s, L.iters.as<int32_t>(), L.nonempty.as<int32_t>(), n, L.cfg.max_inner_iter,
                           L.stats4.as<int64_t>(), L.cum2.as<int64_t>());
  } else {
    HIP_CHECK(hipMemsetAsync(L.small.p, 0, sizeof(double) * (L.k + 1), s));
    HIP_CHECK(hipMemsetAsync(L.stats4.p, 0, sizeof(int64_t) * 4, s));
  }
  // a training step of one rank stamps its rows instead of clearing stat (the M-step reads unstamped rows as
  // zero); sharded steps clear it — the reduce-scatter sums every row of every rank
  L.step_stamped = split && !sharded(L);
  if (L.step_stamped) {
    L.stamp_seq = L.stamp_seq == INT32_MAX ? 0 : L.stamp_seq + 1;  // (never −1, the fresh array's value)
    L.step_sid = L.stamp_seq;
  } else {
    HIP_CHECK(hipMemsetAsync(L.stat.p, 0, sizeof(T) * L.vpad * L.kp, s));  // padded rows stay zero
  }
  if (presort) {
    HIP_CHECK(hipStreamWaitEvent(s, L.ev_sorted, 0));
  } else if (E > 0) {
    size_t tb = L.sort_tmp.bytes;
    HIP_CHECK(term_sort(L.sort_tmp.p, tb, L.keys.as<uint32_t>(), L.skeys.as<uint32_t>(), L.vals.as<uint64_t>(),
                        L.svals.as<uint64_t>(), E, bits_for(L.V), s));
  }
  const lda::StatMap lay = split ? stat_layout(L) : lda::StatMap{};
  if (lay.nsub <= 1) {
    lda::launch_sstats<T>(s, L.skeys.as<uint32_t>(), L.svals.as<uint64_t>(), E, L.r.as<T>(), L.eth.as<T>(), L.kp,
                          L.stat.as<T>(), L.headbuf.as<T>(), L.tailbuf.as<T>(), lda::StatMap{},
                          L.step_stamped ? L.rowstamp.as<int32_t>() : nullptr, L.step_sid);
  } else {
    for (int j = 0; j < lay.nsub; ++j) {
      lda::StatMap m = lay;
      m.sub = j;
      lda::launch_sstats<T>(s, L.skeys.as<uint32_t>(), L.svals.as<uint64_t>(), E, L.r.as<T>(), L.eth.as<T>(),
                            L.kp, L.stat.as<T>(), L.headbuf.as<T>(), L.tailbuf.as<T>(), m);
      if (!L.ev_ss[j]) HIP_CHECK(hipEventCreateWithFlags(&L.ev_ss[j], hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(L.ev_ss[j], s));
    }
  }
  record(L, 3);
}

// the fused M-step pass over one vocabulary slice r, rows [r·Vs, r·Vs + vn): λ update, the next
// expElogβ' rows + logscale, and colsum partials at λ-update block r·Vs/RB, where the one-GPU
// reduction has them.  Nothing in it needs the new colsum (ψ(colsum) is the E-step's per-topic factor).
template <typename T>
void mstep_slice(stc_lda& L, int r, double rho, double scale, const double* gate) {
  const int64_t v0 = (int64_t)r * L.Vs, vn = std::max<int64_t>(0, std::min(L.V - v0, L.Vs));
  const int64_t nbs = L.Vs / lda::kRowsPerBlock;
  lda::launch_lambda_eeb<T>(L.ctx->stream, true, L.lam.as<double>() + v0 * L.k, L.stat.as<T>() + v0 * L.kp,
                            L.Bp.as<T>() + v0 * L.kp, L.logscale.as<double>() + v0, vn, L.k, L.kp, rho, scale,
                            L.eta, gate, L.colpart.as<double>() + (int64_t)r * nbs * L.k, nbs,
                            L.mixed ? L.Bp64.as<double>() + v0 * L.kp : nullptr,
                            L.step_stamped ? L.rowstamp.as<int32_t>() + v0 : nullptr, L.step_sid);
}
// the same pass over sub-chunk j of slice r, whose summed stat rows sit at the sub-chunk layout's
// physical rows (stat_layout); λ / expElogβ' / logscale / colsum partials at their canonical rows
template <typename T>
void mstep_sub(stc_lda& L, const lda::StatMap& m, int r, int j, double rho, double scale, const double* gate) {
  const auto [off, w] = stat_sub_rows(m, j);
  const int64_t v0 = (int64_t)r * L.Vs + off, vn = std::max<int64_t>(0, std::min(L.V - v0, w));
  const int64_t phys = (int64_t)m.n * j * m.vsj + (int64_t)r * w;
  lda::launch_lambda_eeb<T>(L.ctx->stream, true, L.lam.as<double>() + v0 * L.k, L.stat.as<T>() + phys * L.kp,
                            L.Bp.as<T>() + v0 * L.kp, L.logscale.as<double>() + v0, vn, L.k, L.kp, rho, scale,
                            L.eta, gate, L.colpart.as<double>() + (v0 / lda::kRowsPerBlock) * L.k,
                            w / lda::kRowsPerBlock, L.mixed ? L.Bp64.as<double>() + v0 * L.kp : nullptr);
}

// [U] submitMiniBatch tail: the stats merge (treeReduce ≙ RCCL), updateLambda, updateAlpha.
//  * one GPU: the fused λ update + expElogβ' pass over all rows, then colsum and ψ(colsum).
//  * N ranks: reduce-scatter of stat (each rank receives the summed rows of its vocabulary slice) and
//    the logphat / count all-reduce in one group; the slice's fused λ update + expElogβ' pass; ONE
//    group of all-gathers — the per-block colsum partials (k doubles per 64 rows), expElogβ' and
//    logscale — then colsum reduced in the one-GPU block order, so it is identical on every rank.
//    λ stays sharded (lam_stale) until a reader gathers it.  Per rank: stat (N−1)/N·V·kp·T bytes
//    out, expElogβ' the same in, against 2(N−1)/N for an all-reduce, and 1/N of the M-step work.
template <typename T>
void train_tail_split(stc_lda& L, const lda::StatMap& lay, bool had_samp, int64_t n, int64_t E,
                      stc_step_stats* st);
template <typename T>
void train_finish(stc_lda& L, int64_t n, int64_t E, stc_step_stats* st);

//  * N ranks with rs_chunks > 1 (stat_layout: nsub sub-chunks): sstats ran once per sub-chunk
//    (estep_and_stats split) and recorded ev_ss[j]; the reduce-scatter of sub-chunk j (one contiguous
//    buffer in that layout) runs on cstream as soon as ev_ss[j] fires — under the sstats launches of
//    j+1… — with the logphat / count all-reduce in sub-chunk 0's group, and the main stream runs the
//    M-step of sub-chunk j under the reduce-scatter of j+1.  Each element is summed over the same
//    ranks in the same way as by the single reduce-scatter, and sstats builds every row exactly as
//    the single launch does, so the result is the unchunked step's.
template <typename T>
void train_tail(stc_lda& L, int64_t n, int64_t E, stc_step_stats* st) {
  Ctx& c = *L.ctx;
  hipStream_t s = c.stream;
  const bool ranks = sharded(L);
  const lda::StatMap lay = stat_layout(L);
  if (L.tail_fault > 0 && --L.tail_fault == 0) {
    throw Error(STC_ERR_STATE, "injected member failure between sstats and the reduce-scatter (STC_GROUP_STEP_FAULT)");
  }
  const bool had_samp = L.samp_pending;
  if (L.samp_pending) {  // the next draw's counts (side stream) feed this step's collective / readback
    HIP_CHECK(hipStreamWaitEvent(s, L.ev_samp, 0));
    L.samp_pending = false;
  }
  if (ranks && lay.nsub > 1) {
    train_tail_split<T>(L, lay, had_samp, n, E, st);
    return;
  }
  if (c.coll()) {
    coll_group_start(c);
    if (ranks) {
      const size_t cnt = (size_t)(L.Vs * L.kp);
      coll_reduce_scatter(c, L.stat.p, L.stat.as<T>() + (size_t)c.rank * cnt, cnt, RcclType<T>::v, s);
    }
    coll_all_reduce(c, L.small.p, (size_t)(L.k + 1), ncclFloat64, s);
    if (L.pre_inflight)  // the next draw's global batch size (word 3), for the next call
      coll_all_reduce(c, L.dcnt.as<int64_t>() + 3, 1, ncclInt64, s);
    coll_group_end(c);
  }
  if (L.pre_inflight) {
    HIP_CHECK(hipMemcpyAsync(L.hpre, L.dcnt.p, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipEventRecord(L.ev_pre, s));
    L.pre_inflight = false;
    L.pre_valid = true;
  }
  record(L, 4);
  L.iteration += 1;
  const double rho = std::pow(L.cfg.tau0 + (double)L.iteration, -L.cfg.kappa);
  const double batch_size = std::ceil(L.cfg.mini_batch_fraction * (double)L.corpus_total);
  const double scale = (double)L.corpus_total / batch_size;
  const double* gate = L.small.as<double>() + L.k;
  const int64_t nb_all = L.shards * (L.Vs / lda::kRowsPerBlock);
  if (ranks) {
    const size_t nbs = (size_t)(L.Vs / lda::kRowsPerBlock);
    mstep_slice<T>(L, c.rank, rho, scale, gate);
    const size_t cnt = (size_t)(L.Vs * L.kp);
    coll_group_start(c);
    coll_all_gather(c, L.colpart.as<double>() + (size_t)c.rank * nbs * L.k, L.colpart.p, nbs * L.k, ncclFloat64, s);
    coll_all_gather(c, L.Bp.as<T>() + (size_t)c.rank * cnt, L.Bp.p, cnt, RcclType<T>::v, s);
    if (L.mixed) coll_all_gather(c, L.Bp64.as<double>() + (size_t)c.rank * cnt, L.Bp64.p, cnt, ncclFloat64, s);
    coll_all_gather(c, L.logscale.as<double>() + (size_t)c.rank * L.Vs, L.logscale.p, (size_t)L.Vs, ncclFloat64, s);
    coll_group_end(c);
    lda::launch_colsum_reduce(s, L.colpart.as<double>(), nb_all, L.k, gate, L.colsum.as<double>(),
                              L.psic.as<double>());
    L.lam_stale = true;
  } else {  // one GPU: all slices here (one unless STC_VIRTUAL_SHARDS)
    for (int r = 0; r < L.shards; ++r) mstep_slice<T>(L, r, rho, scale, gate);
    lda::launch_colsum_reduce(s, L.colpart.as<double>(), nb_all, L.k, gate, L.colsum.as<double>(),
                              L.psic.as<double>());
  }
  if (L.cfg.optimize_doc_concentration)
    lda::launch_update_alpha(s, L.alpha.as<double>(), L.small.as<double>(), L.k, rho);
  train_finish<T>(L, n, E, st);
}

template <typename T>
void train_tail_split(stc_lda& L, const lda::StatMap& lay, bool had_samp, int64_t n, int64_t E,
                      stc_step_stats* st) {
  Ctx& c = *L.ctx;
  hipStream_t s = c.stream;
  if (!L.cstream) HIP_CHECK(hipStreamCreateWithFlags(&L.cstream, hipStreamNonBlocking));
  hipStream_t cs = L.cstream;
  if (had_samp) HIP_CHECK(hipStreamWaitEvent(cs, L.ev_samp, 0));  // the next draw's count (side stream)
  for (int j = 0; j < lay.nsub; ++j) {
    if (!L.ev_rs[j]) HIP_CHECK(hipEventCreateWithFlags(&L.ev_rs[j], hipEventDisableTiming));
    HIP_CHECK(hipStreamWaitEvent(cs, L.ev_ss[j], 0));
    const int64_t w = stat_sub_rows(lay, j).second;
    T* chunk = L.stat.as<T>() + (int64_t)lay.n * j * lay.vsj * L.kp;
    coll_group_start(c);
    coll_reduce_scatter(c, chunk, chunk + (int64_t)c.rank * w * L.kp, (size_t)(w * L.kp), RcclType<T>::v, cs);
    if (j == 0) {
      coll_all_reduce(c, L.small.p, (size_t)(L.k + 1), ncclFloat64, cs);
      if (L.pre_inflight) coll_all_reduce(c, L.dcnt.as<int64_t>() + 3, 1, ncclInt64, cs);
    }
    coll_group_end(c);
    if (j == 0 && L.pre_inflight) {
      HIP_CHECK(hipMemcpyAsync(L.hpre, L.dcnt.p, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, cs));
      HIP_CHECK(hipEventRecord(L.ev_pre, cs));
      L.pre_inflight = false;
      L.pre_valid = true;
    }
    HIP_CHECK(hipEventRecord(L.ev_rs[j], cs));
  }
  L.iteration += 1;
  const double rho = std::pow(L.cfg.tau0 + (double)L.iteration, -L.cfg.kappa);
  const double batch_size = std::ceil(L.cfg.mini_batch_fraction * (double)L.corpus_total);
  const double scale = (double)L.corpus_total / batch_size;
  const double* gate = L.small.as<double>() + L.k;
  for (int j = 0; j < lay.nsub; ++j) {
    HIP_CHECK(hipStreamWaitEvent(s, L.ev_rs[j], 0));
    if (j == 0) record(L, 4);  // the statistics of sub-chunk 0 and the logphat / count sums are in
    mstep_sub<T>(L, lay, c.rank, j, rho, scale, gate);
  }
  const size_t nbs = (size_t)(L.Vs / lda::kRowsPerBlock), cnt = (size_t)(L.Vs * L.kp);
  coll_group_start(c);
  coll_all_gather(c, L.colpart.as<double>() + (size_t)c.rank * nbs * L.k, L.colpart.p, nbs * L.k, ncclFloat64, s);
  coll_all_gather(c, L.Bp.as<T>() + (size_t)c.rank * cnt, L.Bp.p, cnt, RcclType<T>::v, s);
  if (L.mixed) coll_all_gather(c, L.Bp64.as<double>() + (size_t)c.rank * cnt, L.Bp64.p, cnt, ncclFloat64, s);
  coll_all_gather(c, L.logscale.as<double>() + (size_t)c.rank * L.Vs, L.logscale.p, (size_t)L.Vs, ncclFloat64, s);
  coll_group_end(c);
  lda::launch_colsum_reduce(s, L.colpart.as<double>(), L.shards * (int64_t)nbs, L.k, gate, L.colsum.as<double>(),
                            L.psic.as<double>());
  L.lam_stale = true;
  if (L.cfg.optimize_doc_concentration)
    lda::launch_update_alpha(s, L.alpha.as<double>(), L.small.as<double>(), L.k, rho);
  train_finish<T>(L, n, E, st);
}

template <typename T>
void train_finish(stc_lda& L, int64_t n, int64_t E, stc_step_stats* st) {
  hipStream_t s = L.ctx->stream;
  record(L, 5);
  if (L.timing) {
    L.ev_pending[L.ev_set] = true;
    L.ev_set = (L.ev_set + 1) % 3;
  }
  L.cum_docs += n;
  L.cum_entries += E;
  if (st) {
    int64_t h4[4] = {0, 0, 0, 0};
    double ne = 0.0;
    // a copy to pageable memory can block in the runtime: behind collectives, wait (polling) first
    if (L.ctx->comm) wait_stream(*L.ctx, s);
    HIP_CHECK(hipMemcpyAsync(h4, L.stats4.p, sizeof(h4), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(&ne, L.small.as<double>() + L.k, sizeof(double), hipMemcpyDeviceToHost, s));
    wait_stream(*L.ctx, s);
    st->batch_docs = n;
    st->batch_entries = E;
    st->inner_iters = h4[0];
    st->inner_iters_max = (int32_t)h4[1];
    st->cap_hits = (int32_t)h4[2];
    st->nonempty_docs = (int64_t)ne;
    st->rho = std::pow(L.cfg.tau0 + (double)L.iteration, -L.cfg.kappa);
  }
}

void require_ready(stc_lda& L) {
  if (!L.corpus) throw Error(STC_ERR_STATE, "no corpus: call stc_lda_set_corpus first");
  if (!L.has_topics) throw Error(STC_ERR_STATE, "no topics: call stc_lda_init_random or stc_lda_set_topics");
}

// host-injected membership → partitioned slots on the device; returns the partition
template <typename T>
Part upload_members(stc_lda& L, const int64_t* ids, int64_t n) {
  std::vector<int32_t> h((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    STC_REQUIRE(ids[i] >= 0 && ids[i] < L.corpus->rows, "batch doc id out of range");
    h[(size_t)i] = (int32_t)ids[i];
  }
  ensure_batch<T>(L, n, 0);
  if (n > 0)
    HIP_CHECK(hipMemcpyAsync(L.batch_raw.p, h.data(), 4 * n, hipMemcpyHostToDevice, L.ctx->stream));
  Part p = partition(L, L.corpus->indptr.as<int64_t>(), L.batch_raw.as<int32_t>(), n);  // syncs
  ensure_batch<T>(L, n, p.E);
  slot_offsets(L, n);
  return p;
}

template <typename T>
void step_ids(stc_lda& L, const int64_t* ids, int64_t n, const double* gamma0, stc_step_stats* st) {
  require_ready(L);
  relayout(L);
  ensure_order(L);
  claim_event_set(L);
  record(L, 0);
  const Part p = upload_members<T>(L, ids, n);
  if (L.timing) harvest_all(L);  // partition() drained the stream
  const T* g0 = upload_gamma0<T>(L, gamma0, n);
  if (!g0) g0 = gen_gamma0<T>(L, L.ctx->stream, n, L.cfg.seed, L.iteration + 1, 0, 0);
  estep_and_stats<T>(L, n, p.n_short, p.E, g0, L.iteration + 1, true, mixed_gamma0(L, gamma0, n));
  train_tail<T>(L, n, p.E, st);
}

// A call that failed after queuing the next draw on the side stream (before train_tail ordered the main
// stream behind it) leaves that draw in flight: wait for it and drop it, so nothing samples into the same
// count buffers concurrently and the next call draws synchronously.
void settle_side(stc_lda& L) {
  if (!L.samp_pending) return;
  L.ctx->use();
  wait_stream(*L.ctx, L.side);
  L.samp_pending = false;
  L.pre_inflight = false;
  L.pre_valid = false;
}

// sample draw `draw` on the device: per-doc counts (Poisson / Bernoulli), their scans, and (n, E,
// n_short) into dcnt words 0–2, word 3 = n (all-reduced to the global n by the caller)
void sample_draw(stc_lda& L, int64_t draw, hipStream_t s, DevBuf* tmp) {
  Ctx& c = *L.ctx;
  const int64_t D = L.corpus->rows;
  if (D > 0) {
    lda::launch_sample(s, L.corpus->indptr.as<int64_t>(), D, L.cfg.mini_batch_fraction,
                       L.cfg.sample_with_replacement, L.cfg.seed, draw, c.rank, L.wave_cap,
                       L.s_counts.as<int32_t>(), L.s_weights.as<int64_t>(), L.s_short.as<int32_t>());
    incl_scan<int32_t>(L, L.s_counts.as<int32_t>(), L.s_cincl.as<int32_t>(), D, s, tmp);
    incl_scan<int64_t>(L, L.s_weights.as<int64_t>(), L.s_wincl.as<int64_t>(), D, s, tmp);
    incl_scan<int32_t>(L, L.s_short.as<int32_t>(), L.s_sincl.as<int32_t>(), D, s, tmp);
    // (n, E, n_short) from the scans' last elements: one kernel packs them, one copy to pinned memory
    lda::launch_last3(s, L.s_cincl.as<int32_t>() + (D - 1), L.s_wincl.as<int64_t>() + (D - 1),
                      L.s_sincl.as<int32_t>() + (D - 1), L.dcnt.as<int64_t>());
  } else {  // a rank without documents still takes part in every collective
    HIP_CHECK(hipMemsetAsync(L.dcnt.p, 0, 3 * sizeof(int64_t), s));
  }
  HIP_CHECK(hipMemcpyAsync(L.dcnt.as<int64_t>() + 3, L.dcnt.p, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
}

// [U] OnlineLDAOptimizer.next(): sample a minibatch (device-side), `if (batch.isEmpty()) return this`
// on the GLOBAL batch, else submitMiniBatch.  Draw d's membership is sampled while step d−1 runs
// (after its fill_batch, so the count buffers are free) and its global size is all-reduced with
// step d−1's statistics; the host then waits only on that collective's event — the GPU is still
// busy with step d−1's M-step when step d is enqueued.  The first draw (or one after an empty
// batch, set_corpus or init_random) is sampled and counted synchronously.
template <typename T>
void next_impl(stc_lda& L, stc_step_stats* st) {
  require_ready(L);
  settle_side(L);
  relayout(L);
  ensure_order(L);
  Ctx& c = *L.ctx;
  hipStream_t s = c.stream;
  const int64_t D = L.corpus->rows;
  L.s_counts.reserve(4 * D);
  L.s_weights.reserve(8 * D);
  L.s_short.reserve(4 * D);
  L.s_cincl.reserve(4 * D);
  L.s_wincl.reserve(8 * D);
  L.s_sincl.reserve(4 * D);
  if (!L.hcnt) HIP_CHECK(hipHostMalloc((void**)&L.hcnt, 4 * sizeof(int64_t), hipHostMallocDefault));
  if (!L.hpre) HIP_CHECK(hipHostMalloc((void**)&L.hpre, 4 * sizeof(int64_t), hipHostMallocDefault));
  if (!L.ev_pre) HIP_CHECK(hipEventCreateWithFlags(&L.ev_pre, hipEventDisableTiming));
  L.dcnt.reserve(4 * sizeof(int64_t));
  const int64_t draw = ++L.draws;
  claim_event_set(L);
  record(L, 0);
  int64_t cnt[4];
  // the prefetched draw's batch is built on the side stream (behind its sampling, and behind the previous
  // step's E-step — ev_est), under the previous step's M-step and all-gathers
  const bool prefetched = L.pre_valid && L.pre_draw == draw;
  const bool on_side = prefetched && L.prep_side && L.side && L.ev_est;
  if (prefetched) {
    wait_event(*L.ctx, L.ev_pre);
    std::copy(L.hpre, L.hpre + 4, cnt);
  } else {
    sample_draw(L, draw, s, &L.scan_tmp);
    if (c.coll()) coll_all_reduce(c, L.dcnt.as<int64_t>() + 3, 1, ncclInt64, s);
    HIP_CHECK(hipMemcpyAsync(L.hcnt, L.dcnt.p, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    wait_stream(*L.ctx, s);
    std::copy(L.hcnt, L.hcnt + 4, cnt);
  }
  L.pre_valid = false;
  const int64_t n = cnt[0], E = cnt[1], ns32 = cnt[2], n_global = cnt[3];
  if (L.timing) harvest_all(L);
  // Spark's next(): `if (batch.isEmpty()) return this` — no iteration increment
  if (n_global == 0) {
    if (st) *st = stc_step_stats{};
    return;
  }
  ensure_batch<T>(L, n, E, true);
  const hipStream_t ps = on_side ? L.side : s;
  if (on_side) HIP_CHECK(hipStreamWaitEvent(ps, L.ev_est, 0));
  if (n > 0)
    lda::launch_fill_batch(ps, L.corpus->indptr.as<int64_t>(), D, L.wave_cap, L.s_counts.as<int32_t>(),
                           L.s_cincl.as<int32_t>(), L.s_sincl.as<int32_t>(), ns32, L.batch.as<int32_t>(),
                           L.orig.as<int32_t>(), L.nnzp.as<int64_t>());
  order_slots(L, ns32, ps);
  slot_offsets(L, n, ps, on_side ? &L.side_scan_tmp : &L.scan_tmp);
  const T* g0 = gen_gamma0<T>(L, ps, n, L.cfg.seed, L.iteration + 1, 0, 0);
  // the next draw, on the side stream beside this step's E-step, counted with this step's collective
  if (!L.side) {
    HIP_CHECK(hipStreamCreateWithFlags(&L.side, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&L.ev_fill, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&L.ev_samp, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&L.ev_est, hipEventDisableTiming));
  }
  HIP_CHECK(hipEventRecord(L.ev_fill, ps));  // this draw's counts consumed and its batch built
  if (on_side) HIP_CHECK(hipStreamWaitEvent(s, L.ev_fill, 0));
  else HIP_CHECK(hipStreamWaitEvent(L.side, L.ev_fill, 0));
  sample_draw(L, draw + 1, L.side, &L.side_scan_tmp);
  HIP_CHECK(hipEventRecord(L.ev_samp, L.side));
  L.samp_pending = true;
  L.pre_draw = draw + 1;
  if (c.coll()) {
    L.pre_inflight = true;  // the global size rides on this step's collective (train_tail reads it back)
  } else {
    // one rank: the draw's size is already global — read it back on the side stream as soon as it is sampled
    // (during this step's E-step), so the next call enqueues its batch preparation at once and the side stream
    // builds it under this step's sstats and M-step; read back in train_tail, after the E-step and sstats, the
    // preparation only started under the M-step and the next E-step waited for it (the "sample" phase, 0.29 ms)
    HIP_CHECK(hipMemcpyAsync(L.hpre, L.dcnt.p, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, L.side));
    HIP_CHECK(hipEventRecord(L.ev_pre, L.side));
    L.pre_inflight = false;
    L.pre_valid = true;
  }
  estep_and_stats<T>(L, n, ns32, E, g0, L.iteration + 1, true);
  train_tail<T>(L, n, E, st);
  L.prep_side = true;
}

template <typename T>
void estep_only(stc_lda& L, const int64_t* ids, int64_t n, const double* gamma0, double* gamma_out,
                double* stat_out, int32_t* iters_out) {
  require_ready(L);
  relayout(L);
  ensure_order(L);
  hipStream_t s = L.ctx->stream;
  const Part p = upload_members<T>(L, ids, n);
  // γ₀ drawn inside the E-step kernel when not injected (no n×k buffer: ADVICE r5); the pre-drawn form
  // (gen_gamma0) is used only by the training steps, where it was measured to help
  const T* g0 = upload_gamma0<T>(L, gamma0, n);
  const bool t = L.timing;
  L.timing = false;
  estep_and_stats<T>(L, n, p.n_short, p.E, g0, L.iteration + 1, false, mixed_gamma0(L, gamma0, n), gamma_out != nullptr);
  L.timing = t;
  if (gamma_out && n > 0) {
    std::vector<T> g((size_t)(n * L.k));
    HIP_CHECK(hipMemcpyAsync(g.data(), L.gamma.p, sizeof(T) * g.size(), hipMemcpyDeviceToHost, s));
    wait_stream(*L.ctx, s);
    for (size_t j = 0; j < g.size(); ++j) gamma_out[j] = (double)g[j];
  }
  if (iters_out && n > 0) {
    HIP_CHECK(hipMemcpyAsync(iters_out, L.iters.p, 4 * n, hipMemcpyDeviceToHost, s));
  }
  if (stat_out) {
    L.dtmp.reserve(sizeof(double) * L.V * L.k);
    lda::launch_unscale_stat<T>(s, L.stat.as<T>(), L.logscale.as<double>(), L.psic.as<double>(), L.V, L.k, L.kp,
                                L.dtmp.as<double>());
    HIP_CHECK(hipMemcpyAsync(stat_out, L.dtmp.p, sizeof(double) * L.V * L.k, hipMemcpyDeviceToHost, s));
  }
  wait_stream(*L.ctx, s);
}

template <typename T>
void infer_impl(stc_lda& L, const DCsr& docs, uint64_t seed, int64_t base, const double* gamma0,
                bool bound, double* gamma_out, double* out4 /* corpus, tokens */) {
  if (!L.has_topics) throw Error(STC_ERR_STATE, "no topics: call stc_lda_init_random or stc_lda_set_topics");
  STC_REQUIRE(docs.cols == L.V, "document vectors must have vocab_size columns");
  STC_REQUIRE(docs.dtype == corpus_dtype(L), "document CSR dtype must match the LDA dtype (STC_F64 for STC_MIXED)");
  hipStream_t s = L.ctx->stream;
  const int64_t n = docs.rows;
  ensure_batch<T>(L, n, 0);
  L.r.reserve(sizeof(T) * std::max<int64_t>(docs.nnz, 1));
  L.bound.reserve(sizeof(double) * std::max<int64_t>(n, 1));
  L.scal.reserve(sizeof(double) * 8);
  const Part p = partition(L, docs.indptr.as<int64_t>(), nullptr, n);
  const T* g0 = upload_gamma0<T>(L, gamma0, n);  // nullptr: drawn inside the E-step kernel (as estep_only)
  lda::EStepArgs<T> a = estep_args<T>(L);
  a.indptr = docs.indptr.as<int64_t>();
  a.indices = docs.indices.as<int32_t>();
  a.values = docs.values.as<T>();
  a.batch = L.batch.as<int32_t>();
  a.orig = L.orig.as<int32_t>();
  a.bptr = nullptr;  // entry slots = the rows' CSR positions
  a.gamma0 = g0;
  a.seed = seed;
  a.key_mode = 1;
  a.doc_id_base = base;
  a.r = L.r.as<T>();
  a.gamma = gamma_out ? L.gamma.as<T>() : nullptr;
  a.iters = L.iters.as<int32_t>();
  a.bound = bound ? L.bound.as<double>() : nullptr;
  launch_split<T>(L, docs, a, n, p.n_short, false, bound, n > 0 ? (double)docs.nnz / (double)n : 0.0);
  if (gamma_out && n > 0) {
    std::vector<T> g((size_t)(n * L.k));
    HIP_CHECK(hipMemcpyAsync(g.data(), L.gamma.p, sizeof(T) * g.size(), hipMemcpyDeviceToHost, s));
    wait_stream(*L.ctx, s);
    for (size_t j = 0; j < g.size(); ++j) gamma_out[j] = (double)g[j];
  }
  if (bound) {
    double h[3] = {0, 0, 0};
    HIP_CHECK(hipMemsetAsync(L.scal.p, 0, sizeof(double) * 3, s));
    if (n > 0) lda::launch_sum_f64(s, L.bound.as<double>(), n, L.scal.as<double>());
    if (docs.nnz > 0) lda::launch_sum_vals<T>(s, docs.values.as<T>(), docs.nnz, L.scal.as<double>() + 1);
    HIP_CHECK(hipMemcpyAsync(h, L.scal.p, sizeof(double) * 2, hipMemcpyDeviceToHost, s));
    wait_stream(*L.ctx, s);
    out4[0] = h[0];
    out4[1] = h[1];
  }
}

// the full λ on every rank after sharded M-steps: an all-gather of the slices (collective — every
// rank calls the reader, as every executor calls ldaNext)
void gather_lambda(stc_lda& L) {
  if (!L.lam_stale) return;
  Ctx& c = *L.ctx;
  const size_t cnt = (size_t)(L.Vs * L.k);
  coll_all_gather(c, L.lam.as<double>() + (size_t)c.rank * cnt, L.lam.p, cnt, ncclFloat64, c.stream);
  wait_stream(c, c.stream);
  L.lam_stale = false;
}

// [U] logLikelihoodBound topicsPart: the per-element sum over the rows this rank holds current (its
// slice when λ is sharded — the caller all-reduces it — else all rows), and separately the
// per-topic normaliser terms Σ_k (lgamma(η·V) − lgamma(Σ_v λ_vk)) from the global colsum (added once).
template <typename T>
void topics_part(stc_lda& L, double* elem_part, double* norm_part) {
  hipStream_t s = L.ctx->stream;
  const int64_t nb = 1024;
  L.dtmp.reserve(sizeof(double) * (nb + 1));
  L.scal.reserve(sizeof(double) * 8);
  int64_t v0 = 0, vn = L.V;
  if (L.lam_stale) {
    v0 = (int64_t)L.ctx->rank * L.Vs;
    vn = std::max<int64_t>(0, std::min(L.V - v0, L.Vs));
  }
  HIP_CHECK(hipMemsetAsync(L.dtmp.p, 0, sizeof(double) * nb, s));
  if (vn > 0)
    lda::launch_topics_bound<T>(s, L.lam.as<double>() + v0 * L.k, L.colsum.as<double>(), vn, L.k, L.eta,
                                L.dtmp.as<double>(), nb);
  lda::launch_sum_f64(s, L.dtmp.as<double>(), nb, L.scal.as<double>() + 3);
  double part = 0.0;
  std::vector<double> cs((size_t)L.k);
  HIP_CHECK(hipMemcpyAsync(&part, L.scal.as<double>() + 3, sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(cs.data(), L.colsum.p, sizeof(double) * L.k, hipMemcpyDeviceToHost, s));
  wait_stream(*L.ctx, s);
  // sumEta = η·V (Dirichlet normaliser of q(β_k|λ_k) minus that of p(β_k|η))
  const double lg_sum_eta = std::lgamma(L.eta * (double)L.V);
  double norm = 0.0;
  for (int t = 0; t < L.k; ++t) norm += lg_sum_eta - std::lgamma(cs[(size_t)t]);
  *elem_part = part;
  *norm_part = norm;
}

void allreduce_host(Ctx& c, double* x, int64_t n) {
  if (!c.coll() || n == 0) return;
  DevBuf d;
  d.reserve(sizeof(double) * n);
  HIP_CHECK(hipMemcpyAsync(d.p, x, sizeof(double) * n, hipMemcpyHostToDevice, c.stream));
  coll_all_reduce(c, d.p, (size_t)n, ncclFloat64, c.stream);
  HIP_CHECK(hipMemcpyAsync(x, d.p, sizeof(double) * n, hipMemcpyDeviceToHost, c.stream));
  wait_stream(c, c.stream);
}

void check_csr_host(int64_t rows, int64_t cols, const int64_t* indptr, const int32_t* indices) {
  STC_REQUIRE(rows >= 0 && cols > 0, "csr: rows >= 0 and cols > 0");
  STC_REQUIRE(cols <= (int64_t(1) << 31), "csr: at most 2^31 columns");
  STC_REQUIRE(indptr[0] == 0, "csr: indptr[0] must be 0");
  for (int64_t r = 0; r < rows; ++r) STC_REQUIRE(indptr[r + 1] >= indptr[r], "csr: indptr must be non-decreasing");
  const int64_t nnz = indptr[rows];
  for (int64_t e = 0; e < nnz; ++e)
    STC_REQUIRE(indices[e] >= 0 && (int64_t)indices[e] < cols, "csr: column index out of range");
}

}  // namespace

// =======================================================================================
// C ABI
// =======================================================================================
extern "C" {

const char* stc_last_error(void) { return stc::g_last_error.c_str(); }
int stc_abi_version(void) { return STC_ABI_VERSION; }

int stc_device_count(int* n_out) {
  return guard([&] {
    STC_REQUIRE(n_out, "n_out");
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    *n_out = n;
  });
}

int stc_init(int device, stc_ctx** out) {
  return guard([&] {
    STC_REQUIRE(out, "out");
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    STC_REQUIRE(device >= 0 && device < n, "device index out of range");
    auto c = std::make_unique<stc_ctx>();
    c->device = device;
    HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_CHECK(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device));
    {
      std::lock_guard<std::mutex> lk(g_live_mu);
      g_live.insert(c.get());
    }
    const char* db = std::getenv("STC_DF_BINNED");  // A/B knob: the round-3 binned df count
    c->df_tiled = !(db && db[0] == '1');
    const char* d32 = std::getenv("STC_DF_U32");  // A/B knob: the u32 tiled count for unique-id rows too
    c->df_rows16 = !(d32 && d32[0] == '1');
    const char* tm = std::getenv("STC_TF_MODE");  // A/B knob: HashingTF's structure (stc_internal.h Ctx)
    if (tm && tm[0] >= '0' && tm[0] <= '2' && tm[1] == 0) c->tf_mode = tm[0] - '0';
    const char* tf = std::getenv("STC_TF_FAULT");  // test knob
    c->tf_force_fault = tf && tf[0] == '1';
    const char* ct = std::getenv("STC_COLL_TIMEOUT_MS");  // the deadline of a wait behind RCCL collectives
    if (ct && std::atoll(ct) > 0) c->coll_timeout_ms = std::atoll(ct);
    const char* nc = std::getenv("STC_IDF_NO_CACHE");  // A/B knob: plain idf gathers in the transform
    c->idf_cache = !(nc && nc[0] == '1');
    *out = c.release();
  });
}

int stc_destroy(stc_ctx* ctx) {
  return guard([&] {
    if (!ctx) return;
    {
      std::lock_guard<std::mutex> lk(g_live_mu);
      g_live.erase(ctx);
    }
    (void)hipSetDevice(ctx->device);
    // an aborted communicator is already freed; a live one is destroyed (a group's members first settle
    // their streams in stc_group_destroy, so nothing of it is still queued)
    if (ctx->comm && !ctx->comm_aborted.load()) (void)ncclCommDestroy(ctx->comm);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
  });
}

int stc_synchronize(stc_ctx* ctx) {
  return guard([&] {
    STC_REQUIRE(ctx, "ctx");
    ctx->use();
    wait_stream(*ctx, ctx->stream);
  });
}

int stc_comm_unique_id(uint8_t id_out[128]) {
  return guard([&] {
    STC_REQUIRE(id_out, "id_out");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    RCCL_CHECK(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, 128);
  });
}

int stc_comm_init(stc_ctx* ctx, const uint8_t id[128], int n_ranks, int rank) {
  return guard([&] {
    STC_REQUIRE(ctx && id, "ctx/id");
    STC_REQUIRE(n_ranks >= 1 && rank >= 0 && rank < n_ranks, "rank / n_ranks");
    STC_REQUIRE(!ctx->comm, "communicator already initialised");
    ctx->use();
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    RCCL_CHECK(ncclCommInitRank(&ctx->comm, n_ranks, uid, rank));
    ctx->n_ranks = n_ranks;
    ctx->rank = rank;
  });
}

int stc_comm_allreduce_f64(stc_ctx* ctx, double* host_inout, int64_t n) {
  return guard([&] {
    STC_REQUIRE(ctx && (host_inout || n == 0), "ctx/host_inout");
    ctx->use();
    allreduce_host(*ctx, host_inout, n);
  });
}

int stc_dcsr_upload(stc_ctx* ctx, int64_t n_rows, int64_t n_cols, const int64_t* indptr,
                    const int32_t* indices, const double* values, int value_dtype, stc_dcsr** out) {
  return guard([&] {
    STC_REQUIRE(ctx && indptr && out, "ctx/indptr/out");
    STC_REQUIRE(value_dtype == STC_F32 || value_dtype == STC_F64, "value_dtype");
    const int64_t nnz = indptr[n_rows];
    STC_REQUIRE(nnz == 0 || (indices && values), "indices/values");
    check_csr_host(n_rows, n_cols, indptr, indices);
    ctx->use();
    auto m = std::make_unique<stc_dcsr>();
    m->ctx = ctx;
    m->device = ctx->device;
    m->rows = n_rows;
    m->cols = n_cols;
    m->nnz = nnz;
    m->dtype = value_dtype;
    m->max_row = 0;
    for (int64_t r = 0; r < n_rows; ++r) m->max_row = std::max(m->max_row, indptr[r + 1] - indptr[r]);
    ctx->recycle.take(m->indptr, 8 * (n_rows + 1));
    ctx->recycle.take(m->indices, 4 * std::max<int64_t>(nnz, 1));
    ctx->recycle.take(m->values, (value_dtype == STC_F32 ? 4 : 8) * std::max<int64_t>(nnz, 1));
    HIP_CHECK(hipMemcpyAsync(m->indptr.p, indptr, 8 * (n_rows + 1), hipMemcpyHostToDevice, ctx->stream));
    if (nnz > 0) {
      HIP_CHECK(hipMemcpyAsync(m->indices.p, indices, 4 * nnz, hipMemcpyHostToDevice, ctx->stream));
      if (value_dtype == STC_F64) {
        HIP_CHECK(hipMemcpyAsync(m->values.p, values, 8 * nnz, hipMemcpyHostToDevice, ctx->stream));
        wait_stream(*ctx, ctx->stream);
      } else {
        std::vector<float> f((size_t)nnz);
        for (int64_t e = 0; e < nnz; ++e) f[(size_t)e] = (float)values[e];
        HIP_CHECK(hipMemcpyAsync(m->values.p, f.data(), 4 * nnz, hipMemcpyHostToDevice, ctx->stream));
        wait_stream(*ctx, ctx->stream);
      }
    }
    wait_stream(*ctx, ctx->stream);
    *out = m.release();
  });
}

int stc_dcsr_shape(const stc_dcsr* m, int64_t* n_rows, int64_t* n_cols, int64_t* nnz) {
  return guard([&] {
    STC_REQUIRE(m, "m");
    if (n_rows) *n_rows = m->rows;
    if (n_cols) *n_cols = m->cols;
    if (nnz) *nnz = m->nnz;
  });
}

int stc_dcsr_download(stc_ctx* ctx, const stc_dcsr* m, int64_t* indptr, int32_t* indices, double* values) {
  return guard([&] {
    STC_REQUIRE(ctx && m, "ctx/m");
    STC_REQUIRE(m->ctx == ctx, "the matrix belongs to another stc_ctx");
    ctx->use();
    hipStream_t s = ctx->stream;
    if (indptr) HIP_CHECK(hipMemcpyAsync(indptr, m->indptr.p, 8 * (m->rows + 1), hipMemcpyDeviceToHost, s));
    if (indices && m->nnz) HIP_CHECK(hipMemcpyAsync(indices, m->indices.p, 4 * m->nnz, hipMemcpyDeviceToHost, s));
    if (values && m->nnz) {
      if (m->dtype == STC_F64) {
        HIP_CHECK(hipMemcpyAsync(values, m->values.p, 8 * m->nnz, hipMemcpyDeviceToHost, s));
      } else {
        std::vector<float> f((size_t)m->nnz);
        HIP_CHECK(hipMemcpyAsync(f.data(), m->values.p, 4 * m->nnz, hipMemcpyDeviceToHost, s));
        wait_stream(*ctx, s);
        for (int64_t e = 0; e < m->nnz; ++e) values[e] = f[(size_t)e];
      }
    }
    wait_stream(*ctx, s);
  });
}

int stc_dcsr_free(stc_dcsr* m) {
  return guard([&] {
    if (!m) return;
    if (m->device >= 0) (void)hipSetDevice(m->device);
    // every queued reader first — the context's stream and any other (an LDA handle's side stream sampling
    // from this corpus): a recycled buffer is rewritten by the next taker, so the implicit device
    // synchronisation hipFree gives is kept — outside the process-wide lock, so frees and
    // creates in other threads (a group's members, other devices) do not queue behind this drain
    if (m->device >= 0) (void)hipDeviceSynchronize();
    {  // hand the allocations back to the context that made it, if it still exists (Recycler)
      std::lock_guard<std::mutex> lk(g_live_mu);
      if (m->ctx && g_live.count(static_cast<stc_ctx*>(m->ctx)) && m->ctx->device == m->device) {
        m->ctx->recycle.put(m->indices);
        m->ctx->recycle.put(m->values);
        m->ctx->recycle.put(m->indptr);
      }
    }
    delete m;
  });
}

// ---- HashingTF ------------------------------------------------------------------------
namespace {
struct TokenUpload {
  DevBuf utf8, tok_off, doc_off;
  int64_t max_doc = -1;  // the longest document's token count (doc_off given), −1 unknown
};
void upload_tokens(Ctx& c, TokenUpload& u, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                   int64_t n_tok, const int64_t* doc_off, int64_t n_docs) {
  STC_REQUIRE(n_bytes >= 0 && n_tok >= 0 && n_docs >= 0, "sizes must be >= 0");
  STC_REQUIRE(tok_off && (n_bytes == 0 || utf8), "utf8/tok_off");
  STC_REQUIRE(tok_off[0] == 0 && tok_off[n_tok] <= n_bytes, "tok_off must start at 0 and stay within n_bytes");
  for (int64_t t = 0; t < n_tok; ++t) STC_REQUIRE(tok_off[t + 1] >= tok_off[t], "tok_off must be non-decreasing");
  if (doc_off) {
    STC_REQUIRE(doc_off[0] == 0 && doc_off[n_docs] == n_tok, "doc_off must span [0, n_tok]");
    u.max_doc = 0;
    for (int64_t d = 0; d < n_docs; ++d) {
      STC_REQUIRE(doc_off[d + 1] >= doc_off[d], "doc_off must be non-decreasing");
      u.max_doc = std::max<int64_t>(u.max_doc, doc_off[d + 1] - doc_off[d]);
    }
  }
  u.utf8.reserve(n_bytes + kHashPad);  // the hash reads 32-byte windows of whole aligned dwords
  u.tok_off.reserve(8 * (n_tok + 1));
  if (n_bytes) HIP_CHECK(hipMemcpyAsync(u.utf8.p, utf8, n_bytes, hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemcpyAsync(u.tok_off.p, tok_off, 8 * (n_tok + 1), hipMemcpyHostToDevice, c.stream));
  if (doc_off) {
    u.doc_off.reserve(8 * (n_docs + 1));
    HIP_CHECK(hipMemcpyAsync(u.doc_off.p, doc_off, 8 * (n_docs + 1), hipMemcpyHostToDevice, c.stream));
  }
}
}  // namespace

int stc_tokens_upload(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                      int64_t n_tok, const int64_t* doc_off, int64_t n_docs, stc_dtok** out) {
  return guard([&] {
    STC_REQUIRE(ctx && doc_off && out, "ctx/doc_off/out");
    ctx->use();
    auto t = std::make_unique<stc_dtok>();
    t->ctx = ctx;
    t->device = ctx->device;
    TokenUpload u;
    upload_tokens(*ctx, u, utf8, n_bytes, tok_off, n_tok, doc_off, n_docs);
    wait_stream(*ctx, ctx->stream);
    std::swap(t->utf8.p, u.utf8.p);
    std::swap(t->utf8.bytes, u.utf8.bytes);
    if (n_bytes + kHashPad <= (int64_t(1) << 32)) {  // u32 offsets: half the bytes HashingTF reads for them
      t->tok_off.reserve(4 * (n_tok + 1));
      hashing::narrow_offsets(*ctx, u.tok_off.as<int64_t>(), n_tok + 1, t->tok_off.as<uint32_t>());
      wait_stream(*ctx, ctx->stream);
      t->off32 = true;
    } else {
      std::swap(t->tok_off.p, u.tok_off.p);
      std::swap(t->tok_off.bytes, u.tok_off.bytes);
    }
    std::swap(t->doc_off.p, u.doc_off.p);
    std::swap(t->doc_off.bytes, u.doc_off.bytes);
    t->n_bytes = n_bytes;
    t->n_tok = n_tok;
    t->n_docs = n_docs;
    t->max_doc = u.max_doc;
    *out = t.release();
  });
}

int stc_tokens_free(stc_dtok* t) {
  return guard([&] {
    if (!t) return;
    if (t->device >= 0) (void)hipSetDevice(t->device);
    delete t;
  });
}

int stc_hashing_tf_tokens(stc_ctx* ctx, const stc_dtok* tokens, int32_t num_features, int binary,
                          int hash_variant, int value_dtype, stc_dcsr** out) {
  return guard([&] {
    STC_REQUIRE(ctx && tokens && out, "ctx/tokens/out");
    STC_REQUIRE(tokens->ctx == ctx, "tokens were uploaded on another stc_ctx");
    STC_REQUIRE(num_features > 0, "numFeatures must be > 0");
    STC_REQUIRE(hash_variant == STC_HASH_STANDARD || hash_variant == STC_HASH_SPARK24, "hash_variant");
    STC_REQUIRE(value_dtype == STC_F32 || value_dtype == STC_F64, "value_dtype");
    ctx->use();
    auto m = std::make_unique<stc_dcsr>();
    m->ctx = ctx;
    m->device = ctx->device;
    hashing::build_csr(*ctx, tokens->utf8.as<uint8_t>(), tokens->off32 ? nullptr : tokens->tok_off.as<int64_t>(),
                       tokens->off32 ? tokens->tok_off.as<uint32_t>() : nullptr, tokens->n_tok,
                       tokens->doc_off.as<int64_t>(), tokens->n_docs, num_features, binary, hash_variant,
                       value_dtype, tokens->max_doc, *m);
    *out = m.release();
  });
}

int stc_hash_tokens(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                    int64_t n_tok, int32_t num_features, int hash_variant, int32_t* idx_out) {
  return guard([&] {
    STC_REQUIRE(ctx && (idx_out || n_tok == 0), "ctx/idx_out");
    STC_REQUIRE(num_features > 0, "numFeatures must be > 0");
    STC_REQUIRE(hash_variant == STC_HASH_STANDARD || hash_variant == STC_HASH_SPARK24, "hash_variant");
    ctx->use();
    TokenUpload u;
    upload_tokens(*ctx, u, utf8, n_bytes, tok_off, n_tok, nullptr, 0);
    DevBuf out;
    out.reserve(4 * std::max<int64_t>(n_tok, 1));
    hashing::hash_tokens(*ctx, u.utf8.as<uint8_t>(), u.tok_off.as<int64_t>(), n_tok, num_features,
                         hash_variant, out.as<int32_t>());
    if (n_tok) HIP_CHECK(hipMemcpyAsync(idx_out, out.p, 4 * n_tok, hipMemcpyDeviceToHost, ctx->stream));
    wait_stream(*ctx, ctx->stream);
  });
}

int stc_hashing_tf_dev(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                       int64_t n_tok, const int64_t* doc_off, int64_t n_docs, int32_t num_features,
                       int binary, int hash_variant, int value_dtype, stc_dcsr** out) {
  return guard([&] {
    STC_REQUIRE(ctx && doc_off && out, "ctx/doc_off/out");
    STC_REQUIRE(num_features > 0, "numFeatures must be > 0");
    STC_REQUIRE(hash_variant == STC_HASH_STANDARD || hash_variant == STC_HASH_SPARK24, "hash_variant");
    STC_REQUIRE(value_dtype == STC_F32 || value_dtype == STC_F64, "value_dtype");
    ctx->use();
    TokenUpload u;
    upload_tokens(*ctx, u, utf8, n_bytes, tok_off, n_tok, doc_off, n_docs);
    auto m = std::make_unique<stc_dcsr>();
    m->ctx = ctx;
    m->device = ctx->device;
    hashing::build_csr(*ctx, u.utf8.as<uint8_t>(), u.tok_off.as<int64_t>(), nullptr, n_tok, u.doc_off.as<int64_t>(),
                       n_docs, num_features, binary, hash_variant, value_dtype, u.max_doc, *m);
    *out = m.release();
  });
}

int stc_hashing_tf(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                   int64_t n_tok, const int64_t* doc_off, int64_t n_docs, int32_t num_features,
                   int binary, int hash_variant, int64_t* indptr_out, int32_t* indices_out,
                   double* values_out) {
  stc_dcsr* m = nullptr;
  int rc = stc_hashing_tf_dev(ctx, utf8, n_bytes, tok_off, n_tok, doc_off, n_docs, num_features,
                              binary, hash_variant, STC_F64, &m);
  if (rc != STC_OK) return rc;
  rc = stc_dcsr_download(ctx, m, indptr_out, indices_out, values_out);
  stc_dcsr_free(m);
  return rc;
}

// ---- Tokenizer (K0) ---------------------------------------------------------------------
namespace {
struct Tokens {
  DevBuf utf8, tok_off, doc_off;
  int64_t n_tok = 0, n_bytes = 0;
};
void run_tokenizer(Ctx& c, Tokens& t, const uint8_t* text, int64_t n_bytes, const int64_t* text_off,
                   int64_t n_docs) {
  STC_REQUIRE(n_bytes >= 0 && n_docs >= 0, "sizes must be >= 0");
  STC_REQUIRE(n_docs < (int64_t(1) << 31) - 1, "at most 2^31-2 documents per call");
  STC_REQUIRE(text_off && (n_bytes == 0 || text), "text/text_off");
  STC_REQUIRE(text_off[0] == 0 && text_off[n_docs] == n_bytes, "text_off must span [0, n_bytes]");
  for (int64_t d = 0; d < n_docs; ++d) STC_REQUIRE(text_off[d + 1] >= text_off[d], "text_off must be non-decreasing");
  DevBuf d_text, d_off;
  d_text.reserve(n_bytes + 64);  // k_count reads whole aligned dwords past the last byte
  d_off.reserve(8 * (n_docs + 1));
  if (n_bytes) HIP_CHECK(hipMemcpyAsync(d_text.p, text, n_bytes, hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemcpyAsync(d_off.p, text_off, 8 * (n_docs + 1), hipMemcpyHostToDevice, c.stream));
  tokenizer::tokenize(c, d_text.as<uint8_t>(), d_off.as<int64_t>(), n_docs, t.utf8, t.tok_off, t.doc_off,
                      t.n_tok, t.n_bytes);
}
}  // namespace

int stc_tokenize(stc_ctx* ctx, const uint8_t* text, int64_t n_bytes, const int64_t* text_off,
                 int64_t n_docs, uint8_t* utf8_out, int64_t utf8_cap, int64_t* n_out_bytes,
                 int64_t* tok_off_out, int64_t* n_tok_out, int64_t* doc_off_out) {
  return guard([&] {
    STC_REQUIRE(ctx && n_out_bytes, "ctx/n_out_bytes");
    STC_REQUIRE(utf8_cap >= 0, "utf8_cap must be >= 0");
    const bool query = utf8_out == nullptr;  // the size query: *n_out_bytes (and *n_tok_out) only
    STC_REQUIRE(query ? utf8_cap == 0 : (n_tok_out && tok_off_out && doc_off_out), "outputs");
    ctx->use();
    Tokens t;
    run_tokenizer(*ctx, t, text, n_bytes, text_off, n_docs);
    if (query) {
      *n_out_bytes = t.n_bytes;
      if (n_tok_out) *n_tok_out = t.n_tok;
      return;
    }
    // the lower-cased blob can outgrow the input (İ → i̇, Ⱥ → ⱥ: 2 → 3 bytes); its size is known from the
    // count pass, so a short buffer is refused before anything is copied (*n_out_bytes = the size needed)
    *n_out_bytes = t.n_bytes;
    if (t.n_bytes > utf8_cap)
      throw Error(STC_ERR_INVALID_ARG, "utf8_out holds " + std::to_string(utf8_cap) + " bytes, the lower-cased text needs " +
                                           std::to_string(t.n_bytes));
    hipStream_t s = ctx->stream;
    if (t.n_bytes) HIP_CHECK(hipMemcpyAsync(utf8_out, t.utf8.p, t.n_bytes, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(tok_off_out, t.tok_off.p, 8 * (t.n_tok + 1), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(doc_off_out, t.doc_off.p, 8 * (n_docs + 1), hipMemcpyDeviceToHost, s));
    wait_stream(*ctx, s);
    *n_out_bytes = t.n_bytes;
    *n_tok_out = t.n_tok;
  });
}

int stc_tokenize_hashing_tf_dev(stc_ctx* ctx, const uint8_t* text, int64_t n_bytes,
                                const int64_t* text_off, int64_t n_docs, int32_t num_features,
                                int binary, int hash_variant, int value_dtype, stc_dcsr** out) {
  return guard([&] {
    STC_REQUIRE(ctx && out, "ctx/out");
    STC_REQUIRE(num_features > 0, "numFeatures must be > 0");
    STC_REQUIRE(hash_variant == STC_HASH_STANDARD || hash_variant == STC_HASH_SPARK24, "hash_variant");
    STC_REQUIRE(value_dtype == STC_F32 || value_dtype == STC_F64, "value_dtype");
    ctx->use();
    Tokens t;
    run_tokenizer(*ctx, t, text, n_bytes, text_off, n_docs);
    auto m = std::make_unique<stc_dcsr>();
    m->ctx = ctx;
    m->device = ctx->device;
    hashing::build_csr(*ctx, t.utf8.as<uint8_t>(), t.tok_off.as<int64_t>(), nullptr, t.n_tok, t.doc_off.as<int64_t>(),
                       n_docs, num_features, binary, hash_variant, value_dtype, -1, *m);
    *out = m.release();
  });
}

// ---- IDF --------------------------------------------------------------------------------
}  // extern "C"

struct stc_didf {
  Ctx* ctx = nullptr;
  int device = -1;
  int64_t cols = 0, m = 0;
  DevBuf idf, df;
  DevBuf cache;  // the hot-idf table of idf.hip k_transform_cached (empty: not used)
};

namespace {
// IDF.fit on the device: df (all ranks' when connected), m, idf into the given buffers
void idf_fit_impl(Ctx& c, const DCsr& tf, int64_t min_doc_freq, DevBuf& df, DevBuf& idf, int64_t& m) {
  hipStream_t s = c.stream;
  c.recycle.take(df, 8 * tf.cols);
  c.recycle.take(idf, 8 * tf.cols);
  m = tf.rows;
  if (!c.coll()) {  // m known: idf written by the df reduction itself
    const idf::IdfFinal fin{(double)m, min_doc_freq, idf.as<double>()};
    if (idf::doc_freq(c, tf, df.as<int64_t>(), &fin)) return;
    idf::finalize(c, df.as<int64_t>(), tf.cols, m, min_doc_freq, idf.as<double>());
    return;
  }
  idf::doc_freq(c, tf, df.as<int64_t>());
  {  // DocumentFrequencyAggregator.merge over ranks
    DevBuf mm;
    mm.reserve(8);
    HIP_CHECK(hipMemcpyAsync(mm.p, &m, 8, hipMemcpyHostToDevice, s));
    coll_group_start(c);
    coll_all_reduce(c, df.p, (size_t)tf.cols, ncclInt64, s);
    coll_all_reduce(c, mm.p, 1, ncclInt64, s);
    coll_group_end(c);
    HIP_CHECK(hipMemcpyAsync(&m, mm.p, 8, hipMemcpyDeviceToHost, s));
    wait_stream(c, s);
  }
  idf::finalize(c, df.as<int64_t>(), tf.cols, m, min_doc_freq, idf.as<double>());
}
}  // namespace

extern "C" {

int stc_idf_fit(stc_ctx* ctx, const stc_dcsr* tf, int64_t min_doc_freq, double* idf_out,
                int64_t* df_out, int64_t* m_out) {
  return guard([&] {
    STC_REQUIRE(ctx && tf && idf_out, "ctx/tf/idf_out");
    STC_REQUIRE(tf->ctx == ctx, "the matrix belongs to another stc_ctx");
    STC_REQUIRE(min_doc_freq >= 0, "minDocFreq must be >= 0");
    ctx->use();
    hipStream_t s = ctx->stream;
    DevBuf& df = ctx->scratch[9];  // grow-only on the context: no per-call allocation
    DevBuf& idf = ctx->scratch[10];
    int64_t m = 0;
    idf_fit_impl(*ctx, *tf, min_doc_freq, df, idf, m);
    HIP_CHECK(hipMemcpyAsync(idf_out, idf.p, 8 * tf->cols, hipMemcpyDeviceToHost, s));
    if (df_out) HIP_CHECK(hipMemcpyAsync(df_out, df.p, 8 * tf->cols, hipMemcpyDeviceToHost, s));
    wait_stream(*ctx, s);
    if (m_out) *m_out = m;
  });
}

int stc_idf_fit_dev(stc_ctx* ctx, const stc_dcsr* tf, int64_t min_doc_freq, stc_didf** out) {
  return guard([&] {
    STC_REQUIRE(ctx && tf && out, "ctx/tf/out");
    STC_REQUIRE(tf->ctx == ctx, "the matrix belongs to another stc_ctx");
    STC_REQUIRE(min_doc_freq >= 0, "minDocFreq must be >= 0");
    ctx->use();
    auto md = std::make_unique<stc_didf>();
    md->ctx = ctx;
    md->device = ctx->device;
    md->cols = tf->cols;
    idf_fit_impl(*ctx, *tf, min_doc_freq, md->df, md->idf, md->m);
    idf::build_cache(*ctx, md->df.as<int64_t>(), md->idf.as<double>(), md->cols, md->cache);
    *out = md.release();  // (the stream orders every later use of the model after the fit)
  });
}

int stc_idf_get(stc_ctx* ctx, const stc_didf* md, double* idf_out, int64_t* df_out, int64_t* m_out) {
  return guard([&] {
    STC_REQUIRE(ctx && md, "ctx/model");
    STC_REQUIRE(md->ctx == ctx, "the model belongs to another stc_ctx");
    ctx->use();
    hipStream_t s = ctx->stream;
    if (idf_out) HIP_CHECK(hipMemcpyAsync(idf_out, md->idf.p, 8 * md->cols, hipMemcpyDeviceToHost, s));
    if (df_out) HIP_CHECK(hipMemcpyAsync(df_out, md->df.p, 8 * md->cols, hipMemcpyDeviceToHost, s));
    wait_stream(*ctx, s);
    if (m_out) *m_out = md->m;
  });
}

int stc_didf_shape(const stc_didf* md, int64_t* cols_out, int64_t* m_out) {
  return guard([&] {
    STC_REQUIRE(md, "model");
    if (cols_out) *cols_out = md->cols;
    if (m_out) *m_out = md->m;
  });
}

int stc_idf_transform_dev(stc_ctx* ctx, stc_dcsr* tf, const stc_didf* md, double zero_floor) {
  return guard([&] {
    STC_REQUIRE(ctx && tf && md, "ctx/tf/model");
    STC_REQUIRE(tf->ctx == ctx && md->ctx == ctx, "the matrix or model belongs to another stc_ctx");
    STC_REQUIRE(tf->cols == md->cols, "vector size does not match the IDF size");
    STC_REQUIRE(zero_floor >= 0.0, "zero_floor must be >= 0");
    ctx->use();
    idf::transform(*ctx, *tf, md->idf.as<double>(), zero_floor, &md->cache);
    wait_stream(*ctx, ctx->stream);
  });
}

int stc_didf_free(stc_didf* md) {
  return guard([&] {
    if (!md) return;
    (void)hipSetDevice(md->device);
    (void)hipDeviceSynchronize();  // queued readers of the model first, outside the lock (as stc_dcsr_free)
    {  // back to the context that made it, if it still exists (Recycler)
      std::lock_guard<std::mutex> lk(g_live_mu);
      if (md->ctx && g_live.count(static_cast<stc_ctx*>(md->ctx)) && md->ctx->device == md->device) {
        md->ctx->recycle.put(md->idf);
        md->ctx->recycle.put(md->df);
      }
    }
    delete md;
  });
}

int stc_idf_transform(stc_ctx* ctx, stc_dcsr* tf, const double* idf, double zero_floor) {
  return guard([&] {
    STC_REQUIRE(ctx && tf && idf, "ctx/tf/idf");
    STC_REQUIRE(tf->ctx == ctx, "the matrix belongs to another stc_ctx");
    STC_REQUIRE(zero_floor >= 0.0, "zero_floor must be >= 0");
    ctx->use();
    DevBuf& d = ctx->scratch[11];
    d.reserve(8 * tf->cols);
    HIP_CHECK(hipMemcpyAsync(d.p, idf, 8 * tf->cols, hipMemcpyHostToDevice, ctx->stream));
    idf::transform(*ctx, *tf, d.as<double>(), zero_floor);
    wait_stream(*ctx, ctx->stream);
  });
}

// ---- LDA ----------------------------------------------------------------------------------
void stc_lda_config_default(stc_lda_config* c) {
  if (!c) return;
  *c = stc_lda_config{};
  c->k = 10;
  c->vocab_size = 1 << 18;
  c->doc_concentration = nullptr;
  c->doc_concentration_len = 0;
  c->topic_concentration = -1.0;
  c->tau0 = 1024.0;
  c->kappa = 0.51;
  c->mini_batch_fraction = 0.05;
  c->gamma_shape = 100.0;
  c->optimize_doc_concentration = 1;
  c->sample_with_replacement = 1;
  c->seed = 0;
  c->dtype = STC_F64;  // Spark computes the E-step in Double
  c->max_inner_iter = 0;
}

int stc_lda_create(stc_ctx* ctx, const stc_lda_config* cfg, stc_lda** out) {
  return guard([&] {
    STC_REQUIRE(ctx && cfg && out, "ctx/cfg/out");
    // [U] LDA / OnlineLDAOptimizer setter validation
    STC_REQUIRE(cfg->k > 1, "LDA k (number of clusters) must be > 1");
    STC_REQUIRE(cfg->k <= 4096, "k <= 4096");
    STC_REQUIRE(cfg->vocab_size > 0 && cfg->vocab_size <= (int64_t(1) << 31), "vocab_size in (0, 2^31]");
    STC_REQUIRE(cfg->tau0 > 0, "LDA tau0 must be positive");
    STC_REQUIRE(cfg->kappa > 0, "LDA kappa must be positive");
    STC_REQUIRE(cfg->mini_batch_fraction > 0.0 && cfg->mini_batch_fraction <= 1.0,
                "miniBatchFraction must be in range (0,1]");
    STC_REQUIRE(cfg->gamma_shape > 1.0 / 3.0, "gammaShape must be > 1/3");
    STC_REQUIRE(cfg->dtype == STC_F32 || cfg->dtype == STC_F64 || cfg->dtype == STC_MIXED, "dtype");
    STC_REQUIRE(cfg->mixed_resolve_iters >= 0, "mixed_resolve_iters must be >= 0");
    STC_REQUIRE(cfg->max_inner_iter >= 0, "max_inner_iter must be >= 0");
    ctx->use();
    auto L = std::make_unique<stc_lda>();
    L->ctx = ctx;
    L->cfg = *cfg;
    if (L->cfg.max_inner_iter == 0) L->cfg.max_inner_iter = 100000;
    L->k = cfg->k;
    L->V = cfg->vocab_size;
    // STC_MIXED: the fp32 pipeline (dtype STC_F32 inside the library) plus the fp64 re-solve (mixed_resolve)
    L->mixed = cfg->dtype == STC_MIXED;
    L->dtype = L->mixed ? STC_F32 : cfg->dtype;
    L->mixed_thr = cfg->mixed_resolve_iters > 0 ? cfg->mixed_resolve_iters : 500;
    L->tsize = L->dtype == STC_F32 ? 4 : 8;
    const int W = L->dtype == STC_F32 ? 4 : 2;
    L->kp = (int)ceil_div(L->k, W) * W;
    L->P = ((L->kp / W) % 2 == 1) ? L->kp : L->kp + W;  // P/W odd: conflict-free b128 rows
    L->lds_rows = L->dtype == STC_F32 ? lda::estep_lds_rows<float>(L->k, L->kp, L->P)
                                      : lda::estep_lds_rows<double>(L->k, L->kp, L->P);
    if (L->mixed) {  // the fp64 workgroup kernel's shape at the fp32 row pitch, and the fp64 fast-kernel capacity
      L->P64 = ((L->kp / 2) % 2 == 1) ? L->kp : L->kp + 2;
      L->lds_rows64 = lda::estep_lds_rows<double>(L->k, L->kp, L->P64);
      const int c64 = use_wide(L->k, STC_F64) ? lda::wide_row_cap(L->k) : lda::rows64_row_cap(L->k);
      L->cap64 = c64 > 0 ? c64 : -1;
    }
    const char* nw = std::getenv("STC_DISABLE_WAVE");
    // docs with nnz <= wave_cap run the register-resident kernel (fp32: lda_grid.hip, fp64:
    // lda_rows64.hip), the rest the workgroup kernel (lda.hip); −1: no slot is "short" (not even empty)
    const int cap = use_wide(L->k, L->dtype) ? lda::wide_row_cap(L->k)
                    : L->dtype == STC_F32 ? lda::grid_row_cap(L->k) : lda::rows64_row_cap(L->k);
    L->wave_cap = (!(nw && nw[0] == '1') && cap > 0) ? cap : -1;
    // α / η resolution ([U] OnlineLDAOptimizer.initialize)
    std::vector<double> alpha((size_t)L->k);
    const int alen = cfg->doc_concentration ? cfg->doc_concentration_len : 0;
    if (alen == 0 || (alen == 1 && cfg->doc_concentration[0] == -1.0)) {
      std::fill(alpha.begin(), alpha.end(), 1.0 / L->k);
    } else if (alen == 1) {
      STC_REQUIRE(cfg->doc_concentration[0] >= 0, "docConcentration must be >= 0");
      std::fill(alpha.begin(), alpha.end(), cfg->doc_concentration[0]);
    } else {
      STC_REQUIRE(alen == L->k, "docConcentration must have length 1 or k");
      for (int t = 0; t < L->k; ++t) {
        STC_REQUIRE(cfg->doc_concentration[t] >= 0, "docConcentration entries must be >= 0");
        alpha[(size_t)t] = cfg->doc_concentration[t];
      }
    }
    if (cfg->topic_concentration == -1.0) L->eta = 1.0 / L->k;
    else {
      STC_REQUIRE(cfg->topic_concentration >= 0, "topicConcentration must be >= 0");
      L->eta = cfg->topic_concentration;
    }
    L->cfg.doc_concentration = nullptr;
    L->cfg.doc_concentration_len = 0;
    L->nblocks_m = ceil_div(L->V, lda::kRowsPerBlock);
    const char* vs = std::getenv("STC_VIRTUAL_SHARDS");
    L->virt = vs ? std::max(1, std::min(64, std::atoi(vs))) : 1;
    const char* ho = std::getenv("STC_HOT_ORDER");
    L->hot_order = !(ho && ho[0] == '0');
    const char* sd = std::getenv("STC_SORT_DOCS");
    L->sort_docs = !(sd && sd[0] == '0');
    const char* psr = std::getenv("STC_PRESORT");
    L->presort = psr ? std::max(0, std::min(2, std::atoi(psr))) : 1;
    const char* wt = std::getenv("STC_WIDE_TEAM");
    L->team_force = wt ? std::max(0, std::min(8, std::atoi(wt))) : 0;
    const char* tg = std::getenv("STC_TGRID");
    L->tgrid = !(tg && tg[0] == '0');
    L->tgrid_require = tg && tg[0] == '2';
    const char* fc = std::getenv("STC_COLLECTIVE_MSTEP");
    L->force_coll = fc && fc[0] == '1';
    const char* rc = std::getenv("STC_RS_CHUNKS");
    L->rs_chunks = rc ? std::max(1, std::min(16, std::atoi(rc))) : 4;
    ensure_layout(*L);  // λ, Bp, stat, logscale, colpart for the current shard count
    L->colsum.reserve(8 * L->k);
    L->psic.reserve(16 * L->k);  // ψ(colsum), exp(−ψ(colsum))
    L->alpha.reserve(8 * L->k);
    L->small.reserve(8 * (L->k + 1));
    L->stats4.reserve(8 * 4);
    L->cum2.reserve(8 * 2);
    HIP_CHECK(hipMemsetAsync(L->cum2.p, 0, 16, ctx->stream));
    HIP_CHECK(hipMemcpyAsync(L->alpha.p, alpha.data(), 8 * L->k, hipMemcpyHostToDevice, ctx->stream));
    wait_stream(*ctx, ctx->stream);
    for (auto& s : L->ev)
      for (auto& e : s) HIP_CHECK(hipEventCreate(&e));
    *out = L.release();
  });
}

int stc_lda_destroy(stc_lda* lda) {
  return guard([&] {
    if (!lda) return;
    (void)hipSetDevice(lda->ctx->device);
    // queued work first (with a communicator: a bounded wait; a collective that never completes is
    // aborted with its communicator, which releases its kernels, so the destroy returns)
    Ctx& c = *lda->ctx;
    for (hipStream_t q : {c.stream, lda->side, lda->cstream}) {
      if (!q) continue;
      try {
        wait_stream(c, q);
      } catch (const Error&) {
        abort_comm(c);
      }
      (void)hipStreamSynchronize(q);
    }
    delete lda;
  });
}

int stc_lda_set_corpus(stc_lda* L, const stc_dcsr* corpus, int64_t corpus_size_total) {
  return guard([&] {
    STC_REQUIRE(L && corpus, "lda/corpus");
    STC_REQUIRE(corpus->ctx == L->ctx, "the corpus belongs to another stc_ctx than the LDA handle");
    STC_REQUIRE(corpus->cols == L->V, "corpus must have vocab_size columns");
    STC_REQUIRE(corpus->dtype == corpus_dtype(*L), "corpus value dtype must match the LDA dtype (STC_F64 for STC_MIXED)");
    STC_REQUIRE(corpus->rows < (int64_t(1) << 31), "at most 2^31-1 documents per rank");
    STC_REQUIRE(corpus_size_total >= corpus->rows && corpus_size_total > 0,
                "corpus_size_total must be >= this rank's rows and > 0");
    settle_side(*L);  // a draw still being sampled reads the previous corpus
    if (L->mixed) {  // the fp32 copy of the values the fp32 E-step reads
      L->ctx->use();
      L->vals32.reserve(4 * std::max<int64_t>(corpus->nnz, 1));
      lda::launch_to_f32(L->ctx->stream, corpus->values.as<double>(), L->vals32.as<float>(), corpus->nnz);
      wait_stream(*L->ctx, L->ctx->stream);
      L->vals32_for = corpus;
    }
    L->corpus = corpus;
    L->corpus_total = corpus_size_total;
    L->pre_valid = false;  // a prefetched draw sampled the previous corpus
    L->order_for = nullptr;
  });
}

int stc_lda_init_random(stc_lda* L, uint64_t seed) {
  return guard([&] {
    STC_REQUIRE(L, "lda");
    L->ctx->use();
    lda::launch_init_lambda(L->ctx->stream, L->lam.as<double>(), L->V, L->k, seed, L->cfg.gamma_shape);
    L->lam_stale = false;
    refresh(*L);
    L->iteration = 0;
    L->draws = 0;  // a fresh generator, as Spark's initialize()
    L->pre_valid = false;
    wait_stream(*L->ctx, L->ctx->stream);
  });
}

int stc_lda_set_topics(stc_lda* L, const double* topics, int layout) {
  return guard([&] {
    STC_REQUIRE(L && topics, "lda/topics");
    STC_REQUIRE(layout == STC_LAYOUT_VK || layout == STC_LAYOUT_KV, "layout");
    L->ctx->use();
    const int64_t n = L->V * L->k;
    std::vector<double> h((size_t)n);
    for (int64_t v = 0; v < L->V; ++v)
      for (int t = 0; t < L->k; ++t) {
        const double x = layout == STC_LAYOUT_VK ? topics[v * L->k + t] : topics[(int64_t)t * L->V + v];
        STC_REQUIRE(x > 0.0 && std::isfinite(x), "topics entries must be finite and > 0");
        h[(size_t)(v * L->k + t)] = x;
      }
    HIP_CHECK(hipMemcpyAsync(L->lam.p, h.data(), 8 * n, hipMemcpyHostToDevice, L->ctx->stream));
    L->lam_stale = false;
    refresh(*L);
    wait_stream(*L->ctx, L->ctx->stream);
  });
}

int stc_lda_get_topics(stc_lda* L, double* out, int layout) {
  return guard([&] {
    STC_REQUIRE(L && out, "lda/out");
    STC_REQUIRE(layout == STC_LAYOUT_VK || layout == STC_LAYOUT_KV, "layout");
    STC_REQUIRE(L->has_topics, "no topics yet");
    L->ctx->use();
    gather_lambda(*L);
    const int64_t n = L->V * L->k;
    if (layout == STC_LAYOUT_VK) {
      HIP_CHECK(hipMemcpyAsync(out, L->lam.p, 8 * n, hipMemcpyDeviceToHost, L->ctx->stream));
      wait_stream(*L->ctx, L->ctx->stream);
    } else {
      std::vector<double> h((size_t)n);
      HIP_CHECK(hipMemcpyAsync(h.data(), L->lam.p, 8 * n, hipMemcpyDeviceToHost, L->ctx->stream));
      wait_stream(*L->ctx, L->ctx->stream);
      for (int64_t v = 0; v < L->V; ++v)
        for (int t = 0; t < L->k; ++t) out[(int64_t)t * L->V + v] = h[(size_t)(v * L->k + t)];
    }
  });
}

int stc_lda_set_alpha(stc_lda* L, const double* alpha) {
  return guard([&] {
    STC_REQUIRE(L && alpha, "lda/alpha");
    for (int t = 0; t < L->k; ++t) STC_REQUIRE(alpha[t] >= 0, "alpha entries must be >= 0");
    L->ctx->use();
    HIP_CHECK(hipMemcpyAsync(L->alpha.p, alpha, 8 * L->k, hipMemcpyHostToDevice, L->ctx->stream));
    wait_stream(*L->ctx, L->ctx->stream);
  });
}

int stc_lda_get_alpha(stc_lda* L, double* alpha_out) {
  return guard([&] {
    STC_REQUIRE(L && alpha_out, "lda/alpha_out");
    L->ctx->use();
    HIP_CHECK(hipMemcpyAsync(alpha_out, L->alpha.p, 8 * L->k, hipMemcpyDeviceToHost, L->ctx->stream));
    wait_stream(*L->ctx, L->ctx->stream);
  });
}

int stc_lda_get_eta(stc_lda* L, double* eta_out) {
  return guard([&] {
    STC_REQUIRE(L && eta_out, "lda/eta_out");
    *eta_out = L->eta;
  });
}

int stc_lda_shape(const stc_lda* L, int32_t* k_out, int64_t* vocab_out) {
  return guard([&] {
    STC_REQUIRE(L, "lda");
    if (k_out) *k_out = L->k;
    if (vocab_out) *vocab_out = L->V;
  });
}

int stc_lda_get_iteration(stc_lda* L, int64_t* it) {
  return guard([&] {
    STC_REQUIRE(L && it, "lda/it");
    *it = L->iteration;
  });
}

int stc_lda_step(stc_lda* L, const int64_t* ids, int64_t n, const double* gamma0, stc_step_stats* st) {
  return guard([&] {
    STC_REQUIRE(L && (ids || n == 0) && n >= 0, "lda/ids");
    L->ctx->use();
    if (L->dtype == STC_F32) step_ids<float>(*L, ids, n, gamma0, st);
    else step_ids<double>(*L, ids, n, gamma0, st);
  });
}

int stc_lda_next(stc_lda* L, stc_step_stats* st) {
  return guard([&] {
    STC_REQUIRE(L, "lda");
    L->ctx->use();
    if (L->dtype == STC_F32) next_impl<float>(*L, st);
    else next_impl<double>(*L, st);
  });
}

int stc_lda_estep(stc_lda* L, const int64_t* ids, int64_t n, const double* gamma0, double* gamma_out,
                  double* stat_out, int32_t* iters_out) {
  return guard([&] {
    STC_REQUIRE(L && (ids || n == 0) && n >= 0, "lda/ids");
    L->ctx->use();
    if (L->dtype == STC_F32) estep_only<float>(*L, ids, n, gamma0, gamma_out, stat_out, iters_out);
    else estep_only<double>(*L, ids, n, gamma0, gamma_out, stat_out, iters_out);
  });
}

int stc_lda_bound(stc_lda* L, const stc_dcsr* docs, uint64_t gamma_seed, int64_t doc_id_base,
                  const double* gamma0, double* bound_out, double* corpus_part_out,
                  double* topics_part_out, double* token_count_out) {
  return guard([&] {
    STC_REQUIRE(L && docs, "lda/docs");
    STC_REQUIRE(docs->ctx == L->ctx, "the documents belong to another stc_ctx than the LDA handle");
    L->ctx->use();
    double h[3] = {0, 0, 0};
    double norm = 0;
    const bool sharded = L->lam_stale;
    if (L->dtype == STC_F32 && !L->mixed) {  // (a mixed handle infers in fp64)
      infer_impl<float>(*L, *docs, gamma_seed, doc_id_base, gamma0, true, nullptr, h);
      topics_part<float>(*L, h + 2, &norm);
    } else {
      infer_impl<double>(*L, *docs, gamma_seed, doc_id_base, gamma0, true, nullptr, h);
      topics_part<double>(*L, h + 2, &norm);
    }
    // corpusPart and the token count are sums over the ranks' documents; the topics part's element
    // sum too when λ is sharded (each rank holds its slice), else it is already complete everywhere
    allreduce_host(*L->ctx, h, sharded ? 3 : 2);
    const double tp = h[2] + norm;
    if (bound_out) *bound_out = h[0] + tp;
    if (corpus_part_out) *corpus_part_out = h[0];
    if (topics_part_out) *topics_part_out = tp;
    if (token_count_out) *token_count_out = h[1];
  });
}

int stc_lda_topic_distribution(stc_lda* L, const stc_dcsr* docs, uint64_t gamma_seed,
                               int64_t doc_id_base, const double* gamma0, double* out) {
  return guard([&] {
    STC_REQUIRE(L && docs && (out || docs->rows == 0), "lda/docs/out");
    STC_REQUIRE(docs->ctx == L->ctx, "the documents belong to another stc_ctx than the LDA handle");
    L->ctx->use();
    if (L->dtype == STC_F32 && !L->mixed)  // (a mixed handle infers in fp64)
      infer_impl<float>(*L, *docs, gamma_seed, doc_id_base, gamma0, false, out, nullptr);
    else
      infer_impl<double>(*L, *docs, gamma_seed, doc_id_base, gamma0, false, out, nullptr);
    for (int64_t i = 0; i < docs->rows; ++i) {  // normalize(gamma, 1.0); zeros for empty docs
      double* g = out + i * L->k;
      double sum = 0.0;
      for (int t = 0; t < L->k; ++t) sum += std::fabs(g[t]);
      if (sum > 0.0)
        for (int t = 0; t < L->k; ++t) g[t] /= sum;
    }
  });
}

int stc_lda_describe(stc_lda* L, int32_t max_terms, int32_t* idx_out, double* weight_out) {
  return guard([&] {
    STC_REQUIRE(L && idx_out && weight_out, "lda/idx_out/weight_out");
    STC_REQUIRE(max_terms > 0, "maxTermsPerTopic must be > 0");
    STC_REQUIRE(L->has_topics, "no topics yet");
    STC_REQUIRE(L->V * L->k < (int64_t(1) << 31), "describe: V*k must be < 2^31");
    L->ctx->use();
    gather_lambda(*L);
    hipStream_t s = L->ctx->stream;
    const int64_t n = L->V * L->k;
    const int N = (int)std::min<int64_t>(max_terms, L->V);
    DevBuf kv, kv_s, ix, ix_s, off, tmp;
    kv.reserve(8 * n);
    kv_s.reserve(8 * n);
    ix.reserve(4 * n);
    ix_s.reserve(4 * n);
    off.reserve(8 * (L->k + 1));
    std::vector<int64_t> ho((size_t)L->k + 1);
    for (int t = 0; t <= L->k; ++t) ho[(size_t)t] = (int64_t)t * L->V;
    HIP_CHECK(hipMemcpyAsync(off.p, ho.data(), 8 * (L->k + 1), hipMemcpyHostToDevice, s));
    lda::launch_transpose_kv(s, L->lam.as<double>(), L->V, L->k, kv.as<double>(), ix.as<int32_t>());
    size_t tb = 0;
    // stable descending sort per topic ⇒ ties keep ascending term index (Scala's sortBy(-w))
    HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortPairsDescending(
        nullptr, tb, kv.as<double>(), kv_s.as<double>(), ix.as<int32_t>(), ix_s.as<int32_t>(), (int)n,
        L->k, off.as<int64_t>(), off.as<int64_t>() + 1, 0, 64, s));
    tmp.reserve(tb);
    HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortPairsDescending(
        tmp.p, tb, kv.as<double>(), kv_s.as<double>(), ix.as<int32_t>(), ix_s.as<int32_t>(), (int)n,
        L->k, off.as<int64_t>(), off.as<int64_t>() + 1, 0, 64, s));
    std::vector<double> cs((size_t)L->k);
    HIP_CHECK(hipMemcpyAsync(cs.data(), L->colsum.p, 8 * L->k, hipMemcpyDeviceToHost, s));
    std::vector<double> w((size_t)N);
    for (int t = 0; t < L->k; ++t) {
      HIP_CHECK(hipMemcpyAsync(idx_out + (int64_t)t * N, ix_s.as<int32_t>() + (int64_t)t * L->V, 4 * N,
                               hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipMemcpyAsync(weight_out + (int64_t)t * N, kv_s.as<double>() + (int64_t)t * L->V, 8 * N,
                               hipMemcpyDeviceToHost, s));
    }
    wait_stream(*L->ctx, s);
    for (int t = 0; t < L->k; ++t)  // normalize(topic, 1.0): v / ‖v‖₁ (λ > 0)
      for (int j = 0; j < N; ++j) weight_out[(int64_t)t * N + j] /= cs[(size_t)t];
  });
}

int stc_lda_enable_timing(stc_lda* L, int on) {
  return guard([&] {
    STC_REQUIRE(L, "lda");
    L->timing = on != 0;
    for (double& a : L->acc_ms) a = 0.0;
    L->timed_steps = 0;
    L->ev_pending[0] = L->ev_pending[1] = L->ev_pending[2] = false;
  });
}

int stc_lda_kernel_counts(stc_lda* L, int64_t out[STC_KC_N]) {
  return guard([&] {
    STC_REQUIRE(L && out, "lda/out");
    std::copy(L->kcount, L->kcount + STC_KC_N, out);
  });
}

int stc_lda_phase_times(stc_lda* L, double* ms_out, int64_t* steps_out) {
  return guard([&] {
    STC_REQUIRE(L && ms_out, "lda/ms_out");
    L->ctx->use();
    wait_stream(*L->ctx, L->ctx->stream);
    harvest_all(*L);
    for (int p = 0; p < 5; ++p) ms_out[p] = L->timed_steps ? L->acc_ms[p] / (double)L->timed_steps : 0.0;
    if (steps_out) *steps_out = L->timed_steps;
  });
}

int stc_lda_counters(stc_lda* L, int64_t out[4]) {
  return guard([&] {
    STC_REQUIRE(L && out, "lda/out");
    L->ctx->use();
    int64_t c2[2] = {0, 0};
    HIP_CHECK(hipMemcpyAsync(c2, L->cum2.p, 16, hipMemcpyDeviceToHost, L->ctx->stream));
    wait_stream(*L->ctx, L->ctx->stream);
    out[0] = L->cum_docs;
    out[1] = L->cum_entries;
    out[2] = c2[0];
    out[3] = c2[1];
  });
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// stc_group: one process driving N devices (stc_init(device_ids, n)).  The JVM runs
// the reference in ONE process (Spark local[*], LDATraining.scala:7), so its drop-in needs the N GPUs of
// the node behind one handle: N contexts joined by one communicator (ncclCommInitAll over distinct
// devices; the in-process transport above when every member shares one device), N LDA handles over
// contiguous document shards (balanced by entries), each call run on one host thread per member.
// ---------------------------------------------------------------------------------------
struct stc_group {
  std::vector<stc_ctx*> ctx;
  std::vector<stc_lda*> lda;
  std::vector<stc_dcsr*> shard;
  std::vector<int64_t> row0;  // first corpus row of each member's shard (n + 1 entries)
  std::unique_ptr<LocalColl> local;
  int64_t rows = 0, cols = 0;
  int dtype = STC_F64;
  int transport = STC_TRANSPORT_NONE;  // how the members' collectives travel (stc_group_transport)
  bool threaded = false;               // run even a one-member call on its own host thread (STC_GROUP_RCCL)
  // RCCL fault handling: a member's failure sets `abort` (every member's waits then throw instead of waiting
  // on collectives the failed member never joins) and, after the call, aborts every member's communicator;
  // the group is then `broken`: every later call but destroy fails with STC_ERR_STATE
  std::atomic<bool> abort{false};
  bool broken = false;
  std::string broken_why;
  int n() const { return (int)ctx.size(); }
};

namespace {

void member_ok(int rc) {
  if (rc != STC_OK) throw Error(rc, stc_last_error());
}
void require_usable(const stc_group& g) {
  if (g.broken) throw Error(STC_ERR_STATE, "the group's RCCL communicator was aborted after a member failed (" +
                                               g.broken_why + "): destroy the group and create a new one");
}
// f(i) for every member on its own thread (device set); the first failure is rethrown here.
// In-process transport: a failure releases the members waiting in its barrier, and the group stays usable.
// RCCL: a failure sets the group's abort flag, so every member's next wait throws instead of waiting for a
// collective the failed member never enqueued; a member still blocked inside the runtime after a grace
// period (a copy queued behind such a collective) has its communicator aborted by this thread, which
// releases the collective's kernels; after the join every member's communicator is aborted and the group
// is broken (STC_ERR_STATE from then on; stc_group_destroy returns).
template <typename F>
void for_members(stc_group& g, F f) {
  require_usable(g);
  const int n = g.n();
  const bool rccl = g.transport == STC_TRANSPORT_RCCL;
  std::vector<std::exception_ptr> err((size_t)n);
  std::mutex fm;
  std::condition_variable fcv;
  int first = -1;  // the member that failed first (the others may only report "another member failed")
  int running = n;
  auto run = [&](int i) {
    try {
      g.ctx[(size_t)i]->use();
      f(i);
    } catch (...) {
      err[(size_t)i] = std::current_exception();
      {
        std::lock_guard<std::mutex> lk(fm);
        if (first < 0) first = i;
      }
      if (g.local) g.local->fail();  // release the members waiting in a barrier
      if (rccl) g.abort.store(true);
    }
    std::lock_guard<std::mutex> lk(fm);
    --running;
    fcv.notify_all();
  };
  if (n == 1 && !g.threaded) {
    run(0);
  } else {
    std::vector<std::thread> th;
    th.reserve((size_t)n);
    for (int i = 0; i < n; ++i) th.emplace_back(run, i);
    if (rccl) {
      std::unique_lock<std::mutex> lk(fm);
      fcv.wait(lk, [&] { return running == 0 || first >= 0; });
      if (running > 0 && !fcv.wait_for(lk, std::chrono::seconds(5), [&] { return running == 0; }))
        for (auto* c : g.ctx) abort_comm(*c);  // members still blocked behind the failed member's collectives
    }
    for (auto& t : th) t.join();
  }
  if (g.local) {  // a failed call leaves the transport usable for the next one
    std::lock_guard<std::mutex> lk(g.local->m);
    g.local->broken = false;
    g.local->arrived = 0;
  }
  if (first >= 0) {
    if (rccl) {
      for (auto* c : g.ctx) {
        c->use();
        abort_comm(*c);
      }
      g.broken = true;
      try {
        std::rethrow_exception(err[(size_t)first]);
      } catch (const std::exception& e) {
        g.broken_why = "member " + std::to_string(first) + ": " + e.what();
      } catch (...) {
        g.broken_why = "member " + std::to_string(first);
      }
    }
    std::rethrow_exception(err[(size_t)first]);
  }
}
// contiguous row ranges of a host CSR, one per member, balanced by entries
std::vector<int64_t> shard_rows(const int64_t* indptr, int64_t rows, int n) {
  std::vector<int64_t> r0((size_t)n + 1, rows);
  r0[0] = 0;
  const int64_t nnz = indptr[rows];
  int64_t r = 0;
  for (int q = 1; q < n; ++q) {
    const int64_t target = (nnz * q + n - 1) / n;
    while (r < rows && indptr[r] < target) ++r;
    r0[(size_t)q] = std::max(r, r0[(size_t)q - 1]);
  }
  return r0;
}
// member i's rows [r0[i], r0[i+1]) of a host CSR uploaded to its device (indptr rebased)
stc_dcsr* upload_rows(stc_ctx* ctx, int64_t lo, int64_t hi, int64_t cols, const int64_t* indptr,
                      const int32_t* indices, const double* values, int dtype) {
  std::vector<int64_t> ip((size_t)(hi - lo + 1));
  for (int64_t r = lo; r <= hi; ++r) ip[(size_t)(r - lo)] = indptr[r] - indptr[lo];
  stc_dcsr* d = nullptr;
  member_ok(stc_dcsr_upload(ctx, hi - lo, cols, ip.data(), indices ? indices + indptr[lo] : nullptr,
                            values ? values + indptr[lo] : nullptr, dtype, &d));
  return d;
}
void check_host_csr(int64_t rows, int64_t cols, const int64_t* indptr, const int32_t* indices,
                    const double* values) {
  STC_REQUIRE(indptr && rows >= 0, "indptr / rows");
  STC_REQUIRE(indptr[rows] == 0 || (indices && values), "indices / values");
  check_csr_host(rows, cols, indptr, indices);
}

}  // namespace

extern "C" {

int stc_group_create(const int* device_ids, int n_devices, const stc_lda_config* cfg, stc_group** out) {
  return guard([&] {
    STC_REQUIRE(device_ids && cfg && out, "device_ids/cfg/out");
    STC_REQUIRE(n_devices >= 1 && n_devices <= kMaxMembers, "1 <= n_devices <= 16");
    int nd = 0;
    HIP_CHECK(hipGetDeviceCount(&nd));
    bool same = true, distinct = true;
    for (int i = 0; i < n_devices; ++i) {
      STC_REQUIRE(device_ids[i] >= 0 && device_ids[i] < nd, "device index out of range");
      same &= device_ids[i] == device_ids[0];
      for (int j = 0; j < i; ++j) distinct &= device_ids[i] != device_ids[j];
    }
    STC_REQUIRE(same || distinct, "device_ids: all distinct (RCCL) or all the same device (in-process)");
    auto g = std::make_unique<stc_group>();
    struct Cleanup {
      stc_group* g;
      ~Cleanup() {
        if (!g) return;
        for (auto* l : g->lda) (void)stc_lda_destroy(l);
        for (auto* c : g->ctx) (void)stc_destroy(c);
      }
    } cleanup{g.get()};
    for (int i = 0; i < n_devices; ++i) {
      stc_ctx* c = nullptr;
      member_ok(stc_init(device_ids[i], &c));
      g->ctx.push_back(c);
    }
    // debug knob STC_GROUP_RCCL=1: a group of distinct devices — one device included — builds its RCCL
    // communicator with ncclCommInitAll, runs the collective (vocabulary-sliced) M-step even with one member,
    // and drives every member from its own host thread: the configs[2] drop-in path (one JVM, N GPUs,
    // LDATraining.scala:7) exercised end to end on a one-GPU box, where no two-device communicator exists
    const char* gr = getenv("STC_GROUP_RCCL");
    const bool rccl1 = gr && gr[0] == '1' && distinct;
    if (n_devices > 1 && same) {
      g->local = std::make_unique<LocalColl>(n_devices);
      g->transport = STC_TRANSPORT_IN_PROCESS;
    }
    if (n_devices > 1 || rccl1) {
      std::vector<ncclComm_t> comms((size_t)n_devices, nullptr);
      if (!g->local) {
        RCCL_CHECK(ncclCommInitAll(comms.data(), n_devices, device_ids));
        g->transport = STC_TRANSPORT_RCCL;
      }
      g->threaded = rccl1;
      for (int i = 0; i < n_devices; ++i) {
        g->ctx[(size_t)i]->comm = comms[(size_t)i];
        g->ctx[(size_t)i]->local = g->local.get();
        g->ctx[(size_t)i]->n_ranks = n_devices;
        g->ctx[(size_t)i]->rank = i;
      }
    }
    for (auto* c : g->ctx) c->abort_flag = &g->abort;
    // test knob STC_GROUP_STEP_FAULT=i[:s]: member i's s-th step (default the first) fails, after its E-step
    // and sstats and before its reduce-scatter (its peers' collectives then never complete: the RCCL
    // failure path)
    const char* sf = getenv("STC_GROUP_STEP_FAULT");
    const int step_fault = sf && sf[0] ? atoi(sf) : -1;
    const char* sfc = sf ? std::strchr(sf, ':') : nullptr;
    const int step_fault_at = sfc ? std::max(1, atoi(sfc + 1)) : 1;
    for (int i = 0; i < n_devices; ++i) {
      stc_lda* l = nullptr;
      member_ok(stc_lda_create(g->ctx[(size_t)i], cfg, &l));
      if (rccl1) l->force_coll = true;  // the sliced M-step and its collectives on a 1-rank communicator too
      l->tail_fault = i == step_fault ? step_fault_at : 0;
      g->lda.push_back(l);
    }
    g->dtype = corpus_dtype(*g->lda[0]);  // the shards' value dtype
    g->row0.assign((size_t)n_devices + 1, 0);
    cleanup.g = nullptr;
    *out = g.release();
  });
}

int stc_group_destroy(stc_group* g) {
  return guard([&] {
    if (!g) return;
    for (auto* l : g->lda) (void)stc_lda_destroy(l);
    for (auto* d : g->shard) (void)stc_dcsr_free(d);
    for (auto* c : g->ctx) {
      c->local = nullptr;
      (void)stc_destroy(c);
    }
    delete g;
  });
}

int stc_group_size(const stc_group* g, int* n_out) {
  return guard([&] {
    STC_REQUIRE(g && n_out, "group/n_out");
    *n_out = g->n();
  });
}

int stc_group_transport(const stc_group* g, int* transport_out) {
  return guard([&] {
    STC_REQUIRE(g && transport_out, "group/transport_out");
    *transport_out = g->transport;
  });
}

int stc_group_member(stc_group* g, int i, stc_lda** lda_out) {
  return guard([&] {
    STC_REQUIRE(g && lda_out && i >= 0 && i < g->n(), "group/member index");
    *lda_out = g->lda[(size_t)i];
  });
}

int stc_group_set_corpus(stc_group* g, int64_t n_rows, int64_t n_cols, const int64_t* indptr, const int32_t* indices,
                         const double* values) {
  return guard([&] {
    STC_REQUIRE(g, "group");
    check_host_csr(n_rows, n_cols, indptr, indices, values);
    const std::vector<int64_t> r0 = shard_rows(indptr, n_rows, g->n());
    std::vector<stc_dcsr*> shard((size_t)g->n(), nullptr);
    try {
      // every shard uploaded before any member is switched to it: a failed upload (out of memory) leaves
      // every member on its previous shard
      const char* fe = getenv("STC_GROUP_UPLOAD_FAULT");  // debug knob: member i's upload fails (tests)
      const int fault = fe ? atoi(fe) : -1;
      for_members(*g, [&](int i) {
        if (i == fault) throw Error(STC_ERR_OOM, "injected shard upload failure (STC_GROUP_UPLOAD_FAULT)");
        shard[(size_t)i] = upload_rows(g->ctx[(size_t)i], r0[(size_t)i], r0[(size_t)i + 1], n_cols, indptr, indices,
                                       values, g->dtype);
      });
      for_members(*g, [&](int i) { member_ok(stc_lda_set_corpus(g->lda[(size_t)i], shard[(size_t)i], n_rows)); });
    } catch (...) {
      // members already switched go back to their previous shard (or to none) before the new ones are freed
      for (int i = 0; i < g->n(); ++i) {
        stc_lda* l = g->lda[(size_t)i];
        if (!shard[(size_t)i] || l->corpus != shard[(size_t)i]) continue;
        stc_dcsr* old = (size_t)i < g->shard.size() ? g->shard[(size_t)i] : nullptr;
        if (!old || stc_lda_set_corpus(l, old, g->rows) != STC_OK) l->corpus = nullptr;
      }
      for (auto* d : shard) (void)stc_dcsr_free(d);
      throw;
    }
    for (auto* d : g->shard) (void)stc_dcsr_free(d);
    g->shard = shard;
    g->row0 = r0;
    g->rows = n_rows;
    g->cols = n_cols;
  });
}

int stc_group_release_corpus(stc_group* g) {
  return guard([&] {
    STC_REQUIRE(g, "group");
    require_usable(*g);
    for (int i = 0; i < g->n(); ++i) {
      stc_lda* l = g->lda[(size_t)i];
      g->ctx[(size_t)i]->use();
      settle_side(*l);
      wait_stream(*g->ctx[(size_t)i], g->ctx[(size_t)i]->stream);
      l->corpus = nullptr;
      l->order_for = nullptr;
      l->pre_valid = false;
    }
    for (auto* d : g->shard) (void)stc_dcsr_free(d);
    g->shard.clear();
    g->rows = 0;
  });
}

int stc_group_init_random(stc_group* g, uint64_t seed) {
  return guard([&] {
    STC_REQUIRE(g, "group");
    for_members(*g, [&](int i) { member_ok(stc_lda_init_random(g->lda[(size_t)i], seed)); });
  });
}

int stc_group_set_topics(stc_group* g, const double* topics, int layout) {
  return guard([&] {
    STC_REQUIRE(g && topics, "group/topics");
    for_members(*g, [&](int i) { member_ok(stc_lda_set_topics(g->lda[(size_t)i], topics, layout)); });
  });
}

int stc_group_get_topics(stc_group* g, double* topics_out, int layout) {
  return guard([&] {
    STC_REQUIRE(g && topics_out, "group/topics_out");
    // gathering the sharded λ is collective: member 0 copies it out, the others only take part
    for_members(*g, [&](int i) {
      if (i == 0) member_ok(stc_lda_get_topics(g->lda[0], topics_out, layout));
      else gather_lambda(*g->lda[(size_t)i]);
    });
  });
}

int stc_group_get_alpha(stc_group* g, double* alpha_out) {
  return guard([&] {
    STC_REQUIRE(g && alpha_out, "group/alpha_out");
    require_usable(*g);
    g->ctx[0]->use();
    member_ok(stc_lda_get_alpha(g->lda[0], alpha_out));  // α is replicated on every member
  });
}

int stc_group_get_iteration(stc_group* g, int64_t* iteration_out) {
  return guard([&] {
    STC_REQUIRE(g && iteration_out, "group/iteration_out");
    *iteration_out = g->lda[0]->iteration;
  });
}

int stc_group_synchronize(stc_group* g) {
  return guard([&] {
    STC_REQUIRE(g, "group");
    require_usable(*g);
    for (int i = 0; i < g->n(); ++i) {
      g->ctx[(size_t)i]->use();
      wait_stream(*g->ctx[(size_t)i], g->ctx[(size_t)i]->stream);
      if (g->lda[(size_t)i]->side) wait_stream(*g->ctx[(size_t)i], g->lda[(size_t)i]->side);  // the next draw
    }
  });
}

static void merge_stats(stc_step_stats* out, const std::vector<stc_step_stats>& st) {
  if (!out) return;
  *out = stc_step_stats{};
  for (const auto& s : st) {
    out->batch_docs += s.batch_docs;
    out->batch_entries += s.batch_entries;
    out->inner_iters += s.inner_iters;
    out->inner_iters_max = std::max(out->inner_iters_max, s.inner_iters_max);
    out->cap_hits += s.cap_hits;
  }
  out->nonempty_docs = st[0].nonempty_docs;  // already summed over the members
  out->rho = st[0].rho;
}

int stc_group_next(stc_group* g, stc_step_stats* stats) {
  return guard([&] {
    STC_REQUIRE(g, "group");
    std::vector<stc_step_stats> st((size_t)g->n());
    for_members(*g, [&](int i) { member_ok(stc_lda_next(g->lda[(size_t)i], stats ? &st[(size_t)i] : nullptr)); });
    merge_stats(stats, st);
  });
}

int stc_group_step(stc_group* g, const int64_t* batch_doc_ids, int64_t n, const double* gamma0, stc_step_stats* stats) {
  return guard([&] {
    STC_REQUIRE(g && (batch_doc_ids || n == 0) && n >= 0, "group/batch_doc_ids");
    const int m = g->n();
    const int64_t k = g->lda[0]->k;
    std::vector<std::vector<int64_t>> ids((size_t)m);
    std::vector<std::vector<double>> g0((size_t)m);
    for (int64_t j = 0; j < n; ++j) {
      const int64_t d = batch_doc_ids[j];
      STC_REQUIRE(d >= 0 && d < g->rows, "batch doc id out of range");
      const int q = (int)(std::upper_bound(g->row0.begin(), g->row0.end(), d) - g->row0.begin()) - 1;
      ids[(size_t)q].push_back(d - g->row0[(size_t)q]);
      if (gamma0) g0[(size_t)q].insert(g0[(size_t)q].end(), gamma0 + j * k, gamma0 + (j + 1) * k);
    }
    std::vector<stc_step_stats> st((size_t)m);
    for_members(*g, [&](int i) {
      const auto& v = ids[(size_t)i];
      member_ok(stc_lda_step(g->lda[(size_t)i], v.data(), (int64_t)v.size(), gamma0 ? g0[(size_t)i].data() : nullptr,
                             stats ? &st[(size_t)i] : nullptr));
    });
    merge_stats(stats, st);
  });
}

int stc_group_describe(stc_group* g, int32_t max_terms, int32_t* idx_out, double* weight_out) {
  return guard([&] {
    STC_REQUIRE(g && idx_out && weight_out, "group/idx_out/weight_out");
    for_members(*g, [&](int i) {
      if (i == 0) member_ok(stc_lda_describe(g->lda[0], max_terms, idx_out, weight_out));
      else gather_lambda(*g->lda[(size_t)i]);
    });
  });
}

int stc_group_bound(stc_group* g, int64_t n_rows, int64_t n_cols, const int64_t* indptr, const int32_t* indices,
                    const double* values, uint64_t gamma_seed, int64_t doc_id_base, const double* gamma0,
                    double* bound_out, double* corpus_part_out, double* topics_part_out, double* token_count_out) {
  return guard([&] {
    STC_REQUIRE(g && bound_out, "group/bound_out");
    check_host_csr(n_rows, n_cols, indptr, indices, values);
    const std::vector<int64_t> r0 = shard_rows(indptr, n_rows, g->n());
    const int64_t k = g->lda[0]->k;
    double res[4] = {0, 0, 0, 0};
    for_members(*g, [&](int i) {
      const int64_t lo = r0[(size_t)i], hi = r0[(size_t)i + 1];
      stc_dcsr* d = upload_rows(g->ctx[(size_t)i], lo, hi, n_cols, indptr, indices, values, g->dtype);
      double r[4] = {0, 0, 0, 0};
      // every member's γ₀ keys continue the global row numbering (doc_id_base + row), so the bound is
      // the one a single handle computes over all rows
      const int rc = stc_lda_bound(g->lda[(size_t)i], d, gamma_seed, doc_id_base + lo, gamma0 ? gamma0 + lo * k : nullptr,
                                   &r[0], &r[1], &r[2], &r[3]);
      (void)stc_dcsr_free(d);
      member_ok(rc);
      if (i == 0) std::copy(r, r + 4, res);  // the bound is all-reduced: every member holds the total
    });
    *bound_out = res[0];
    if (corpus_part_out) *corpus_part_out = res[1];
    if (topics_part_out) *topics_part_out = res[2];
    if (token_count_out) *token_count_out = res[3];
  });
}

int stc_group_topic_distribution(stc_group* g, int64_t n_rows, int64_t n_cols, const int64_t* indptr,
                                 const int32_t* indices, const double* values, uint64_t gamma_seed,
                                 int64_t doc_id_base, const double* gamma0, double* out) {
  return guard([&] {
    STC_REQUIRE(g && out, "group/out");
    check_host_csr(n_rows, n_cols, indptr, indices, values);
    const std::vector<int64_t> r0 = shard_rows(indptr, n_rows, g->n());
    const int64_t k = g->lda[0]->k;
    for_members(*g, [&](int i) {
      const int64_t lo = r0[(size_t)i], hi = r0[(size_t)i + 1];
      stc_dcsr* d = upload_rows(g->ctx[(size_t)i], lo, hi, n_cols, indptr, indices, values, g->dtype);
      const int rc = stc_lda_topic_distribution(g->lda[(size_t)i], d, gamma_seed, doc_id_base + lo,
                                                gamma0 ? gamma0 + lo * k : nullptr, out + lo * k);
      (void)stc_dcsr_free(d);
      member_ok(rc);
    });
  });
}

}  // extern "C"
