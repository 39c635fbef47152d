// stc_internal.h — internals shared by the libstc.so translation units (gfx950 / HIP only).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "stc.h"

namespace stc {

// device UTF-8 token blobs are allocated this many bytes past their end: hashing_tf.hip reads each
// token as a 32-byte window of whole aligned dwords from its aligned start
constexpr int64_t kHashPad = 64;

// ---------------------------------------------------------------------------------------
// Errors: every entry point runs inside guard(); failures throw stc::Error and come back to
// the caller as a status code + thread-local message (stc_last_error).  Never abort().
// ---------------------------------------------------------------------------------------
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

template <typename F>
int guard(F&& f) {
  try {
    f();
    return STC_OK;
  } catch (const Error& e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error("host out of memory");
    return STC_ERR_OOM;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return STC_ERR_STATE;
  }
}

#define STC_REQUIRE(cond, msg)                                                          \
  do {                                                                                  \
    if (!(cond)) throw ::stc::Error(STC_ERR_INVALID_ARG, std::string("requirement failed: ") + (msg)); \
  } while (0)

#define HIP_CHECK(expr)                                                                 \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      int c_ = (e_ == hipErrorOutOfMemory) ? STC_ERR_OOM : STC_ERR_HIP;                 \
      throw ::stc::Error(c_, std::string(#expr) + ": " + hipGetErrorString(e_) + " @" + \
                                 __FILE__ + ":" + std::to_string(__LINE__));            \
    }                                                                                   \
  } while (0)

#define RCCL_CHECK(expr)                                                                \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess)                                                              \
      throw ::stc::Error(STC_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

#define KERNEL_CHECK() HIP_CHECK(hipGetLastError())

// ---------------------------------------------------------------------------------------
// Device buffer (grow-only scratch).  Allocation happens only outside the launch sequence.
// ---------------------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void reserve(size_t n) {
    if (n <= bytes) return;
    release();
    size_t want = n < 256 ? 256 : n;
    HIP_CHECK(hipMalloc(&p, want));
    bytes = want;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

// Device allocations a freed stc_dcsr handed back to the context that made it, so the next output of a
// similar size (HashingTF, upload) takes one instead of calling hipMalloc (tens of µs for GB-sized
// buffers, inside every call).  At most kMax are kept; the context frees them when it is destroyed.
struct Recycler {
  static constexpr size_t kMax = 6;
  static constexpr size_t kMin = size_t(1) << 20;  // smaller buffers are freed, not kept
  std::mutex mu;
  std::vector<std::pair<void*, size_t>> bufs;
  void put(DevBuf& b) {  // takes b's allocation (b is empty afterwards)
    if (!b.p || b.bytes < kMin) return;
    std::lock_guard<std::mutex> lk(mu);
    if (bufs.size() >= kMax) {  // drop the smallest kept one (or this one)
      size_t sm = 0;
      for (size_t i = 1; i < bufs.size(); ++i)
        if (bufs[i].second < bufs[sm].second) sm = i;
      if (bufs[sm].second >= b.bytes) return;
      (void)hipFree(bufs[sm].first);
      bufs.erase(bufs.begin() + (std::ptrdiff_t)sm);
    }
    bufs.emplace_back(b.p, b.bytes);
    b.p = nullptr;
    b.bytes = 0;
  }
  void take(DevBuf& b, size_t n) {  // b.reserve(n), from a kept allocation of n…2n bytes when one exists
    if (n <= b.bytes) return;
    {
      std::lock_guard<std::mutex> lk(mu);
      size_t best = bufs.size();
      for (size_t i = 0; i < bufs.size(); ++i)
        if (bufs[i].second >= n && bufs[i].second <= 2 * n && (best == bufs.size() || bufs[i].second < bufs[best].second))
          best = i;
      if (best < bufs.size()) {
        b.release();
        b.p = bufs[best].first;
        b.bytes = bufs[best].second;
        bufs.erase(bufs.begin() + (std::ptrdiff_t)best);
        return;
      }
    }
    b.reserve(n);
  }
  ~Recycler() {
    for (auto& x : bufs) (void)hipFree(x.first);
  }
};

// ---------------------------------------------------------------------------------------
// Context: one device, one stream, optional RCCL communicator.
// ---------------------------------------------------------------------------------------
struct LocalColl;  // in-process collectives of the stc_group members that share one device (api.hip)
struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  LocalColl* local = nullptr;  // set instead of comm for same-device group members (owned by the group)
  int n_ranks = 1;
  int rank = 0;
  int cus = 256;          // compute units (the df count sizes its grid to one workgroup per CU)
  bool df_tiled = true;   // idf.hip doc_freq: the tiled count (false: the binned one, STC_DF_BINNED=1)
  bool df_rows16 = true;  // … its row-grouped u16 form for unique-id rows (STC_DF_U32=1: off)
  // hashing_tf.hip build_csr when every document fits the register sort (STC_TF_MODE): 0 the round-3
  // passes (hash + sort → sorted keys, scan, runs), 1 (default) hash + sort + emit in one look-back pass,
  // 2 a flat hash then the look-back sort + emit pass
  int tf_mode = 1;
  bool tf_force_fault = false;  // test knob (STC_TF_FAULT=1): every look-back gives up at once
  int64_t tf_fallbacks = 0;     // single passes that fell back to the sorted-key passes
  bool idf_cache = true;  // idf.hip: the device IDF model's hot-idf LDS table (STC_IDF_NO_CACHE=1: off)
  Recycler recycle;    // freed stc_dcsr allocations for the next outputs (stc_dcsr_free)
  DevBuf scratch[12];  // grow-only scratch of the featurisation kernels (hashing_tf.hip, idf.hip, api.hip IDF)
  DevBuf coll_tmp;    // the in-process all-reduce's staging buffer
  // RCCL failure handling (api.hip wait_stream / wait_event): with a communicator, every wait on work that
  // may hold a collective polls with a deadline instead of blocking in the runtime
  const std::atomic<bool>* abort_flag = nullptr;  // the group's: set once any of its members has failed
  std::atomic<bool> comm_aborted{false};          // comm was aborted (ncclCommAbort): never used again
  int64_t coll_timeout_ms = 120000;               // STC_COLL_TIMEOUT_MS (read at stc_init)
  bool in_group = false;                          // between ncclGroupStart and ncclGroupEnd
  bool coll_enqueued = false;                     // a collective was ever enqueued (waits poll from then on)
  void use() const { HIP_CHECK(hipSetDevice(device)); }
  bool coll() const { return comm != nullptr || local != nullptr; }
};

struct DCsr {
  Ctx* ctx = nullptr;  // the context that made it; only it may read the buffers (checked at the ABI)
  int device = -1;     // for stc_dcsr_free, which may run after that context is gone
  int64_t rows = 0, cols = 0, nnz = 0;
  int64_t max_row = -1;  // longest row's nnz when known (host uploads), −1 otherwise
  int dtype = STC_F64;
  // every value is > 0 (a HashingTF output: counts / binary 1; kept by a floored IDF transform), so a
  // df count needs only the indices (cleared by anything that may write a value ≤ 0)
  bool positive = false;
  // every row holds an id at most once (a HashingTF output; kept by the transform): idf.hip may count df
  // in u16 per group of ≤ 65535 rows
  bool unique_ids = false;
  DevBuf indptr;   // int64[rows+1]
  DevBuf indices;  // int32[nnz]
  DevBuf values;   // float/double[nnz]
};

// ---------------------------------------------------------------------------------------
// Counter-based RNG shared bit-for-bit with oracle/oracle.py (splitmix64 streams, uniform
// in (0,1) from the top 53 bits, Box–Muller normal, Marsaglia–Tsang Gamma(shape, 1/shape)).
// ---------------------------------------------------------------------------------------
__host__ __device__ inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t doc_stream(uint64_t seed, uint64_t key) {
  return splitmix64(seed ^ splitmix64(key));
}
__host__ __device__ inline double rng_uniform(uint64_t stream, uint64_t ctr) {
  uint64_t x = splitmix64(stream + ctr * 0xD1B54A32D192ED03ull);
  return ((double)(x >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}
__host__ __device__ inline double gamma_sample(uint64_t stream, int topic, double shape) {
  const double d = shape - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  double v = 1.0;
  for (int attempt = 0; attempt < 64; ++attempt) {
    const uint64_t base = ((uint64_t)topic << 8) + 3u * (uint64_t)attempt;
    const double u1 = rng_uniform(stream, base);
    const double u2 = rng_uniform(stream, base + 1);
    const double x = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = rng_uniform(stream, base + 2);
    if (u < 1.0 - 0.0331 * (x * x) * (x * x)) break;
    if (log(u) < 0.5 * x * x + d * (1.0 - v + log(v))) break;
  }
  return d * v / shape;
}
// γ₀ key of a training minibatch member (mirrors oracle.train_doc_key)
__host__ __device__ inline uint64_t train_doc_key(int64_t iteration, int rank, int64_t pos) {
  return (((uint64_t)iteration & 0xFFFFFFull) << 40) | (((uint64_t)rank & 0xFFull) << 32) |
         ((uint64_t)pos & 0xFFFFFFFFull);
}

// ---------------------------------------------------------------------------------------
// Breeze 0.13.2 digamma / trigamma (recurrence to x > 5 + asymptotic series).
// ---------------------------------------------------------------------------------------
template <typename R>
__host__ __device__ inline R digamma_t(R x) {
  R r = 0;
  while (x <= R(5)) {
    r -= R(1) / x;
    x += R(1);
  }
  const R f = R(1) / (x * x);
  const R t = f * (R(-1.0 / 12.0) + f * (R(1.0 / 120.0) + f * (R(-1.0 / 252.0) + f * (R(1.0 / 240.0) +
              f * (R(-1.0 / 132.0) + f * (R(691.0 / 32760.0) + f * (R(-1.0 / 12.0) + f * R(3617.0) / R(8160.0))))))));
  return r + log(x) - R(0.5) / x + t;
}
// ln x for positive normal x: v_log_f32 (log2) · ln 2, without the denormal-range fixup __logf carries
__device__ __forceinline__ float ln_pos(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }
// fp32 digamma for the E-step inner loop: ψ(x) = ψ(x+4) − 1/x − (3x²+12x+11)/((x+1)(x+2)(x+3))
// unconditionally (no data-dependent loop ⇒ no lane divergence; the three shifted reciprocals share
// one v_rcp_f32, 1/x keeps its own for the small-γ end), v_log_f32, and Breeze's asymptotic series
// at x+4 ≥ 4 (first omitted term < 2e-9).  Accuracy vs the shift-6 form: tools/dg_check.py.
__device__ inline float digamma_fast(float x) {
  const float num = fmaf(fmaf(3.f, x, 12.f), x, 11.f);
  const float den = fmaf(fmaf(x + 6.f, x, 11.f), x, 6.f);
  const float r = __builtin_amdgcn_rcpf(x) + num * __builtin_amdgcn_rcpf(den);
  const float y = x + 4.f;
  const float iy = __builtin_amdgcn_rcpf(y);
  const float f = iy * iy;
  const float t = f * (-1.f / 12.f + f * (1.f / 120.f + f * (-1.f / 252.f + f * (1.f / 240.f + f * (-1.f / 132.f)))));
  return ln_pos(y) - 0.5f * iy + t - r;
}

// fp64 1/q from v_rcp_f64 and two Newton steps (≤ 1 ulp apart from the correctly rounded quotient)
__device__ __forceinline__ double rcp_nr(double q) {
  double r = __builtin_amdgcn_rcp(q);
  r = fma(r, fma(-q, r, 1.0), r);
  return fma(r, fma(-q, r, 1.0), r);
}
// Breeze evaluates its 8-term asymptotic series S8 at y_B = x + ⌊5 − x⌋ + 1 ∈ (5, 6]; the fast forms
// below evaluate it at x + 6 ∈ (6, 11] (one rational for the six recurrence terms).  S8's truncation
// error E(y) = ψ(y) − S8(y) reaches 8e-13 at y = 5, which a slowly-dying topic of a long E-step
// amplifies past 1e-7 relative, so the difference E(x + 6) − E(y_B) is added back: E(y) = f⁹·P(f),
// f = 1/y², P fitted to 7e-18 absolute on y ∈ [5, 11.5] (tools/fit_breeze_digamma.py).
__device__ __forceinline__ double breeze_trunc(double iy) {
  const double f = iy * iy, f2 = f * f, f4 = f2 * f2;
  return f4 * f4 * f * (-3.053401198888146 + f * (26.284421368293753 + f * (-260.94994774566294 +
                        f * (2372.137971404805 + f * -12318.55039822477))));
}
__device__ __forceinline__ double breeze_shift_fix(double x, double iy6, bool sh) {
  const double yb = sh ? x + (floor(5.0 - x) + 1.0) : 6.0;  // E needs ~1e-4 relative: raw v_rcp_f64
  return breeze_trunc(iy6) - breeze_trunc(__builtin_amdgcn_rcp(yb));
}
// fp64 digamma for the M-step's V×k elements, branch-free: Breeze's recurrence Σ_{i<6} 1/(x+i) for
// x ≤ 5 as one rational Q'(x)/Q(x), Q = x(x+1)…(x+5), the same 8-term asymptotic series at y = x + 6
// (or y = x when x > 5, where Breeze does not shift) and breeze_shift_fix.  Agrees with
// digamma_t<double> to a few ulp; the loop form costs a divergent chain of up to six fp64 divisions.
__device__ inline double digamma_fast_d(double x) {
  const bool sh = x <= 5.0;
  const double q = ((((((x + 15.0) * x + 85.0) * x + 225.0) * x + 274.0) * x + 120.0) * x);
  const double p = (((((6.0 * x + 75.0) * x + 340.0) * x + 675.0) * x + 548.0) * x + 120.0);
  const double iq = rcp_nr(sh ? q : 1.0);
  double c = p * iq;
  c = fma(fma(-q, c, p), iq, c);  // one residual correction of p/q
  const double y = sh ? x + 6.0 : x;
  const double iy = rcp_nr(y);
  const double f = iy * iy;
  const double t = f * (-1.0 / 12.0 + f * (1.0 / 120.0 + f * (-1.0 / 252.0 + f * (1.0 / 240.0 +
                   f * (-1.0 / 132.0 + f * (691.0 / 32760.0 + f * (-1.0 / 12.0 + f * (3617.0 / 8160.0))))))));
  return (sh ? breeze_shift_fix(x, iy, sh) - c : 0.0) + log(y) - 0.5 * iy + t;
}
// exp(ψ(x) − cst) for the fp64 E-step's eθ = exp(ψ(γ) − ψ(Σγ)), without the logarithm: with ψ(x) =
// ln y − 0.5/y + t(y) − s(x) as in digamma_fast_d, exp(ψ(x) − cst) = y · exp(t − 0.5/y − s − cst).
__device__ inline double exp_digamma_minus_d(double x, double cst) {
  const bool sh = x <= 5.0;
  const double q = ((((((x + 15.0) * x + 85.0) * x + 225.0) * x + 274.0) * x + 120.0) * x);
  const double p = (((((6.0 * x + 75.0) * x + 340.0) * x + 675.0) * x + 548.0) * x + 120.0);
  const double iq = rcp_nr(sh ? q : 1.0);
  double c = p * iq;
  c = fma(fma(-q, c, p), iq, c);
  const double y = sh ? x + 6.0 : x;
  const double iy = rcp_nr(y);
  const double f = iy * iy;
  const double t = f * (-1.0 / 12.0 + f * (1.0 / 120.0 + f * (-1.0 / 252.0 + f * (1.0 / 240.0 +
                   f * (-1.0 / 132.0 + f * (691.0 / 32760.0 + f * (-1.0 / 12.0 + f * (3617.0 / 8160.0))))))));
  return y * exp(((sh ? breeze_shift_fix(x, iy, sh) - c : 0.0) - 0.5 * iy + t) - cst);
}

__host__ __device__ inline double trigamma_d(double x) {
  double r = 0;
  while (x <= 5.0) {
    r += 1.0 / (x * x);
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  const double t = f * (1 / 6.0 + f * (-1 / 30.0 + f * (1 / 42.0 + f * (-1 / 30.0 + f * (5 / 66.0 +
                   f * (-691 / 2730.0 + f * (7 / 6.0 - f * 3617 / 510.0)))))));
  return r + 1.0 / x + f / 2.0 + t / x;
}

// ---------------------------------------------------------------------------------------
// Wave64 / block reductions
// ---------------------------------------------------------------------------------------
// fp32 wave64 all-reduce without LDS: two permlane swaps (across 32 / 16 lanes) and four DPP
// involutions inside each 16-lane row (row_mirror, row_half_mirror, quad_perm 1032 and 2301).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  // all-lanes-valid permutations only (mirrors, quad_perm): bound_ctrl never fires, no `old` operand
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// v_readlane of a float / double (wave-uniform lane index)
__device__ __forceinline__ float readlane_t(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ double readlane_t(double v, int l) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// max of two non-negative floats as an unsigned compare of their bits (no NaN canonicalisation)
__device__ __forceinline__ float max_nonneg(float a, float b) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b)));
}
// Compiler hazard (ROCm 7.2 hipcc, gfx950): with __builtin_amdgcn_permlane{16,32}_swap the compiler
// sometimes reads the FIRST result register for both results (`v_add v0, v0, v0` after the swap;
// seen whenever both operands carry the same value, even through an opaque copy).  The swaps are
// therefore issued as inline asm with both registers in/out; `s_nop 1` covers the VALU-write →
// permlane-read hazard the compiler inserts for the builtin.  `volatile` keeps the compiler from
// re-materialising a swap inside a divergent branch (inactive partner lanes ⇒ garbage).
__device__ __forceinline__ void pswap32(unsigned& x, unsigned& y) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void pswap16(unsigned& x, unsigned& y) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ float swap32_pair(float v, bool add, float w) {
  unsigned x = __builtin_bit_cast(unsigned, v), y = __builtin_bit_cast(unsigned, w);
  pswap32(x, y);
  const float a = __builtin_bit_cast(float, x), b = __builtin_bit_cast(float, y);
  return add ? a + b : fmaxf(a, b);
}
__device__ __forceinline__ float swap16_pair(float v, bool add, float w) {
  unsigned x = __builtin_bit_cast(unsigned, v), y = __builtin_bit_cast(unsigned, w);
  pswap16(x, y);
  const float a = __builtin_bit_cast(float, x), b = __builtin_bit_cast(float, y);
  return add ? a + b : fmaxf(a, b);
}
// Batched swaps: up to four independent swaps behind one hazard nop.
template <bool D32>
__device__ __forceinline__ void pswap_4(unsigned& a0, unsigned& b0, unsigned& a1, unsigned& b1, unsigned& a2,
                                        unsigned& b2, unsigned& a3, unsigned& b3) {
  if constexpr (D32)
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3\n\t"
                 "v_permlane32_swap_b32 %4, %5\n\tv_permlane32_swap_b32 %6, %7"
                 : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3));
  else
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\t"
                 "v_permlane16_swap_b32 %4, %5\n\tv_permlane16_swap_b32 %6, %7"
                 : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3));
}
template <bool D32>
__device__ __forceinline__ void pswap_2(unsigned& a0, unsigned& b0, unsigned& a1, unsigned& b1) {
  if constexpr (D32)
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3"
                 : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1));
  else
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3"
                 : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1));
}
template <bool D32>
__device__ __forceinline__ void pswap_1(unsigned& a0, unsigned& b0) {
  if constexpr (D32) pswap32(a0, b0);
  else pswap16(a0, b0);
}
// reduce-scatter step over lane distance 32 (D32) or 16, N pairs: lanes with the role bit clear
// keep the xs set, the others the ys set; out[i] = this lane's kept value + the partner's
template <bool D32, int N>
__device__ __forceinline__ void swap_add_n(const float* xs, const float* ys, float* out) {
  unsigned x[N], y[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    x[i] = __builtin_bit_cast(unsigned, xs[i]);
    y[i] = __builtin_bit_cast(unsigned, ys[i]);
  }
  constexpr int N4 = N / 4 * 4;
#pragma unroll
  for (int b = 0; b < N4; b += 4) pswap_4<D32>(x[b], y[b], x[b + 1], y[b + 1], x[b + 2], y[b + 2], x[b + 3], y[b + 3]);
  if constexpr (N - N4 >= 2) pswap_2<D32>(x[N4], y[N4], x[N4 + 1], y[N4 + 1]);
  if constexpr ((N - N4) % 2 == 1) pswap_1<D32>(x[N - 1], y[N - 1]);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = __builtin_bit_cast(float, x[i]) + __builtin_bit_cast(float, y[i]);
}
// three wave all-reduces at once (Σ a, Σ b, max c ≥ 0): the swaps share their hazard nops
__device__ __forceinline__ void wave_reduce3(float& a, float& b, float& c) {
  {
    unsigned a0 = __builtin_bit_cast(unsigned, a), a1 = a0, b0 = __builtin_bit_cast(unsigned, b), b1 = b0,
             c0 = __builtin_bit_cast(unsigned, c), c1 = c0, d0 = 0, d1 = 0;
    pswap_4<true>(a0, a1, b0, b1, c0, c1, d0, d1);
    a = __builtin_bit_cast(float, a0) + __builtin_bit_cast(float, a1);
    b = __builtin_bit_cast(float, b0) + __builtin_bit_cast(float, b1);
    c = max_nonneg(__builtin_bit_cast(float, c0), __builtin_bit_cast(float, c1));
  }
  {
    unsigned a0 = __builtin_bit_cast(unsigned, a), a1 = a0, b0 = __builtin_bit_cast(unsigned, b), b1 = b0,
             c0 = __builtin_bit_cast(unsigned, c), c1 = c0, d0 = 0, d1 = 0;
    pswap_4<false>(a0, a1, b0, b1, c0, c1, d0, d1);
    a = __builtin_bit_cast(float, a0) + __builtin_bit_cast(float, a1);
    b = __builtin_bit_cast(float, b0) + __builtin_bit_cast(float, b1);
    c = max_nonneg(__builtin_bit_cast(float, c0), __builtin_bit_cast(float, c1));
  }
  a += dpp_f<0x140>(a);
  b += dpp_f<0x140>(b);
  c = max_nonneg(c, dpp_f<0x140>(c));
  a += dpp_f<0x141>(a);
  b += dpp_f<0x141>(b);
  c = max_nonneg(c, dpp_f<0x141>(c));
  a += dpp_f<0xB1>(a);
  b += dpp_f<0xB1>(b);
  c = max_nonneg(c, dpp_f<0xB1>(c));
  a += dpp_f<0x4E>(a);
  b += dpp_f<0x4E>(b);
  c = max_nonneg(c, dpp_f<0x4E>(c));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = swap32_pair(v, true, v);
  v = swap16_pair(v, true, v);
  v += dpp_f<0x140>(v);  // row_mirror
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = swap32_pair(v, false, v);
  v = swap16_pair(v, false, v);
  v = fmaxf(v, dpp_f<0x140>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  return v;
}

template <typename R>
__device__ inline R wave_sum(R v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename R>
__device__ inline R wave_max(R v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// kernels-side entry points (implemented in the .hip files)
namespace hashing {
void hash_tokens(Ctx& c, const uint8_t* d_utf8, const int64_t* d_tok_off, int64_t n_tok,
                 int32_t num_features, int variant, int32_t* d_idx);
void row_order_by_df(Ctx& c, const DCsr& m, const int64_t* d_df, int32_t* d_order);
// token offsets as int64 (d_tok_off64) or, when d_tok_off32 is given, u32 (a resident upload's narrowed copy)
void build_csr(Ctx& c, const uint8_t* d_utf8, const int64_t* d_tok_off64, const uint32_t* d_tok_off32, int64_t n_tok,
               const int64_t* d_doc_off, int64_t n_docs, int32_t num_features, int binary,
               int variant, int value_dtype, int64_t max_doc /* longest document's tokens, −1 unknown */,
               DCsr& out);
void narrow_offsets(Ctx& c, const int64_t* d_src, int64_t n, uint32_t* d_dst);
}  // namespace hashing
namespace tokenizer {
// Spark ML Tokenizer on device: d_text/d_text_off (n_docs+1) in; lower-cased, separator-free blob,
// token offsets (n_tok+1) and per-document token offsets (n_docs+1) out (the blob may be up to half
// as long again as the input: Java 8 lower-cases a few 2-byte characters to 3 bytes).
void tokenize(Ctx& c, const uint8_t* d_text, const int64_t* d_text_off, int64_t n_docs,
              DevBuf& out_utf8, DevBuf& out_tok_off, DevBuf& out_doc_off, int64_t& n_tok,
              int64_t& n_out_bytes);
}  // namespace tokenizer
namespace idf {
// idf finalised inside the df reduction when the caller already knows m (no collective in between)
struct IdfFinal {
  double m;
  int64_t min_df;
  double* idf;
};
// df (cols); with fin, also idf when the path allows — returns true then (else call finalize)
bool doc_freq(Ctx& c, const DCsr& m, int64_t* d_df /* cols */, const IdfFinal* fin = nullptr);
void finalize(Ctx& c, const int64_t* d_df, int64_t cols, int64_t m, int64_t min_df, double* d_idf);
// cache: the hot-idf table build_cache made for this idf (nullptr: plain gathers)
void transform(Ctx& c, DCsr& m, const double* d_idf, double zero_floor, const DevBuf* cache = nullptr);
// the device IDF model's hot-idf table (false, cache untouched: vocabulary too large or disabled)
bool build_cache(Ctx& c, const int64_t* d_df, const double* d_idf, int64_t cols, DevBuf& cache);
}  // namespace idf

}  // namespace stc
