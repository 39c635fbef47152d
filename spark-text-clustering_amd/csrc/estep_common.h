// estep_common.h — pieces shared by the register-resident E-step kernels (lda_grid.hip,
// lda_grid.hip): Spark's φ epsilon in log space, packed-FMA operand type, reduce-scatter helpers
// and the diagnostic s_memtime stamps.
#pragma once

#include "lda_kernels.h"

namespace stc {
namespace lda {

constexpr double kLogEps = -230.25850929940458;  // ln(1e-100): Spark's φ epsilon (see lda.hip)
constexpr float kTiny = 1.17549435e-38f;         // FLT_MIN

typedef float f2 __attribute__((ext_vector_type(2)));  // v_pk_fma_f32 operand pair

constexpr int hup(int n) { return (n + 1) / 2; }

// reduce-scatter step through a DPP involution (row_mirror / row_half_mirror / quad_perm): lanes
// with the role bit clear keep topic set X, the others Y; the partner sends the set it drops.
template <int CTRL>
__device__ __forceinline__ float rs_dpp(float x, float y, bool hi) {
  const float keep = hi ? y : x;
  const float send = hi ? x : y;
  return keep + dpp_f<CTRL>(send);
}
// DPP controls (all lanes valid): row_mirror i↔15−i, row_half_mirror i↔7−i, row_ror:8 i↔i^8 (in a
// 16-lane row), quad_perm [3,2,1,0] i↔i^3, [1,0,3,2] i↔i^1, [2,3,0,1] i↔i^2
constexpr int DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_ROW_ROR8 = 0x128,
              DPP_QP_3210 = 0x1B, DPP_QP_1032 = 0xB1, DPP_QP_2301 = 0x4E;

// ---- fp64 cross-lane helpers (lda_rows64.hip, lda_wide.hip): a double moves as two dwords
typedef unsigned long long u64;

__device__ __forceinline__ unsigned lo32(double v) { return (unsigned)__builtin_bit_cast(u64, v); }
__device__ __forceinline__ unsigned hi32(double v) { return (unsigned)(__builtin_bit_cast(u64, v) >> 32); }
__device__ __forceinline__ double mkd(unsigned lo, unsigned hi) {
  return __builtin_bit_cast(double, ((u64)hi << 32) | lo);
}
// 64-bit DPP move as two 32-bit moves (all-lanes-valid permutations only)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)lo32(v), CTRL, 0xF, 0xF, true);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)hi32(v), CTRL, 0xF, 0xF, true);
  return mkd(lo, hi);
}
template <int CTRL>
__device__ __forceinline__ double rs_dpp_d(double x, double y, bool hi) {
  const double keep = hi ? y : x;
  const double send = hi ? x : y;
  return keep + dpp_d<CTRL>(send);
}
// reduce-scatter over lane distance 32 (D32) or 16 for N double pairs: both dwords of each value go
// through one v_permlane*_swap each (two values per hazard nop)
template <bool D32, int N>
__device__ __forceinline__ void swap_add_nd(const double* xs, const double* ys, double* out) {
  unsigned xl[N], xh[N], yl[N], yh[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    xl[i] = lo32(xs[i]);
    xh[i] = hi32(xs[i]);
    yl[i] = lo32(ys[i]);
    yh[i] = hi32(ys[i]);
  }
  constexpr int N2 = N / 2 * 2;
#pragma unroll
  for (int b = 0; b < N2; b += 2)
    pswap_4<D32>(xl[b], yl[b], xh[b], yh[b], xl[b + 1], yl[b + 1], xh[b + 1], yh[b + 1]);
  if constexpr (N % 2 == 1) pswap_2<D32>(xl[N - 1], yl[N - 1], xh[N - 1], yh[N - 1]);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = mkd(xl[i], xh[i]) + mkd(yl[i], yh[i]);
}
// The s-partial reduce-scatter of the grid E-steps (lda_rows64.hip, lda_team64.hip): lane = tl + 8·rl holds
// x[p] for its topic lane's KL ≤ 16 topics (zero-padded to 16); the eight row lanes rl (lane bits 3, 4, 5)
// are summed in a fixed order — bit 5 by permlane32 swaps, bit 4 by permlane16 swaps, bit 3 by row_ror:8 —
// so that lane (tl, rl) returns the wave sums of topics 2·rl and 2·rl + 1 of its topic lane.
__device__ __forceinline__ void rs_rows8(const double (&x)[16], int lane, double& s0, double& s1) {
  double a[8], b[4];
  swap_add_nd<true, 8>(x, x + 8, a);   // bit 5: topics [0, 8) | [8, 16)
  swap_add_nd<false, 4>(a, a + 4, b);  // bit 4: [0, 4) | [4, 8) of those
  const bool h3 = (lane & 8) != 0;     // bit 3: {0, 1} | {2, 3}
  s0 = rs_dpp_d<DPP_ROW_ROR8>(b[0], b[2], h3);
  s1 = rs_dpp_d<DPP_ROW_ROR8>(b[1], b[3], h3);
}

// fp64 wave64 all-reduce (sum) without LDS
__device__ __forceinline__ double wave_sum_d(double v) {
  {
    unsigned a = lo32(v), b = a, c = hi32(v), d = c;
    pswap_2<true>(a, b, c, d);
    v = mkd(a, c) + mkd(b, d);
  }
  {
    unsigned a = lo32(v), b = a, c = hi32(v), d = c;
    pswap_2<false>(a, b, c, d);
    v = mkd(a, c) + mkd(b, d);
  }
  v += dpp_d<DPP_ROW_MIRROR>(v);
  v += dpp_d<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_d<DPP_QP_1032>(v);
  v += dpp_d<DPP_QP_2301>(v);
  return v;
}

// Diagnostic build only (make stamp → libstc_stamp.so, tools/stamp_estep.py): s_memtime stamps at
// the phase boundaries of the inner loop, summed per phase over every wave of a launch.  The
// product library compiles STAMP(i) to nothing.
#ifdef STC_STAMP
constexpr int kStamps = 12;
// one copy per translation unit (no relocatable device code): each TU exports its own reader
static __device__ unsigned long long g_stamps[kStamps];
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP_DECL unsigned long long st_acc[::stc::lda::kStamps] = {}, st_last = ::stc::lda::stamp_now();
#define STAMP(i)                                         \
  do {                                                   \
    const unsigned long long t_ = ::stc::lda::stamp_now(); \
    st_acc[i] += t_ - st_last;                           \
    st_last = t_;                                        \
  } while (0)
#define STAMP_FLUSH                                                  \
  if ((threadIdx.x & 63) == 0)                                       \
    for (int i_ = 0; i_ < ::stc::lda::kStamps; ++i_) atomicAdd(&::stc::lda::g_stamps[i_], st_acc[i_]);
// diagnostic reader: copies (and optionally clears) this TU's per-phase cycle sums
#define STC_STAMP_READER(NAME)                                                                  \
  extern "C" int NAME(unsigned long long* out, int n, int reset) {                              \
    if (n > ::stc::lda::kStamps) n = ::stc::lda::kStamps;                                       \
    if (hipDeviceSynchronize() != hipSuccess) return 3;                                         \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(::stc::lda::g_stamps), n * sizeof(unsigned long long)) != hipSuccess) \
      return 3;                                                                                 \
    if (reset) {                                                                                \
      unsigned long long z[::stc::lda::kStamps] = {};                                           \
      if (hipMemcpyToSymbol(HIP_SYMBOL(::stc::lda::g_stamps), z, sizeof(z)) != hipSuccess) return 3; \
    }                                                                                           \
    return 0;                                                                                   \
  }
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH
#define STC_STAMP_READER(NAME)
#endif

}  // namespace lda
}  // namespace stc
