// psi64.h — the fp64 E-step's per-topic ψ/exp chain (the ψ phases of lda_rows64.hip, lda_team64.hip and
// lda_wide.hip), in its own header so tools/ubench_f64.hip can time it in isolation.  The forms measured
// and rejected in rounds 3–5 (the round-3 Horner chain, the LDS-table v3, v4 with the series in VGPRs)
// are gone from the source; their numbers are in DESIGN.md §3.
#pragma once

#include "estep_common.h"

namespace stc {
namespace lda {
namespace psi64 {

// ---- the per-topic ψ/exp chain of the ψ phase, shaped for VALU count: every polynomial in Horner
// form with its coefficient as the instruction's SGPR operand (a GFX9 VOP3 takes one constant-bus
// operand), so no constant costs a v_mov pair; branch-free (the shift part is computed for every lane
// and selected), so the compiler cannot sink it into a divergent branch.  Same Breeze series and
// truncation fix as stc_internal.h exp_digamma_minus_d; exp() is Cody–Waite + a degree-13 Taylor
// polynomial in even/odd halves (truncation 4e-18 relative).
__device__ __forceinline__ double fma_s(double a, double b, double c) {  // a·b + c, c in an SGPR pair
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
}
__device__ __forceinline__ double fma_sb(double a, double b, double c) {  // a·b + c, b in an SGPR pair
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
  return d;
}
__device__ __forceinline__ double mul_s(double a, double b) {
  double d;
  asm("v_mul_f64 %0, %1, %2" : "=v"(d) : "v"(a), "s"(b));
  return d;
}
__device__ __forceinline__ double add_s(double a, double b) {
  double d;
  asm("v_add_f64 %0, %1, %2" : "=v"(d) : "v"(a), "s"(b));
  return d;
}
__device__ __forceinline__ double sub_s(double b, double a) {  // b − a, b in an SGPR pair
  double d;
  asm("v_add_f64 %0, -%1, %2" : "=v"(d) : "v"(a), "s"(b));
  return d;
}
// ---- round-4 form (exp_digamma_minus_v2): the same Breeze ψ and exp, fewer fp64 instructions.
//  * Breeze's truncation fix E(x + 6) − E(y_B) (≤ 8e-13, needs ~1e-5 relative) in ONE packed-fp32
//    stream for both arguments (v_pk_fma_f32 / v_pk_mul_f32): 1.1e-18 absolute against the fp64 form;
//    Breeze's shift count ⌊5 − x⌋ + 1 stays fp64 (exact), only y_B's value is rounded to fp32.
//  * the six recurrence terms as (2x+5)·(3u² + 20u + 24) / (u(u+4)(u+6)), u = x(x+5): the pairs
//    1/(x+i) + 1/(x+5−i) share the numerator 2x+5 (two instructions and one level shorter than p/q).
//  * RCP_STEPS Newton steps after v_rcp_f64 (tools/ubench_f64 measures the raw reciprocal's error).
typedef float pkf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double trunc_fix_pk(double f6, double xs) {
  const double nb = floor(sub_s(5.0, xs)) + 1.0;  // Breeze's shift count (exact)
  const float rb = __builtin_amdgcn_rcpf((float)xs + (float)nb);
  const pkf2 u = {(float)f6, rb * rb};
  pkf2 a = u * (pkf2)(-12318.55039822477f) + (pkf2)(2372.137971404805f);
  a = a * u + (pkf2)(-260.94994774566294f);
  a = a * u + (pkf2)(26.284421368293753f);
  a = a * u + (pkf2)(-3.053401198888146f);
  const pkf2 u2 = u * u, u4 = u2 * u2, u8 = u4 * u4;
  const pkf2 e = (u8 * u) * a;
  return (double)(e.x - e.y);
}
template <int RCP_STEPS>
__device__ __forceinline__ double rcp_n(double q) {
  double r = __builtin_amdgcn_rcp(q);
#pragma unroll
  for (int i = 0; i < RCP_STEPS; ++i) r = fma(r, fma(-q, r, 1.0), r);
  return r;
}
template <int RCP_STEPS>
__device__ __forceinline__ double exp_digamma_minus_v2(double x, double cst) {
  const bool sh = x <= 5.0;
  const double xs = sh ? x : 1.0;
  // Σ_{i<6} 1/(xs+i) = num/den
  const double u = xs * add_s(xs, 5.0);
  const double num = fma_s(add_s(mul_s(u, 3.0), 20.0), u, 24.0) * fma(xs, 2.0, 5.0);
  const double den = u * fma_s(add_s(u, 10.0), u, 24.0);
  const double iq = rcp_n<RCP_STEPS>(den);
  double c = num * iq;
  c = fma(fma(-den, c, num), iq, c);
  const double y = sh ? add_s(x, 6.0) : x;
  const double iy = rcp_n<RCP_STEPS>(y);
  const double f = iy * iy;
  double t = add_s(mul_s(f, 3617.0 / 8160.0), -1.0 / 12.0);
  t = fma_s(t, f, 691.0 / 32760.0);
  t = fma_s(t, f, -1.0 / 132.0);
  t = fma_s(t, f, 1.0 / 240.0);
  t = fma_s(t, f, -1.0 / 252.0);
  t = fma_s(t, f, 1.0 / 120.0);
  t = fma_s(t, f, -1.0 / 12.0) * f;
  const double shift = sh ? trunc_fix_pk(f, xs) - c : 0.0;
  const double z = (fma(-0.5, iy, shift) + t) - cst;
  const double n = __builtin_rint(mul_s(z, 1.4426950408889634));
  double r = fma_sb(n, -6.93147180369123816490e-01, z);
  r = fma_sb(n, -1.90821492927058770002e-10, r);
  const double r2 = r * r;
  double e = add_s(mul_s(r2, 1.0 / 479001600.0), 1.0 / 3628800.0);
  e = fma_s(e, r2, 1.0 / 40320.0);
  e = fma_s(e, r2, 1.0 / 720.0);
  e = fma_s(e, r2, 1.0 / 24.0);
  e = fma(e, r2, 0.5);
  e = fma(e, r2, 1.0);
  double o = add_s(mul_s(r2, 1.0 / 6227020800.0), 1.0 / 39916800.0);
  o = fma_s(o, r2, 1.0 / 362880.0);
  o = fma_s(o, r2, 1.0 / 5040.0);
  o = fma_s(o, r2, 1.0 / 120.0);
  o = fma_s(o, r2, 1.0 / 6.0);
  o = fma(o, r2, 1.0);
  const double ez = __builtin_ldexp(fma(r, o, e), (int)fmax(n, -1100.0));  // n < -1100: 0
  return y * ez;
}

// the exp() constants of the v4 chain, filled into an LDS table once per document (then read into VGPRs)
enum PsiKSlot {
  PK_LOG2E, PK_LN2HI, PK_LN2LO,
  PK_E0, PK_E1, PK_E2, PK_E3, PK_E4,  // 1/12!, 1/10!, 1/8!, 1/6!, 1/4!
  PK_O0, PK_O1, PK_O2, PK_O3, PK_O5,  // 1/13!, 1/11!, 1/9!, 1/7!, 1/5!
  PK_O4,                              // 1/6 (1/3!)
  PK_N
};
struct alignas(16) PsiK {
  double k[(PK_N + 1) / 2 * 2];
};
// fill the table (any threads of the block, then a barrier before the first use)
__device__ __forceinline__ void psik_fill(PsiK& t, int tid, int nthr) {
  const double v[PK_N] = {1.4426950408889634, -6.93147180369123816490e-01, -1.90821492927058770002e-10,
                          1.0 / 479001600.0, 1.0 / 3628800.0, 1.0 / 40320.0, 1.0 / 720.0, 1.0 / 24.0,
                          1.0 / 6227020800.0, 1.0 / 39916800.0, 1.0 / 362880.0, 1.0 / 5040.0, 1.0 / 120.0,
                          1.0 / 6.0};
  for (int i = tid; i < PK_N; i += nthr) t.k[i] = v[i];
}
// ---- v4: the v2 chain with the exp() constants held in VGPRs across the caller's loop (PsiExpK, loaded
// once per document from the LDS table and laundered so the compiler cannot rematerialise them): 28
// VGPRs for 28 fewer s_mov_b32 per evaluation; the digamma part keeps its SGPR operands.  Bit-identical
// to v2 (same instructions, operands from VGPRs).
struct PsiExpK {
  double log2e, ln2hi, ln2lo, e0, e1, e2, e3, e4, o0, o1, o2, o3, o5, o4;  // o5 = 1/5!
};
__device__ __forceinline__ PsiExpK psi_expk_load(const PsiK& T) {
  const double* K = T.k;
  PsiExpK c{K[PK_LOG2E], K[PK_LN2HI], K[PK_LN2LO], K[PK_E0], K[PK_E1], K[PK_E2], K[PK_E3], K[PK_E4],
            K[PK_O0],    K[PK_O1],    K[PK_O2],    K[PK_O3], K[PK_O5], K[PK_O4]};
  asm volatile("" : "+v"(c.log2e), "+v"(c.ln2hi), "+v"(c.ln2lo), "+v"(c.e0), "+v"(c.e1), "+v"(c.e2), "+v"(c.e3));
  asm volatile("" : "+v"(c.e4), "+v"(c.o0), "+v"(c.o1), "+v"(c.o2), "+v"(c.o3), "+v"(c.o5), "+v"(c.o4));
  return c;
}
__device__ __forceinline__ double exp_vk(double z, const PsiExpK& C) {
#pragma clang fp contract(off)
  const double n = __builtin_rint(z * C.log2e);
  double r = __builtin_fma(n, C.ln2hi, z);
  r = __builtin_fma(n, C.ln2lo, r);
  const double r2 = r * r;
  double e = r2 * C.e0 + C.e1;
  e = __builtin_fma(e, r2, C.e2);
  e = __builtin_fma(e, r2, C.e3);
  e = __builtin_fma(e, r2, C.e4);
  e = __builtin_fma(e, r2, 0.5);
  e = __builtin_fma(e, r2, 1.0);
  double o = r2 * C.o0 + C.o1;
  o = __builtin_fma(o, r2, C.o2);
  o = __builtin_fma(o, r2, C.o3);
  o = __builtin_fma(o, r2, C.o5);
  o = __builtin_fma(o, r2, C.o4);
  o = __builtin_fma(o, r2, 1.0);
  return __builtin_ldexp(__builtin_fma(r, o, e), (int)fmax(n, -1100.0));  // n < -1100: 0
}
template <int RCP_STEPS>
__device__ __forceinline__ double exp_digamma_minus_v4(double x, double cst, const PsiExpK& C) {
  const bool sh = x <= 5.0;
  const double xs = sh ? x : 1.0;
  const double u = xs * add_s(xs, 5.0);
  const double num = fma_s(add_s(mul_s(u, 3.0), 20.0), u, 24.0) * fma(xs, 2.0, 5.0);
  const double den = u * fma_s(add_s(u, 10.0), u, 24.0);
  const double iq = rcp_n<RCP_STEPS>(den);
  double c = num * iq;
  c = fma(fma(-den, c, num), iq, c);
  const double y = sh ? add_s(x, 6.0) : x;
  const double iy = rcp_n<RCP_STEPS>(y);
  const double f = iy * iy;
  double t = add_s(mul_s(f, 3617.0 / 8160.0), -1.0 / 12.0);
  t = fma_s(t, f, 691.0 / 32760.0);
  t = fma_s(t, f, -1.0 / 132.0);
  t = fma_s(t, f, 1.0 / 240.0);
  t = fma_s(t, f, -1.0 / 252.0);
  t = fma_s(t, f, 1.0 / 120.0);
  t = fma_s(t, f, -1.0 / 12.0) * f;
  const double shift = sh ? trunc_fix_pk(f, xs) - c : 0.0;
  const double z = (fma(-0.5, iy, shift) + t) - cst;
  return y * exp_vk(z, C);
}

}  // namespace psi64
using psi64::exp_digamma_minus_v2;
using psi64::PsiK;
using psi64::psik_fill;
using psi64::PsiExpK;
using psi64::psi_expk_load;
using psi64::exp_digamma_minus_v4;
}  // namespace lda
}  // namespace stc
