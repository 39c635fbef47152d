// psi64.h — the fp64 E-step's per-topic ψ/exp chain (lda_rows64.hip's ψ phase), in its own header so
// tools/ubench_f64.hip can time it and its alternatives in isolation.
#pragma once

#include "estep_common.h"

#ifndef PSI_V4_SERIES
#define PSI_V4_SERIES 0  // 1: v4 also holds Breeze's series coefficients in VGPRs (12 more VGPRs; measured 30.10 vs 29.97 ms headline, so off)
#endif

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
// Breeze's truncation term E(y) = f⁹·P(f), f = 1/y² (tools/fit_breeze_digamma.py)
__device__ __forceinline__ double trunc_f(double f) {
  double a = add_s(mul_s(f, -12318.55039822477), 2372.137971404805);
  a = fma_s(a, f, -260.94994774566294);
  a = fma_s(a, f, 26.284421368293753);
  a = fma_s(a, f, -3.053401198888146);
  const double f2 = f * f, f4 = f2 * f2;
  return ((f4 * f4) * f) * a;
}
__device__ __forceinline__ double exp_digamma_minus_s(double x, double cst) {
  const bool sh = x <= 5.0;
  const double xs = sh ? x : 1.0;
  // Σ_{i<6} 1/(xs+i) = p/q, q = xs(xs+1)…(xs+5)
  double q = fma_s(add_s(xs, 15.0), xs, 85.0);
  q = fma_s(q, xs, 225.0);
  q = fma_s(q, xs, 274.0);
  q = fma_s(q, xs, 120.0) * xs;
  double p = fma_s(add_s(mul_s(xs, 6.0), 75.0), xs, 340.0);
  p = fma_s(p, xs, 675.0);
  p = fma_s(p, xs, 548.0);
  p = fma_s(p, xs, 120.0);
  const double iq = rcp_nr(q);
  double c = p * iq;
  c = fma(fma(-q, c, p), iq, c);
  const double y = sh ? add_s(x, 6.0) : x;
  const double iy = rcp_nr(y);
  const double f = iy * iy;
  double t = add_s(mul_s(f, 3617.0 / 8160.0), -1.0 / 12.0);
  t = fma_s(t, f, 691.0 / 32760.0);
  t = fma_s(t, f, -1.0 / 132.0);
  t = fma_s(t, f, 1.0 / 240.0);
  t = fma_s(t, f, -1.0 / 252.0);
  t = fma_s(t, f, 1.0 / 120.0);
  t = fma_s(t, f, -1.0 / 12.0) * f;
  const double yb = xs + (floor(sub_s(5.0, xs)) + 1.0);  // Breeze's y ∈ (5, 6] (E needs ~1e-4 relative)
  const double rb = __builtin_amdgcn_rcp(yb);
  const double fix = trunc_f(f) - trunc_f(rb * rb);
  const double shift = sh ? fix - c : 0.0;
  const double z = ((shift - 0.5 * iy) + t) - cst;
  // exp(z): n = rint(z / ln2), r = z − n·ln2 (hi/lo), e^r = E(r²) + r·O(r²)
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

// ---- the same chain with its constants read from a 16-B aligned LDS table (v3): the instruction stream
// of exp_digamma_minus_v2 — same operations, same order, same roundings, so the result is bit-identical
// — but every non-inline constant is a VGPR operand loaded by ds_read_b128 (two constants per read)
// instead of an SGPR pair built by two s_mov_b32 per evaluation (the compiler rematerialises them each
// time: ≈ 50 scalar moves per chain, each taking the wave's issue slot).
__device__ __forceinline__ double fma_v(double a, double b, double c) {  // a·b + c, no contraction choices
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ double mul_v(double a, double b) {
  double d;
  asm("v_mul_f64 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ double add_v(double a, double b) {
  double d;
  asm("v_add_f64 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ double sub_v(double b, double a) {  // b − a
  double d;
  asm("v_add_f64 %0, -%1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// table slots (doubles; the packed-fp32 pairs of the truncation fix are one slot each)
enum PsiKSlot {
  PK_5, PK_3, PK_20, PK_24, PK_10, PK_6,
  PK_S0, PK_S1, PK_S2, PK_S3, PK_S4, PK_S5, PK_S6,  // 3617/8160, −1/12, 691/32760, −1/132, 1/240, −1/252, 1/120
  PK_LOG2E, PK_LN2HI, PK_LN2LO,
  PK_E0, PK_E1, PK_E2, PK_E3, PK_E4,                 // 1/12!, 1/10!, 1/8!, 1/6!, 1/4!
  PK_O0, PK_O1, PK_O2, PK_O3, PK_O4,                 // 1/13!, 1/11!, 1/9!, 1/7!, 1/6 (1/5! is PK_S6)
  PK_NMIN,                                           // −1100
  PK_T0, PK_T1, PK_T2, PK_T3, PK_T4,                 // the truncation fix's fp32 coefficients, splatted pairs
  PK_N
};
struct alignas(16) PsiK {
  double k[(PK_N + 1) / 2 * 2];
};
// fill the table (any threads of the block, then a barrier before the first use)
__device__ __forceinline__ void psik_fill(PsiK& t, int tid, int nthr) {
  const double v[PK_N - 5] = {5.0, 3.0, 20.0, 24.0, 10.0, 6.0,
                              3617.0 / 8160.0, -1.0 / 12.0, 691.0 / 32760.0, -1.0 / 132.0, 1.0 / 240.0, -1.0 / 252.0,
                              1.0 / 120.0,
                              1.4426950408889634, -6.93147180369123816490e-01, -1.90821492927058770002e-10,
                              1.0 / 479001600.0, 1.0 / 3628800.0, 1.0 / 40320.0, 1.0 / 720.0, 1.0 / 24.0,
                              1.0 / 6227020800.0, 1.0 / 39916800.0, 1.0 / 362880.0, 1.0 / 5040.0, 1.0 / 6.0,
                              -1100.0};
  const float f[5] = {-12318.55039822477f, 2372.137971404805f, -260.94994774566294f, 26.284421368293753f,
                      -3.053401198888146f};
  for (int i = tid; i < PK_N; i += nthr) {
    if (i < PK_T0) {
      t.k[i] = v[i];
    } else {
      const pkf2 p = {f[i - PK_T0], f[i - PK_T0]};
      t.k[i] = __builtin_bit_cast(double, p);
    }
  }
}
__device__ __forceinline__ double trunc_fix_pk_t(double f6, double xs, const double* K) {
  const double nb = floor(sub_v(K[PK_5], xs)) + 1.0;  // Breeze's shift count (exact)
  const float rb = __builtin_amdgcn_rcpf((float)xs + (float)nb);
  const pkf2 u = {(float)f6, rb * rb};
  const pkf2 c0 = __builtin_bit_cast(pkf2, K[PK_T0]), c1 = __builtin_bit_cast(pkf2, K[PK_T1]),
             c2 = __builtin_bit_cast(pkf2, K[PK_T2]), c3 = __builtin_bit_cast(pkf2, K[PK_T3]),
             c4 = __builtin_bit_cast(pkf2, K[PK_T4]);
  pkf2 a = u * c0 + c1;
  a = a * u + c2;
  a = a * u + c3;
  a = a * u + c4;
  const pkf2 u2 = u * u, u4 = u2 * u2, u8 = u4 * u4;
  const pkf2 e = (u8 * u) * a;
  return (double)(e.x - e.y);
}
template <int RCP_STEPS>
__device__ __forceinline__ double exp_digamma_minus_v3(double x, double cst, const PsiK& T) {
  const double* K = T.k;
  const bool sh = x <= 5.0;
  const double xs = sh ? x : 1.0;
  const double u = xs * add_v(xs, K[PK_5]);
  const double num = fma_v(add_v(mul_v(u, K[PK_3]), K[PK_20]), u, K[PK_24]) * fma(xs, 2.0, 5.0);
  const double den = u * fma_v(add_v(u, K[PK_10]), u, K[PK_24]);
  const double iq = rcp_n<RCP_STEPS>(den);
  double c = num * iq;
  c = fma(fma(-den, c, num), iq, c);
  const double y = sh ? add_v(x, K[PK_6]) : x;
  const double iy = rcp_n<RCP_STEPS>(y);
  const double f = iy * iy;
  double t = add_v(mul_v(f, K[PK_S0]), K[PK_S1]);
  t = fma_v(t, f, K[PK_S2]);
  t = fma_v(t, f, K[PK_S3]);
  t = fma_v(t, f, K[PK_S4]);
  t = fma_v(t, f, K[PK_S5]);
  t = fma_v(t, f, K[PK_S6]);
  t = fma_v(t, f, K[PK_S1]) * f;
  const double shift = sh ? trunc_fix_pk_t(f, xs, K) - c : 0.0;
  const double z = (fma(-0.5, iy, shift) + t) - cst;
  const double n = __builtin_rint(mul_v(z, K[PK_LOG2E]));
  double r = fma_v(n, K[PK_LN2HI], z);
  r = fma_v(n, K[PK_LN2LO], r);
  const double r2 = r * r;
  double e = add_v(mul_v(r2, K[PK_E0]), K[PK_E1]);
  e = fma_v(e, r2, K[PK_E2]);
  e = fma_v(e, r2, K[PK_E3]);
  e = fma_v(e, r2, K[PK_E4]);
  e = fma(e, r2, 0.5);
  e = fma(e, r2, 1.0);
  double o = add_v(mul_v(r2, K[PK_O0]), K[PK_O1]);
  o = fma_v(o, r2, K[PK_O2]);
  o = fma_v(o, r2, K[PK_O3]);
  o = fma_v(o, r2, K[PK_S6]);
  o = fma_v(o, r2, K[PK_O4]);
  o = fma(o, r2, 1.0);
  const double ez = __builtin_ldexp(fma(r, o, e), (int)fmax(n, K[PK_NMIN]));  // n < -1100: 0
  return y * ez;
}

// ---- v4: the v2 chain with the exp() constants held in VGPRs across the caller's loop (PsiExpK, loaded
// once per document from the LDS table and laundered so the compiler cannot rematerialise them): 28
// VGPRs for 28 fewer s_mov_b32 per evaluation; the digamma part keeps its SGPR operands.  Bit-identical
// to v2 (same instructions, operands from VGPRs).
struct PsiExpK {
  double log2e, ln2hi, ln2lo, e0, e1, e2, e3, e4, o0, o1, o2, o3, o5, o4;  // o5 = 1/5!
#if PSI_V4_SERIES
  double s0, s1, s2, s3, s4, s5;  // Breeze's series: 3617/8160, −1/12, 691/32760, −1/132, 1/240, −1/252 (1/120 = o5)
#endif
};
__device__ __forceinline__ PsiExpK psi_expk_load(const PsiK& T) {
  const double* K = T.k;
  PsiExpK c{K[PK_LOG2E], K[PK_LN2HI], K[PK_LN2LO], K[PK_E0], K[PK_E1], K[PK_E2], K[PK_E3], K[PK_E4],
            K[PK_O0],    K[PK_O1],    K[PK_O2],    K[PK_O3], K[PK_S6], K[PK_O4]};
  asm volatile("" : "+v"(c.log2e), "+v"(c.ln2hi), "+v"(c.ln2lo), "+v"(c.e0), "+v"(c.e1), "+v"(c.e2), "+v"(c.e3));
  asm volatile("" : "+v"(c.e4), "+v"(c.o0), "+v"(c.o1), "+v"(c.o2), "+v"(c.o3), "+v"(c.o5), "+v"(c.o4));
#if PSI_V4_SERIES
  c.s0 = K[PK_S0];
  c.s1 = K[PK_S1];
  c.s2 = K[PK_S2];
  c.s3 = K[PK_S3];
  c.s4 = K[PK_S4];
  c.s5 = K[PK_S5];
  asm volatile("" : "+v"(c.s0), "+v"(c.s1), "+v"(c.s2), "+v"(c.s3), "+v"(c.s4), "+v"(c.s5));
#endif
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
#if PSI_V4_SERIES
__device__ __forceinline__ double series_vk(double f, const PsiExpK& C) {
#pragma clang fp contract(off)
  double t = f * C.s0 + C.s1;
  t = __builtin_fma(t, f, C.s2);
  t = __builtin_fma(t, f, C.s3);
  t = __builtin_fma(t, f, C.s4);
  t = __builtin_fma(t, f, C.s5);
  t = __builtin_fma(t, f, C.o5);
  return __builtin_fma(t, f, C.s1) * f;
}
#endif
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
#if PSI_V4_SERIES
  const double t = series_vk(f, C);
#else
  double t = add_s(mul_s(f, 3617.0 / 8160.0), -1.0 / 12.0);
  t = fma_s(t, f, 691.0 / 32760.0);
  t = fma_s(t, f, -1.0 / 132.0);
  t = fma_s(t, f, 1.0 / 240.0);
  t = fma_s(t, f, -1.0 / 252.0);
  t = fma_s(t, f, 1.0 / 120.0);
  t = fma_s(t, f, -1.0 / 12.0) * f;
#endif
  const double shift = sh ? trunc_fix_pk(f, xs) - c : 0.0;
  const double z = (fma(-0.5, iy, shift) + t) - cst;
  return y * exp_vk(z, C);
}

}  // namespace psi64
using psi64::exp_digamma_minus_s;
using psi64::exp_digamma_minus_v2;
using psi64::exp_digamma_minus_v3;
using psi64::PsiK;
using psi64::psik_fill;
using psi64::PsiExpK;
using psi64::psi_expk_load;
using psi64::exp_digamma_minus_v4;
}  // namespace lda
}  // namespace stc
