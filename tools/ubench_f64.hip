// ubench_f64.hip — latency / issue microbenchmarks for the fp64 E-step's building blocks on gfx950
// (MI355X): dependent and independent v_fma_f64, v_rcp_f64, the ψ/exp chain of the ψ phase
// (psi64.h exp_digamma_minus_v2, one and two Newton steps), a dependent ds_read_b128, the
// fp64 wave reduction, and a 4-wave s_barrier — each with 1, 2 and 3 waves per SIMD (one workgroup
// of 4·W waves on one CU).  Prints one JSON line per case: cycles per operation per wave (s_memtime
// around the loop, max over the waves).  Build: make -C tools ubench (hipcc, gfx950).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "psi64.h"

using namespace stc;
using namespace stc::lda;

constexpr int kN = 256;  // operations per timed loop

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

enum Op { FMA_DEP, FMA_IND8, RCP_DEP, LDS_DEP, WSUM, BARRIER, RCPNR_DEP, PSI_V2_2, PSI_V2_1,
          PKFMA_IND8, FMA_BANK_SAME, FMA_BANK_SPLIT, FMA_SHARED_E };

template <int OP>
__global__ void k_bench(double* out, unsigned long long* cyc, double a, double b) {
  __shared__ double lds[4096];
  const int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += blockDim.x) lds[i] = 0.0;
  __syncthreads();
  double x = 1.0 + 1e-3 * (tid & 63), y = 2.0 + 1e-3 * (tid & 31);
  double acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = x + j;
  int idx = (tid & 63) * 2;
  unsigned long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms the instruction cache
    __syncthreads();
    t0 = now();
    if (OP == FMA_DEP) {
#pragma unroll 16
      for (int i = 0; i < kN; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    } else if (OP == FMA_IND8) {
#pragma unroll 4
      for (int i = 0; i < kN / 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[j]) : "v"(a), "v"(b));
    } else if (OP == RCP_DEP) {
#pragma unroll 16
      for (int i = 0; i < kN; ++i) asm volatile("v_rcp_f64 %0, %0" : "+v"(x));
    } else if (OP == RCPNR_DEP) {
#pragma unroll 8
      for (int i = 0; i < kN; ++i) {
        x = rcp_nr(x);
        asm volatile("" : "+v"(x));
      }
    } else if (OP == PSI_V2_2 || OP == PSI_V2_1) {
#pragma unroll 2
      for (int i = 0; i < kN / 16; ++i) {
        x = fma(OP == PSI_V2_2 ? exp_digamma_minus_v2<2>(x, a) : exp_digamma_minus_v2<1>(x, a), 0.25, b);
        asm volatile("" : "+v"(x));
      }
    } else if (OP == PKFMA_IND8) {
      typedef float f2_t __attribute__((ext_vector_type(2)));
      f2_t p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) p[j] = (f2_t){(float)acc[j], (float)(acc[j] + 1.0)};
      const f2_t fa = {(float)a, (float)a}, fb = {(float)b, (float)b};
#pragma unroll 4
      for (int i = 0; i < kN / 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[j]) : "v"(fa), "v"(fb));
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = p[j].x + p[j].y;
    } else if (OP == FMA_BANK_SAME || OP == FMA_BANK_SPLIT || OP == FMA_SHARED_E) {
      // register-bank patterns of the E-step's v_fmac_f64 acc, B, e: explicit VGPRs (v64+ is free here)
      // SAME: acc, B, e all start on a bank ≡ 0 (mod 4); SPLIT: acc ≡ 0, B ≡ 2, e ≡ 0 (B on the other
      // bank pair); SHARED_E: the kernel's shape — 8 accumulators, 8 B, one e for all
#pragma unroll 4
      for (int i = 0; i < kN / 8; ++i) {
        if (OP == FMA_BANK_SAME)
          asm volatile(
              "v_fmac_f64 v[64:65], v[96:97], v[128:129]\n v_fmac_f64 v[68:69], v[100:101], v[132:133]\n"
              "v_fmac_f64 v[72:73], v[104:105], v[136:137]\n v_fmac_f64 v[76:77], v[108:109], v[140:141]\n"
              "v_fmac_f64 v[80:81], v[112:113], v[144:145]\n v_fmac_f64 v[84:85], v[116:117], v[148:149]\n"
              "v_fmac_f64 v[88:89], v[120:121], v[152:153]\n v_fmac_f64 v[92:93], v[124:125], v[156:157]" ::
                  : "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159");
        else if (OP == FMA_BANK_SPLIT)
          asm volatile(
              "v_fmac_f64 v[64:65], v[98:99], v[128:129]\n v_fmac_f64 v[68:69], v[102:103], v[132:133]\n"
              "v_fmac_f64 v[72:73], v[106:107], v[136:137]\n v_fmac_f64 v[76:77], v[110:111], v[140:141]\n"
              "v_fmac_f64 v[80:81], v[114:115], v[144:145]\n v_fmac_f64 v[84:85], v[118:119], v[148:149]\n"
              "v_fmac_f64 v[88:89], v[122:123], v[152:153]\n v_fmac_f64 v[92:93], v[126:127], v[156:157]" ::
                  : "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159");
        else
          asm volatile(
              "v_fmac_f64 v[64:65], v[98:99], v[128:129]\n v_fmac_f64 v[68:69], v[102:103], v[128:129]\n"
              "v_fmac_f64 v[72:73], v[106:107], v[128:129]\n v_fmac_f64 v[76:77], v[110:111], v[128:129]\n"
              "v_fmac_f64 v[80:81], v[114:115], v[128:129]\n v_fmac_f64 v[84:85], v[118:119], v[128:129]\n"
              "v_fmac_f64 v[88:89], v[122:123], v[128:129]\n v_fmac_f64 v[92:93], v[126:127], v[128:129]" ::
                  : "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159");
      }
    } else if (OP == LDS_DEP) {
#pragma unroll 8
      for (int i = 0; i < kN; ++i) {
        const double2 v = *reinterpret_cast<const double2*>(&lds[idx]);
        idx = (idx + 2 + (int)v.x) & 4095 & ~1;
      }
      x += idx;
    } else if (OP == WSUM) {
#pragma unroll 4
      for (int i = 0; i < kN / 8; ++i) {
        x = wave_sum_d(x) * 1e-2;
        asm volatile("" : "+v"(x));
      }
    } else if (OP == BARRIER) {
#pragma unroll 8
      for (int i = 0; i < kN; ++i) __syncthreads();
    }
    t1 = now();
  }
  double s = x + y;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + tid] = s;
  if ((tid & 63) == 0) cyc[blockIdx.x * 64 + (tid >> 6)] = t1 - t0;
}

// operations per timed loop, for the per-op figure
static int ops(int op) {
  switch (op) {
    case PSI_V2_2: case PSI_V2_1: return kN / 16;
    case WSUM: return kN / 8;
    default: return kN;
  }
}

template <int OP>
static void run(const char* name, int waves_per_simd, double* d_out, unsigned long long* d_cyc) {
  const int threads = 64 * 4 * waves_per_simd;
  hipLaunchKernelGGL(k_bench<OP>, dim3(1), dim3(threads), 0, 0, d_out, d_cyc, 0.999, 1e-3);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("{\"case\": \"%s\", \"error\": \"launch failed\"}\n", name);
    std::exit(1);
  }
  std::vector<unsigned long long> c(64);
  (void)hipMemcpy(c.data(), d_cyc, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (int w = 0; w < threads / 64; ++w) mx = c[w] > mx ? c[w] : mx;
  std::printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_op\": %.2f}\n", name, waves_per_simd,
              (double)mx / ops(OP));
}

// accuracy of the raw v_rcp_f64 and of one / two Newton steps: max |r·q − 1| in units of 2^-52 over
// q = 2^e · m, e ∈ [-20, 40), m ∈ [1, 2) on a fine grid
__global__ void k_rcp_err(double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const double q = ldexp(1.0 + (double)(i & 0xFFFFF) * 0x1p-20 + 0x1p-45 * (i >> 20), (i >> 20) - 20);
  const double r0 = __builtin_amdgcn_rcp(q);
  const double r1 = fma(r0, fma(-q, r0, 1.0), r0);
  const double r2 = fma(r1, fma(-q, r1, 1.0), r1);
  const double e0 = fabs(fma(r0, q, -1.0)) * 0x1p52, e1 = fabs(fma(r1, q, -1.0)) * 0x1p52,
               e2 = fabs(fma(r2, q, -1.0)) * 0x1p52;
  out[3 * i] = e0;
  out[3 * i + 1] = e1;
  out[3 * i + 2] = e2;
}

int main() {
  double* d_out = nullptr;
  unsigned long long* d_cyc = nullptr;
  if (hipMalloc(&d_out, 4096 * sizeof(double)) != hipSuccess || hipMalloc(&d_cyc, 64 * 8) != hipSuccess) {
    std::printf("{\"error\": \"hipMalloc\"}\n");
    return 1;
  }
  {
    const int n = 60 << 20;
    double* d_e = nullptr;
    if (hipMalloc(&d_e, sizeof(double) * 3 * (size_t)n) == hipSuccess) {
      hipLaunchKernelGGL(k_rcp_err, dim3(n / 256), dim3(256), 0, 0, d_e);
      std::vector<double> e(3 * (size_t)n);
      (void)hipMemcpy(e.data(), d_e, sizeof(double) * e.size(), hipMemcpyDeviceToHost);
      double m[3] = {0, 0, 0};
      for (size_t i = 0; i < e.size(); ++i) m[i % 3] = e[i] > m[i % 3] ? e[i] : m[i % 3];
      std::printf("{\"case\": \"rcp_f64_error_ulp52\", \"raw\": %.4g, \"newton1\": %.4g, \"newton2\": %.4g}\n",
                  m[0], m[1], m[2]);
      (void)hipFree(d_e);
    }
  }
  for (int w = 1; w <= 3; ++w) {
    run<FMA_DEP>("fma_f64_dependent", w, d_out, d_cyc);
    run<FMA_IND8>("fma_f64_8_independent", w, d_out, d_cyc);
    run<RCP_DEP>("rcp_f64_dependent", w, d_out, d_cyc);
    run<RCPNR_DEP>("rcp_nr_dependent", w, d_out, d_cyc);
    run<PSI_V2_2>("exp_digamma_minus_v2_nr2_dependent", w, d_out, d_cyc);
    run<PSI_V2_1>("exp_digamma_minus_v2_nr1_dependent", w, d_out, d_cyc);
    run<PKFMA_IND8>("pk_fma_f32_8_independent", w, d_out, d_cyc);
    run<FMA_BANK_SAME>("fmac_f64_banks_same", w, d_out, d_cyc);
    run<FMA_BANK_SPLIT>("fmac_f64_banks_split", w, d_out, d_cyc);
    run<FMA_SHARED_E>("fmac_f64_shared_e", w, d_out, d_cyc);
    run<LDS_DEP>("ds_read_b128_dependent", w, d_out, d_cyc);
    run<WSUM>("wave_sum_d_dependent", w, d_out, d_cyc);
    run<BARRIER>("s_barrier", w, d_out, d_cyc);
  }
  (void)hipFree(d_out);
  (void)hipFree(d_cyc);
  return 0;
}
