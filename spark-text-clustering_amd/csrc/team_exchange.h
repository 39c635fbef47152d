// team_exchange.h — the inter-workgroup exchange of the team E-step kernels (lda_wide.hip
// k_estep_wide_mc / _tc, lda_team64.hip k_estep_tgrid64): a team of workgroups on one XCD trades values
// through 16-byte {epoch, value} granules in global memory (MI355X_MICROARCH.md inter-workgroup
// visibility; cdna_hip_programming.md Guideline 16, R2: the data is the flag), with every spin bounded.
#pragma once

#include "estep_common.h"

namespace stc {
namespace lda {
namespace team {

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;  // buffer aux bit: sc1 (write-through store / L1-bypassing load)
#ifndef WIDE_GRANULE_STORE_AUX
// the granule stores' cache policy: plain (0) keeps the line in the XCD's L2, where the team's other
// members (same blockIdx % 8, so the same XCD) poll it; sc1 (write-through) drops it and every poll
// then goes to the MALL.  Config 4 fp64 E-step 324 → 307 ms (r04).  A member on another XCD would read
// its own L2's stale line: tags never match, the bounded spin times out, the one-CU rerun keeps the result.
#define WIDE_GRANULE_STORE_AUX 0
#endif

template <typename T>
__device__ __forceinline__ void put_granule(__amdgpu_buffer_rsrc_t rs, int idx, unsigned epoch, T v) {
  unsigned long long bits;
  if constexpr (sizeof(T) == 8) bits = __builtin_bit_cast(unsigned long long, v);
  else bits = __builtin_bit_cast(unsigned int, v);
  // the epoch in both 8-byte halves: a reader takes the granule only when both tags match, so a
  // store whose halves become visible at different times is re-polled, never consumed torn (the
  // memory model guarantees single-copy atomicity up to 64 bits only)
  const u32x4 g = {epoch, (unsigned)bits, epoch, (unsigned)(bits >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(g, rs, idx * 16, 0, WIDE_GRANULE_STORE_AUX);
}
template <typename T>
__device__ __forceinline__ bool get_granule(__amdgpu_buffer_rsrc_t rs, int idx, unsigned epoch, T& v) {
  const u32x4 g = __builtin_amdgcn_raw_buffer_load_b128(rs, idx * 16, 0, kSc1);
  const unsigned long long bits = ((unsigned long long)g.w << 32) | g.y;
  if constexpr (sizeof(T) == 8) v = __builtin_bit_cast(T, bits);
  else v = __builtin_bit_cast(T, (unsigned)bits);
  return g.x == epoch && g.z == epoch;
}
__device__ __forceinline__ bool spin_give_up(unsigned spins, unsigned* tmo, unsigned limit) {
  // the team's timeout word is read every 32nd poll only (one request fewer per poll round)
  if (spins < limit && ((spins & 31u) != 31u ||
                        __hip_atomic_load((gu32*)tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u))
    return false;
  __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}


}  // namespace team
using team::get_granule;
using team::put_granule;
using team::spin_give_up;
}  // namespace lda
}  // namespace stc
