// idf.hip — K3 (document frequency), K4 (idf finalise), K5 (TF·IDF transform) for gfx950.
//
// Replaces [U] mllib.feature.IDF.fit (DocumentFrequencyAggregator.add/merge/idf) and
// IDFModel.transform, reached from LDAClustering.scala:177 (`new IDF(2).fit(tf).idf`) and
// :180-192 (tf × idf with the idf==0 → 1e-4 floor).
//
// df is a column histogram of a Zipf-skewed CSR: the hottest term sits in nearly every row, so
// per-entry global atomics would serialise on a handful of addresses.  k_df_hist pre-aggregates
// each workgroup's slice in LDS (see there); bytes: the CSR's indices + values read once.
#include "stc_internal.h"

namespace stc {
namespace idf {

static int grid_for(int64_t n) {
  int64_t g = ceil_div(n, 256);
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

// df[j] += 1 for every entry with value > 0 (DocumentFrequencyAggregator.add: rows hold each id
// once).  Each workgroup counts a contiguous slice of entries in an LDS hash table (open addressing,
// ≤ 8 probes, claimed by CAS) and flushes it with one global atomic per distinct id: a Zipf corpus's
// hot ids — present in almost every row — cost one global atomic per workgroup instead of one per
// row.  Ids that find no slot add to the global count directly.  Integer adds: exact and
// order-independent, so df is identical run to run.
constexpr int kDfSlots = 8192;
constexpr int kDfThreads = 1024;

template <typename V>
__global__ __launch_bounds__(kDfThreads) void k_df_hist(const int32_t* __restrict__ idx, const V* __restrict__ val,
                                                        int64_t nnz, int64_t per_block,
                                                        unsigned long long* __restrict__ df) {
  __shared__ int32_t key[kDfSlots];
  __shared__ uint32_t cnt[kDfSlots];
  for (int i = threadIdx.x; i < kDfSlots; i += kDfThreads) {
    key[i] = -1;
    cnt[i] = 0;
  }
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * per_block;
  const int64_t e1 = e0 + per_block < nnz ? e0 + per_block : nnz;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kDfThreads) {
    if (!(val[e] > V(0))) continue;
    const int32_t id = idx[e];
    uint32_t h = ((uint32_t)id * 2654435761u) >> 19;  // 13 bits
    bool done = false;
    for (int probe = 0; probe < 8 && !done; ++probe, h = (h + 1) & (kDfSlots - 1)) {
      const int32_t k = atomicCAS(&key[h], -1, id);
      if (k == -1 || k == id) {
        atomicAdd(&cnt[h], 1u);
        done = true;
      }
    }
    if (!done) atomicAdd(&df[id], 1ull);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kDfSlots; i += kDfThreads)
    if (key[i] >= 0) atomicAdd(&df[key[i]], (unsigned long long)cnt[i]);
}

void doc_freq(Ctx& c, const DCsr& m, int64_t* d_df) {
  HIP_CHECK(hipMemsetAsync(d_df, 0, sizeof(int64_t) * m.cols, c.stream));
  if (m.nnz == 0) return;
  // ≈ 2 workgroups per CU, each a contiguous slice (hot ids repeat within it)
  const int64_t blocks = std::min<int64_t>(512, ceil_div(m.nnz, (int64_t)kDfThreads));
  const int64_t per = ceil_div(m.nnz, blocks);
  auto* df = reinterpret_cast<unsigned long long*>(d_df);
  if (m.dtype == STC_F32)
    k_df_hist<float><<<(unsigned)blocks, kDfThreads, 0, c.stream>>>(m.indices.as<int32_t>(), m.values.as<float>(),
                                                                     m.nnz, per, df);
  else
    k_df_hist<double><<<(unsigned)blocks, kDfThreads, 0, c.stream>>>(m.indices.as<int32_t>(), m.values.as<double>(),
                                                                      m.nnz, per, df);
  KERNEL_CHECK();
}

// DocumentFrequencyAggregator.idf(): df >= minDocFreq ? ln((m + 1) / (df + 1)) : 0
__global__ __launch_bounds__(256) void k_idf(const int64_t* __restrict__ df, int64_t cols, double m,
                                             int64_t min_df, double* __restrict__ idf) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < cols; j += (int64_t)gridDim.x * 256) {
    const int64_t d = df[j];
    idf[j] = d >= min_df ? log((m + 1.0) / ((double)d + 1.0)) : 0.0;
  }
}

void finalize(Ctx& c, const int64_t* d_df, int64_t cols, int64_t m, int64_t min_df, double* d_idf) {
  k_idf<<<grid_for(cols), 256, 0, c.stream>>>(d_df, cols, (double)m, min_df, d_idf);
  KERNEL_CHECK();
}

// IDFModel.transform: v *= idf[j]  (reference mode: an idf of exactly 0 → zero_floor)
template <typename V>
__global__ __launch_bounds__(256) void k_transform(const int32_t* __restrict__ idx, V* __restrict__ val,
                                                   int64_t nnz, const double* __restrict__ idf,
                                                   double zero_floor) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * 256) {
    double w = idf[idx[e]];
    if (zero_floor > 0.0 && w == 0.0) w = zero_floor;
    val[e] = (V)((double)val[e] * w);
  }
}

void transform(Ctx& c, DCsr& m, const double* d_idf, double zero_floor) {
  if (m.nnz == 0) return;
  if (m.dtype == STC_F32)
    k_transform<float><<<grid_for(m.nnz), 256, 0, c.stream>>>(m.indices.as<int32_t>(), m.values.as<float>(),
                                                              m.nnz, d_idf, zero_floor);
  else
    k_transform<double><<<grid_for(m.nnz), 256, 0, c.stream>>>(m.indices.as<int32_t>(), m.values.as<double>(),
                                                               m.nnz, d_idf, zero_floor);
  KERNEL_CHECK();
}

}  // namespace idf
}  // namespace stc
