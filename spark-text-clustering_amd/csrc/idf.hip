// idf.hip — K3 (document frequency), K4 (idf finalise), K5 (TF·IDF transform) for gfx950.
//
// Replaces [U] mllib.feature.IDF.fit (DocumentFrequencyAggregator.add/merge/idf) and
// IDFModel.transform, reached from LDAClustering.scala:177 (`new IDF(2).fit(tf).idf`) and
// :180-192 (tf × idf with the idf==0 → 1e-4 floor).
//
// df is a column histogram of a Zipf-skewed CSR: the hottest term sits in nearly every row, so
// per-entry global atomics would serialise on a handful of addresses; doc_freq counts vocabulary
// tiles in LDS instead (see there).
#include <hipcub/hipcub.hpp>

#include "stc_internal.h"

namespace stc {
namespace idf {

static int grid_for(int64_t n) {
  int64_t g = ceil_div(n, 256);
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

// df[j] = #entries (rows hold each id once) with id j and value > 0 (DocumentFrequencyAggregator.add).
// A Zipf corpus's hot ids sit in almost every row, and device-scope atomics run at a few G/s, so
// the histogram is built without per-entry global atomics:
//  * numFeatures ≤ 2^18 (k_df_tile): vocabulary tiles of 2^15 ids; workgroup (tile t, entry chunk
//    c) streams the chunk's ids, counts those in its tile in LDS (128 KB of u32), and writes its
//    partial histogram; k_df_reduce sums the partials over the chunks in chunk order.
//  * larger vocabularies: the (value > 0) ids are radix-sorted and each run's [lo, hi) recorded.
// Both are exact integer counts, identical run to run.
constexpr int kTileBits = 15;
constexpr int kTile = 1 << kTileBits;
constexpr int kTileThreads = 1024;

template <typename V>
__global__ __launch_bounds__(kTileThreads) void k_df_tile(const int32_t* __restrict__ idx, const V* __restrict__ val,
                                                          int64_t nnz, int64_t per, int n_tiles, int64_t cols,
                                                          uint32_t* __restrict__ part) {
  extern __shared__ uint32_t cnt[];
  const int t = blockIdx.x % n_tiles;
  const int64_t c = blockIdx.x / n_tiles;
  for (int i = threadIdx.x; i < kTile; i += kTileThreads) cnt[i] = 0;
  __syncthreads();
  // per is a multiple of 8: each thread streams 8 consecutive ids (two 16-byte loads in flight)
  const int64_t e0 = c * per, e1 = e0 + per < nnz ? e0 + per : nnz;
  for (int64_t e = e0 + 8 * threadIdx.x; e < e1; e += 8 * kTileThreads) {
    int32_t id[8];
    if (e + 8 <= e1) {
      const int4 a = *reinterpret_cast<const int4*>(idx + e), b = *reinterpret_cast<const int4*>(idx + e + 4);
      id[0] = a.x; id[1] = a.y; id[2] = a.z; id[3] = a.w;
      id[4] = b.x; id[5] = b.y; id[6] = b.z; id[7] = b.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) id[q] = e + q < e1 ? idx[e + q] : -1;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (id[q] >= 0 && (id[q] >> kTileBits) == t && val[e + q] > V(0)) atomicAdd(&cnt[id[q] & (kTile - 1)], 1u);
  }
  __syncthreads();
  const int64_t j0 = (int64_t)t * kTile;
  uint32_t* out = part + c * cols + j0;
  for (int i = threadIdx.x; i < kTile && j0 + i < cols; i += kTileThreads) out[i] = cnt[i];
}

__global__ __launch_bounds__(256) void k_df_reduce(const uint32_t* __restrict__ part, int64_t chunks, int64_t cols,
                                                   int64_t* __restrict__ df) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < cols; j += (int64_t)gridDim.x * 256) {
    int64_t s = 0;
    for (int64_t c = 0; c < chunks; ++c) s += part[c * cols + j];
    df[j] = s;
  }
}

template <typename V>
__global__ __launch_bounds__(256) void k_keys(const int32_t* __restrict__ idx, const V* __restrict__ val, int64_t nnz,
                                              uint32_t sentinel, uint32_t* __restrict__ keys) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * 256)
    keys[e] = val[e] > V(0) ? (uint32_t)idx[e] : sentinel;
}

__global__ __launch_bounds__(256) void k_runs(const uint32_t* __restrict__ k, int64_t n, uint32_t sentinel,
                                              int64_t* __restrict__ df) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
    const uint32_t v = k[p];
    if (v == sentinel) continue;
    // df = hi − lo: the run's last position adds hi, its first subtracts lo (two atomics per id)
    auto* d = reinterpret_cast<unsigned long long*>(df);
    if (p == n - 1 || k[p + 1] != v) atomicAdd(&d[v], (unsigned long long)(p + 1));
    if (p == 0 || k[p - 1] != v) atomicAdd(&d[v], (unsigned long long)(-p));
  }
}

void doc_freq(Ctx& c, const DCsr& m, int64_t* d_df) {
  hipStream_t s = c.stream;
  HIP_CHECK(hipMemsetAsync(d_df, 0, sizeof(int64_t) * m.cols, s));
  if (m.nnz == 0) return;
  if (m.cols <= (int64_t(8) << kTileBits)) {
    const int T = (int)ceil_div(m.cols, (int64_t)kTile);
    const int64_t C = std::max<int64_t>(1, std::min<int64_t>(ceil_div(m.nnz, (int64_t)65536), 1024 / T));
    const int64_t per = ceil_div(ceil_div(m.nnz, C), (int64_t)8) * 8;
    DevBuf& part = c.scratch[0];
    part.reserve(sizeof(uint32_t) * C * m.cols);
    const size_t lds = sizeof(uint32_t) * kTile;
    if (m.dtype == STC_F32) {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_df_tile<float>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      k_df_tile<float><<<(unsigned)(T * C), kTileThreads, lds, s>>>(m.indices.as<int32_t>(), m.values.as<float>(),
                                                                    m.nnz, per, T, m.cols, part.as<uint32_t>());
    } else {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_df_tile<double>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      k_df_tile<double><<<(unsigned)(T * C), kTileThreads, lds, s>>>(m.indices.as<int32_t>(), m.values.as<double>(),
                                                                     m.nnz, per, T, m.cols, part.as<uint32_t>());
    }
    KERNEL_CHECK();
    k_df_reduce<<<grid_for(m.cols), 256, 0, s>>>(part.as<uint32_t>(), C, m.cols, d_df);
    KERNEL_CHECK();
    return;
  }
  STC_REQUIRE(m.nnz < (int64_t(1) << 31), "idf: at most 2^31-1 entries per call");
  const uint32_t sentinel = (uint32_t)m.cols;
  int nbits = 1;
  while ((int64_t(1) << nbits) <= (int64_t)sentinel) ++nbits;
  DevBuf& keys = c.scratch[0];
  DevBuf& sorted = c.scratch[1];
  DevBuf tmp;
  keys.reserve(4 * m.nnz);
  sorted.reserve(4 * m.nnz);
  if (m.dtype == STC_F32)
    k_keys<float><<<grid_for(m.nnz), 256, 0, s>>>(m.indices.as<int32_t>(), m.values.as<float>(), m.nnz, sentinel,
                                                  keys.as<uint32_t>());
  else
    k_keys<double><<<grid_for(m.nnz), 256, 0, s>>>(m.indices.as<int32_t>(), m.values.as<double>(), m.nnz, sentinel,
                                                   keys.as<uint32_t>());
  KERNEL_CHECK();
  size_t tb = 0;
  HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, keys.as<uint32_t>(), sorted.as<uint32_t>(), (int)m.nnz, 0,
                                              nbits, s));
  tmp.reserve(tb);
  HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp.p, tb, keys.as<uint32_t>(), sorted.as<uint32_t>(), (int)m.nnz, 0,
                                              nbits, s));
  k_runs<<<grid_for(m.nnz), 256, 0, s>>>(sorted.as<uint32_t>(), m.nnz, sentinel, d_df);
  KERNEL_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));  // tmp dies at scope exit
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

// IDFModel.transform: v *= idf[j]  (reference mode: an idf of exactly 0 → zero_floor).  Four entries
// per thread and step: one 16-byte load of ids, two of values, four independent idf gathers (the
// 2 MB idf vector stays in L2), two 16-byte stores.
template <typename V>
__device__ __forceinline__ V idf_scale(V v, double w, double zero_floor) {
  if (zero_floor > 0.0 && w == 0.0) w = zero_floor;
  return (V)((double)v * w);
}
template <typename V>
__global__ __launch_bounds__(256) void k_transform(const int32_t* __restrict__ idx, V* __restrict__ val,
                                                   int64_t nnz, const double* __restrict__ idf,
                                                   double zero_floor) {
  const int64_t n4 = nnz / 4;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n4; q += (int64_t)gridDim.x * 256) {
    const int4 i = reinterpret_cast<const int4*>(idx)[q];
    V* p = val + 4 * q;
    const double w0 = idf[i.x], w1 = idf[i.y], w2 = idf[i.z], w3 = idf[i.w];
    p[0] = idf_scale(p[0], w0, zero_floor);
    p[1] = idf_scale(p[1], w1, zero_floor);
    p[2] = idf_scale(p[2], w2, zero_floor);
    p[3] = idf_scale(p[3], w3, zero_floor);
  }
  const int64_t e = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x;  // the last nnz % 4 entries
  if (e < nnz) val[e] = idf_scale(val[e], idf[idx[e]], zero_floor);
}

void transform(Ctx& c, DCsr& m, const double* d_idf, double zero_floor) {
  if (m.nnz == 0) return;
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(ceil_div(m.nnz / 4, 256), 1), 8192);
  if (m.dtype == STC_F32)
    k_transform<float><<<g, 256, 0, c.stream>>>(m.indices.as<int32_t>(), m.values.as<float>(), m.nnz, d_idf,
                                                zero_floor);
  else
    k_transform<double><<<g, 256, 0, c.stream>>>(m.indices.as<int32_t>(), m.values.as<double>(), m.nnz, d_idf,
                                                 zero_floor);
  KERNEL_CHECK();
}

}  // namespace idf
}  // namespace stc
