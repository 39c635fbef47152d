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
//  * numFeatures ≤ 2^18: vocabulary tiles of 2^15 ids counted in LDS (128 KB of u32) per chunk group,
//    partial histograms summed in group order by k_df_reduce.  k_df_tiled (default) streams a group's
//    ids once per tile from L2; k_df_bin + k_df_binned (round 3, STC_DF_BINNED=1) first split each
//    chunk by tile into a u16 bin array.
//  * larger vocabularies: the (value > 0) ids are radix-sorted and each run's [lo, hi) recorded.
// Both are exact integer counts, identical run to run.
constexpr int kTileBits = 15;
constexpr int kTile = 1 << kTileBits;
constexpr int kTileThreads = 1024;

// Binned variant (one read of the CSR): k_df_bin splits each chunk of kBinChunk entries by tile —
// the (value > 0) ids' low 15 bits as u16, tile-major inside the chunk's own region of the bin array
// (no global scan: a chunk's region is its kBinChunk slots) — and k_df_binned counts one tile over a
// group of chunks in LDS.  Bytes per entry: 4 + s (id, value) read, 2 written, 2 read.
constexpr int kBinChunk = 16384;
constexpr int kBinThreads = 1024;
constexpr int kBinPer = kBinChunk / kBinThreads;  // entries per thread
constexpr int kMaxTiles = 8;  // numFeatures ≤ 2^18 (32 tiles for 2^20 measured 2.2× slower than the sort)

template <typename V, int MT>
__global__ __launch_bounds__(kBinThreads) void k_df_bin(const int32_t* __restrict__ idx, const V* __restrict__ val,
                                                        int64_t nnz, int n_tiles, uint16_t* __restrict__ bins,
                                                        int32_t* __restrict__ tab /* [chunk][2·kMaxTiles] */) {
  __shared__ int32_t wtot[kBinThreads / 64][MT];
  __shared__ int32_t tbase[MT + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t c = blockIdx.x, e0 = c * kBinChunk;
  uint32_t ent[kBinPer];  // tile << 16 | low id, or ~0u
  int cnt[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) cnt[t] = 0;
#pragma unroll
  for (int u = 0; u < kBinPer; ++u) {
    const int64_t e = e0 + u * kBinThreads + tid;
    uint32_t x = ~0u;
    if (e < nnz && (val == nullptr || val[e] > V(0))) {  // val = nullptr: every value is known > 0
      const uint32_t id = (uint32_t)idx[e];
      x = ((id >> kTileBits) << 16) | (id & (kTile - 1));
    }
    ent[u] = x;
#pragma unroll
    for (int t = 0; t < MT; ++t) cnt[t] += (x >> 16) == (uint32_t)t ? 1 : 0;
  }
  // exclusive prefix of each tile's counts over the block's threads (thread order)
  int pre[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    int v = cnt[t];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    pre[t] = v - cnt[t];
    if (lane == 63) wtot[wave][t] = v;
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int t = 0; t < MT; ++t) {
      tbase[t] = run;
      int tot = 0;
      for (int w = 0; w < kBinThreads / 64; ++w) tot += wtot[w][t];
      tab[c * 2 * kMaxTiles + t] = run;                 // the tile's offset inside the chunk region
      tab[c * 2 * kMaxTiles + kMaxTiles + t] = tot;     // and its count
      run += tot;
    }
    tbase[MT] = run;
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    int wb = 0;
    for (int w = 0; w < wave; ++w) wb += wtot[w][t];
    pre[t] += tbase[t] + wb;
  }
  uint16_t* out = bins + e0;
#pragma unroll
  for (int u = 0; u < kBinPer; ++u) {
    const uint32_t x = ent[u];
    if (x != ~0u) {
      const int t = (int)(x >> 16);
      int pos = 0;
#pragma unroll
      for (int q = 0; q < MT; ++q)
        if (q == t) pos = pre[q]++;
      out[pos] = (uint16_t)(x & 0xFFFF);
    }
  }
}

__global__ __launch_bounds__(kTileThreads) void k_df_binned(const uint16_t* __restrict__ bins,
                                                            const int32_t* __restrict__ tab, int64_t chunks,
                                                            int64_t per_group, int n_tiles, int64_t cols,
                                                            uint32_t* __restrict__ part) {
  extern __shared__ uint32_t cnt[];
  const int t = blockIdx.x % n_tiles;
  const int64_t g = blockIdx.x / n_tiles;
  for (int i = threadIdx.x; i < kTile; i += kTileThreads) cnt[i] = 0;
  __syncthreads();
  const int64_t c0 = g * per_group, c1 = c0 + per_group < chunks ? c0 + per_group : chunks;
  for (int64_t c = c0; c < c1; ++c) {
    const int32_t off = tab[c * 2 * kMaxTiles + t], n = tab[c * 2 * kMaxTiles + kMaxTiles + t];
    const uint16_t* b = bins + c * kBinChunk + off;
    for (int i = threadIdx.x; i < n; i += kTileThreads) atomicAdd(&cnt[b[i]], 1u);
  }
  __syncthreads();
  const int64_t j0 = (int64_t)t * kTile;
  uint32_t* out = part + g * cols + j0;
  for (int i = threadIdx.x; i < kTile && j0 + i < cols; i += kTileThreads) out[i] = cnt[i];
}

// Tiled variant (round 4, the default for numFeatures ≤ 2^18): no bin array.  Workgroup (g, t) streams
// the whole index range of chunk group g and counts the ids of vocabulary tile t in LDS; the T
// workgroups of one group are placed on one XCD (blockIdx % 8 picks the XCD) and start together, so
// the group's indices come from HBM once and are re-read T times from that XCD's L2.  Bytes per
// entry from HBM: 4 (id) [+ s (value) when not known positive]; one workgroup per CU (128 KB of LDS).
constexpr int kTiledThreads = 1024;
constexpr int kTiledUnroll = 4;  // int4 index loads in flight per thread

__device__ __forceinline__ void tile_add(uint32_t* cnt, uint32_t id, uint32_t t) {
  if ((id >> kTileBits) == t) atomicAdd(&cnt[id & (kTile - 1)], 1u);
}

template <typename V>
__global__ __launch_bounds__(kTiledThreads) void k_df_tiled(const int32_t* __restrict__ idx,
                                                            const V* __restrict__ val, int64_t nnz,
                                                            int n_tiles, int64_t groups, int64_t per,
                                                            int64_t cols, uint32_t* __restrict__ part) {
  extern __shared__ uint32_t cnt[];
  const int64_t b = blockIdx.x;
  int t;
  int64_t g;
  if (groups % 8 == 0) {  // XCD-aware: the n_tiles workgroups of a group share blockIdx % 8
    const int64_t l = b >> 3;
    t = (int)(l % n_tiles);
    g = (l / n_tiles) * 8 + (b & 7);
  } else {
    t = (int)(b % n_tiles);
    g = b / n_tiles;
  }
  const int tid = threadIdx.x;
  for (int i = tid; i < kTile; i += kTiledThreads) cnt[i] = 0;
  __syncthreads();
  const int64_t e0 = g * per, e1 = e0 + per < nnz ? e0 + per : nnz;  // per % 4 == 0
  const uint32_t ut = (uint32_t)t;
  if (val == nullptr) {  // every value known > 0: ids only, 16-byte loads
    const int4* i4 = reinterpret_cast<const int4*>(idx + e0);
    const int64_t n4 = e1 > e0 ? (e1 - e0) >> 2 : 0;
    int64_t q = tid;
    for (; q + (kTiledUnroll - 1) * kTiledThreads < n4; q += kTiledUnroll * kTiledThreads) {
      int4 v[kTiledUnroll];
#pragma unroll
      for (int u = 0; u < kTiledUnroll; ++u) v[u] = i4[q + u * kTiledThreads];
#pragma unroll
      for (int u = 0; u < kTiledUnroll; ++u) {
        tile_add(cnt, (uint32_t)v[u].x, ut);
        tile_add(cnt, (uint32_t)v[u].y, ut);
        tile_add(cnt, (uint32_t)v[u].z, ut);
        tile_add(cnt, (uint32_t)v[u].w, ut);
      }
    }
    for (; q < n4; q += kTiledThreads) {
      const int4 v = i4[q];
      tile_add(cnt, (uint32_t)v.x, ut);
      tile_add(cnt, (uint32_t)v.y, ut);
      tile_add(cnt, (uint32_t)v.z, ut);
      tile_add(cnt, (uint32_t)v.w, ut);
    }
    for (int64_t e = e0 + 4 * n4 + tid; e < e1; e += kTiledThreads) tile_add(cnt, (uint32_t)idx[e], ut);
  } else {
    for (int64_t e = e0 + tid; e < e1; e += kTiledThreads)
      if (val[e] > V(0)) tile_add(cnt, (uint32_t)idx[e], ut);
  }
  __syncthreads();
  const int64_t j0 = (int64_t)t * kTile;
  uint32_t* out = part + g * cols + j0;
  for (int i = tid; i < kTile && j0 + i < cols; i += kTiledThreads) out[i] = cnt[i];
}

// Row-grouped u16 variant (round 4, HashingTF output: every row holds an id at most once).  A group
// of ≤ 65535 rows counts any id at most 65535 times, so two ids share one u32 LDS word as u16 halves
// and a 128 KB tile spans 2^16 ids: 4 tiles at 2^18 buckets (half the L2 re-reads of k_df_tiled).
// Workgroup (g, t) reads its rows' entry range from indptr.
constexpr int kTile16Bits = 16;
__device__ __forceinline__ void tile16_add(uint32_t* cnt, uint32_t id, uint32_t t) {
  if ((id >> kTile16Bits) == t) atomicAdd(&cnt[(id & 0xFFFF) >> 1], 1u << (16 * (id & 1)));
}
__global__ __launch_bounds__(kTiledThreads) void k_df_rows16(const int32_t* __restrict__ idx,
                                                             const int64_t* __restrict__ indptr, int64_t rows,
                                                             int n_tiles, int64_t groups, int64_t rpg,
                                                             int64_t cols, uint32_t* __restrict__ part) {
  extern __shared__ uint32_t cnt[];
  const int64_t b = blockIdx.x;
  int t;
  int64_t g;
  if (groups % 8 == 0) {  // XCD-aware, as k_df_tiled
    const int64_t l = b >> 3;
    t = (int)(l % n_tiles);
    g = (l / n_tiles) * 8 + (b & 7);
  } else {
    t = (int)(b % n_tiles);
    g = b / n_tiles;
  }
  const int tid = threadIdx.x;
  for (int i = tid; i < kTile; i += kTiledThreads) cnt[i] = 0;  // 2^15 words = 2^16 u16 counters
  __syncthreads();
  const int64_t r0 = g * rpg, r1 = r0 + rpg < rows ? r0 + rpg : rows;
  const int64_t e0 = indptr[r0], e1 = indptr[r1];
  const uint32_t ut = (uint32_t)t;
  const int64_t a0 = (e0 + 3) & ~int64_t(3);  // the int4-aligned middle [a0, a1)
  const int64_t a1 = e1 & ~int64_t(3);
  if (a0 >= a1) {
    for (int64_t e = e0 + tid; e < e1; e += kTiledThreads) tile16_add(cnt, (uint32_t)idx[e], ut);
  } else {
    if (e0 + tid < a0) tile16_add(cnt, (uint32_t)idx[e0 + tid], ut);
    if (a1 + tid < e1) tile16_add(cnt, (uint32_t)idx[a1 + tid], ut);
    const int4* i4 = reinterpret_cast<const int4*>(idx + a0);
    const int64_t n4 = (a1 - a0) >> 2;
    int64_t q = tid;
    for (; q + (kTiledUnroll - 1) * kTiledThreads < n4; q += kTiledUnroll * kTiledThreads) {
      int4 v[kTiledUnroll];
#pragma unroll
      for (int u = 0; u < kTiledUnroll; ++u) v[u] = i4[q + u * kTiledThreads];
#pragma unroll
      for (int u = 0; u < kTiledUnroll; ++u) {
        tile16_add(cnt, (uint32_t)v[u].x, ut);
        tile16_add(cnt, (uint32_t)v[u].y, ut);
        tile16_add(cnt, (uint32_t)v[u].z, ut);
        tile16_add(cnt, (uint32_t)v[u].w, ut);
      }
    }
    for (; q < n4; q += kTiledThreads) {
      const int4 v = i4[q];
      tile16_add(cnt, (uint32_t)v.x, ut);
      tile16_add(cnt, (uint32_t)v.y, ut);
      tile16_add(cnt, (uint32_t)v.z, ut);
      tile16_add(cnt, (uint32_t)v.w, ut);
    }
  }
  __syncthreads();
  const int64_t j0 = (int64_t)t << kTile16Bits;
  uint32_t* out = part + g * cols + j0;
  for (int i = tid; i < (1 << kTile16Bits) && j0 + i < cols; i += kTiledThreads)
    out[i] = (cnt[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
}

__global__ __launch_bounds__(256) void k_df_reduce(const uint32_t* __restrict__ part, int64_t chunks, int64_t cols,
                                                   int64_t* __restrict__ df, double m, int64_t min_df,
                                                   double* __restrict__ idf /* nullptr: df only */) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < cols; j += (int64_t)gridDim.x * 256) {
    int64_t s = 0;
    for (int64_t c = 0; c < chunks; ++c) s += part[c * cols + j];
    df[j] = s;
    if (idf) idf[j] = s >= min_df ? log((m + 1.0) / ((double)s + 1.0)) : 0.0;  // as k_idf
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

bool doc_freq(Ctx& c, const DCsr& m, int64_t* d_df, const IdfFinal* fin) {
  hipStream_t s = c.stream;
  const double fin_m = fin ? fin->m : 0.0;
  const int64_t fin_min = fin ? fin->min_df : 0;
  double* const fin_idf = fin ? fin->idf : nullptr;
  if (m.nnz == 0) {
    HIP_CHECK(hipMemsetAsync(d_df, 0, sizeof(int64_t) * m.cols, s));
    return false;
  }
  if (m.unique_ids && m.cols <= (int64_t(kMaxTiles / 2) << kTile16Bits) && c.df_tiled && c.df_rows16 &&
      m.rows > 0) {
    const int T = (int)ceil_div(m.cols, (int64_t)1 << kTile16Bits);
    const int64_t want = std::max<int64_t>(1, (int64_t)c.cus / T);
    int64_t G = std::max<int64_t>(std::min<int64_t>(want, ceil_div(m.nnz, (int64_t)65536)), 1);
    if (G >= 8) G -= G % 8;
    int64_t rpg = std::min<int64_t>(ceil_div(m.rows, G), 65535);  // ≤ 65535 rows: the u16 bound
    G = ceil_div(m.rows, rpg);
    DevBuf& part = c.scratch[0];
    part.reserve(sizeof(uint32_t) * G * m.cols);
    const size_t lds = sizeof(uint32_t) * kTile;
    HIP_CHECK(hipFuncSetAttribute((const void*)k_df_rows16, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_df_rows16<<<(unsigned)(T * G), kTiledThreads, lds, s>>>(m.indices.as<int32_t>(), m.indptr.as<int64_t>(), m.rows,
                                                              T, G, rpg, m.cols, part.as<uint32_t>());
    KERNEL_CHECK();
    k_df_reduce<<<grid_for(m.cols), 256, 0, s>>>(part.as<uint32_t>(), G, m.cols, d_df, fin_m, fin_min, fin_idf);
    KERNEL_CHECK();
    return fin != nullptr;
  }
  if (m.cols <= (int64_t(kMaxTiles) << kTileBits) && c.df_tiled) {
    const int T = (int)ceil_div(m.cols, (int64_t)kTile);
    // groups: a multiple of 8 (the XCD mapping) with T·groups ≈ one workgroup per CU, fewer for small
    // inputs (≥ 64 Ki entries per group)
    const int64_t want = std::max<int64_t>(1, (int64_t)c.cus / T);
    int64_t G = std::min<int64_t>(want, ceil_div(m.nnz, (int64_t)65536));
    if (G >= 8) G -= G % 8;
    G = std::max<int64_t>(G, 1);
    const int64_t per = ceil_div(ceil_div(m.nnz, G), (int64_t)4) * 4;
    G = ceil_div(m.nnz, per);  // (rounding `per` up can leave G off a multiple of 8: the plain mapping)
    DevBuf& part = c.scratch[0];
    part.reserve(sizeof(uint32_t) * G * m.cols);
    const size_t lds = sizeof(uint32_t) * kTile;
    if (m.dtype == STC_F32) {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_df_tiled<float>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
      k_df_tiled<float><<<(unsigned)(T * G), kTiledThreads, lds, s>>>(
          m.indices.as<int32_t>(), m.positive ? nullptr : m.values.as<float>(), m.nnz, T, G, per, m.cols,
          part.as<uint32_t>());
    } else {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_df_tiled<double>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
      k_df_tiled<double><<<(unsigned)(T * G), kTiledThreads, lds, s>>>(
          m.indices.as<int32_t>(), m.positive ? nullptr : m.values.as<double>(), m.nnz, T, G, per, m.cols,
          part.as<uint32_t>());
    }
    KERNEL_CHECK();
    k_df_reduce<<<grid_for(m.cols), 256, 0, s>>>(part.as<uint32_t>(), G, m.cols, d_df, fin_m, fin_min, fin_idf);
    KERNEL_CHECK();
    return fin != nullptr;
  }
  if (m.cols <= (int64_t(kMaxTiles) << kTileBits)) {
    const int T = (int)ceil_div(m.cols, (int64_t)kTile);
    const int64_t chunks = ceil_div(m.nnz, (int64_t)kBinChunk);
    const int64_t G = std::max<int64_t>(1, std::min<int64_t>(chunks, 1024 / T));  // chunk groups
    const int64_t per_group = ceil_div(chunks, G);
    const int64_t groups = ceil_div(chunks, per_group);
    DevBuf& bins = c.scratch[1];
    DevBuf& tab = c.scratch[2];
    DevBuf& part = c.scratch[0];
    bins.reserve(sizeof(uint16_t) * chunks * kBinChunk);
    tab.reserve(sizeof(int32_t) * chunks * 2 * kMaxTiles);
    part.reserve(sizeof(uint32_t) * groups * m.cols);
    // a CSR whose values are all known > 0 (HashingTF output) is counted from its indices alone
    auto bin = [&](auto mt) {
      constexpr int MT = decltype(mt)::value;
      if (m.dtype == STC_F32)
        k_df_bin<float, MT><<<(unsigned)chunks, kBinThreads, 0, s>>>(
            m.indices.as<int32_t>(), m.positive ? nullptr : m.values.as<float>(), m.nnz, T, bins.as<uint16_t>(),
            tab.as<int32_t>());
      else
        k_df_bin<double, MT><<<(unsigned)chunks, kBinThreads, 0, s>>>(
            m.indices.as<int32_t>(), m.positive ? nullptr : m.values.as<double>(), m.nnz, T, bins.as<uint16_t>(),
            tab.as<int32_t>());
    };
    bin(std::integral_constant<int, kMaxTiles>{});
    KERNEL_CHECK();
    const size_t lds = sizeof(uint32_t) * kTile;
    HIP_CHECK(hipFuncSetAttribute((const void*)k_df_binned, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_df_binned<<<(unsigned)(T * groups), kTileThreads, lds, s>>>(bins.as<uint16_t>(), tab.as<int32_t>(), chunks,
                                                                  per_group, T, m.cols, part.as<uint32_t>());
    KERNEL_CHECK();
    k_df_reduce<<<grid_for(m.cols), 256, 0, s>>>(part.as<uint32_t>(), groups, m.cols, d_df, fin_m, fin_min, fin_idf);
    KERNEL_CHECK();
    return fin != nullptr;
  }
  STC_REQUIRE(m.nnz < (int64_t(1) << 31), "idf: at most 2^31-1 entries per call");
  HIP_CHECK(hipMemsetAsync(d_df, 0, sizeof(int64_t) * m.cols, s));  // k_runs adds into it
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
  return false;
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
// Round 4: two quads per thread and step with all their loads issued before any use, and the index
// and value streams marked non-temporal so they do not evict the idf vector from L2.
template <typename V>
__global__ __launch_bounds__(256) void k_transform(const int32_t* __restrict__ idx, V* __restrict__ val,
                                                   int64_t nnz, const double* __restrict__ idf,
                                                   double zero_floor) {
  typedef V V4 __attribute__((ext_vector_type(4)));
  typedef int32_t I4 __attribute__((ext_vector_type(4)));
  const int64_t n4 = nnz / 4;
  const int64_t S = (int64_t)gridDim.x * 256;
  const I4* i4 = reinterpret_cast<const I4*>(idx);
  V4* v4 = reinterpret_cast<V4*>(val);
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n4; q += 2 * S) {
    const bool two = q + S < n4;
    const I4 ia = __builtin_nontemporal_load(i4 + q);
    const I4 ib = two ? __builtin_nontemporal_load(i4 + q + S) : I4{};
    V4 a = __builtin_nontemporal_load(v4 + q);
    V4 b = two ? __builtin_nontemporal_load(v4 + q + S) : V4{};
    const double wa0 = idf[ia.x], wa1 = idf[ia.y], wa2 = idf[ia.z], wa3 = idf[ia.w];
    const double wb0 = idf[ib.x], wb1 = idf[ib.y], wb2 = idf[ib.z], wb3 = idf[ib.w];
    a.x = idf_scale(a.x, wa0, zero_floor);
    a.y = idf_scale(a.y, wa1, zero_floor);
    a.z = idf_scale(a.z, wa2, zero_floor);
    a.w = idf_scale(a.w, wa3, zero_floor);
    __builtin_nontemporal_store(a, v4 + q);
    if (two) {
      b.x = idf_scale(b.x, wb0, zero_floor);
      b.y = idf_scale(b.y, wb1, zero_floor);
      b.z = idf_scale(b.z, wb2, zero_floor);
      b.w = idf_scale(b.w, wb3, zero_floor);
      __builtin_nontemporal_store(b, v4 + q + S);
    }
  }
  const int64_t e = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x;  // the last nnz % 4 entries
  if (e < nnz) val[e] = idf_scale(val[e], idf[idx[e]], zero_floor);
}

// ---- hot-idf LDS cache (round 4): k_transform is bound by its idf gathers (one random 8-byte L2 read per
// entry).  With a Zipf vocabulary most entries hit few ids: the device IDF model keeps, for each of 2^14
// slots (id mod 2^14), the idf of the slot's highest-df id and that id's tag (id >> 14, u8), so a
// workgroup holds 144 KB of the table in LDS and gathers from L2 only on a tag miss.  Config 2: ~75 %
// of entries hit.  Tags need ids < 2^21 (numFeatures ≤ 2^21; larger vocabularies use k_transform).
#ifndef IDF_CACHE_BITS
#define IDF_CACHE_BITS 14  // 2^14 slots, 144 KB: one workgroup per CU
#endif
constexpr int kCacheBits = IDF_CACHE_BITS;
constexpr int kCacheWgPerCu = IDF_CACHE_BITS <= 13 ? 2 : 1;  // workgroups whose tables fit a CU's LDS
constexpr int kCacheSlots = 1 << kCacheBits;
constexpr int kCacheThreads = 1024;
#ifndef IDF_CACHE_UNROLL
#define IDF_CACHE_UNROLL 4
#endif
constexpr int kCacheUnroll = IDF_CACHE_UNROLL;  // quads per thread and step (2: 0.81 ms)
constexpr uint8_t kCacheEmpty = 0xFF;

__global__ __launch_bounds__(256) void k_idf_cache(const int64_t* __restrict__ df, const double* __restrict__ idf,
                                                   int64_t cols, double* __restrict__ cval,
                                                   uint8_t* __restrict__ ctag) {
  const int sl = blockIdx.x * 256 + threadIdx.x;
  if (sl >= kCacheSlots) return;
  int best = -1;
  int64_t bdf = -1;
  for (int t = 0; ((int64_t)t << kCacheBits) + sl < cols; ++t) {
    const int64_t d = df[((int64_t)t << kCacheBits) + sl];
    if (d > bdf) {  // ties: the lowest tag
      bdf = d;
      best = t;
    }
  }
  ctag[sl] = best < 0 ? kCacheEmpty : (uint8_t)best;
  cval[sl] = best < 0 ? 0.0 : idf[((int64_t)best << kCacheBits) + sl];
}

template <typename V>
__global__ __launch_bounds__(kCacheThreads) void k_transform_cached(const int32_t* __restrict__ idx,
                                                                   V* __restrict__ val, int64_t nnz,
                                                                   const double* __restrict__ idf,
                                                                   const double* __restrict__ cval,
                                                                   const uint8_t* __restrict__ ctag,
                                                                   double zero_floor) {
  extern __shared__ double lv[];  // [kCacheSlots] values, then [kCacheSlots] u8 tags
  uint8_t* lt = reinterpret_cast<uint8_t*>(lv + kCacheSlots);
  {
    typedef double D2 __attribute__((ext_vector_type(2)));
    const D2* s2 = reinterpret_cast<const D2*>(cval);
    D2* l2 = reinterpret_cast<D2*>(lv);
    for (int i = threadIdx.x; i < kCacheSlots / 2; i += kCacheThreads) l2[i] = s2[i];
    const uint4* t4 = reinterpret_cast<const uint4*>(ctag);
    uint4* lt4 = reinterpret_cast<uint4*>(lt);
    for (int i = threadIdx.x; i < kCacheSlots / 16; i += kCacheThreads) lt4[i] = t4[i];
  }
  __syncthreads();
  auto w_of = [&](int32_t id) -> double {
    const int sl = id & (kCacheSlots - 1);
    return lt[sl] == (uint8_t)(id >> kCacheBits) ? lv[sl] : idf[id];
  };
  typedef V V4 __attribute__((ext_vector_type(4)));
  typedef int32_t I4 __attribute__((ext_vector_type(4)));
  const int64_t n4 = nnz / 4;
  const int64_t S = (int64_t)gridDim.x * kCacheThreads;
  const I4* i4 = reinterpret_cast<const I4*>(idx);
  V4* v4 = reinterpret_cast<V4*>(val);
  // kCacheUnroll quads per thread and step, every load issued before the first lookup: one workgroup per
  // CU (the table's LDS) leaves 4 waves per SIMD, so the memory parallelism has to come from each thread
  for (int64_t q0 = (int64_t)blockIdx.x * kCacheThreads + threadIdx.x; q0 < n4; q0 += kCacheUnroll * S) {
    I4 ii[kCacheUnroll];
    V4 vv[kCacheUnroll];
#pragma unroll
    for (int u = 0; u < kCacheUnroll; ++u) {
      const int64_t q = q0 + u * S;
      ii[u] = q < n4 ? __builtin_nontemporal_load(i4 + q) : I4{};
      vv[u] = q < n4 ? __builtin_nontemporal_load(v4 + q) : V4{};
    }
#pragma unroll
    for (int u = 0; u < kCacheUnroll; ++u) {
      const int64_t q = q0 + u * S;
      const double w0 = w_of(ii[u].x), w1 = w_of(ii[u].y), w2 = w_of(ii[u].z), w3 = w_of(ii[u].w);
      V4 a = vv[u];
      a.x = idf_scale(a.x, w0, zero_floor);
      a.y = idf_scale(a.y, w1, zero_floor);
      a.z = idf_scale(a.z, w2, zero_floor);
      a.w = idf_scale(a.w, w3, zero_floor);
      if (q < n4) __builtin_nontemporal_store(a, v4 + q);
    }
  }
  const int64_t e = 4 * n4 + (int64_t)blockIdx.x * kCacheThreads + threadIdx.x;  // the last nnz % 4 entries
  if (e < nnz) val[e] = idf_scale(val[e], w_of(idx[e]), zero_floor);
}

bool build_cache(Ctx& c, const int64_t* d_df, const double* d_idf, int64_t cols, DevBuf& cache) {
  if (cols > (int64_t(1) << 21) || !c.idf_cache) return false;
  cache.reserve(sizeof(double) * kCacheSlots + kCacheSlots);
  double* cval = cache.as<double>();
  k_idf_cache<<<kCacheSlots / 256, 256, 0, c.stream>>>(d_df, d_idf, cols, cval,
                                                       reinterpret_cast<uint8_t*>(cval + kCacheSlots));
  KERNEL_CHECK();
  return true;
}

void transform(Ctx& c, DCsr& m, const double* d_idf, double zero_floor, const DevBuf* cache) {
  // idf ≥ 0: values stay > 0 only when an idf of 0 is floored (the reference's 1e-4 mode)
  m.positive = m.positive && zero_floor > 0.0;
  if (m.nnz == 0) return;
  if (cache && cache->p && m.cols <= (int64_t(1) << 21)) {
    const double* cval = cache->as<double>();
    const uint8_t* ctag = reinterpret_cast<const uint8_t*>(cval + kCacheSlots);
    const size_t lds = sizeof(double) * kCacheSlots + kCacheSlots;
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)c.cus * kCacheWgPerCu, ceil_div(m.nnz / 4, (int64_t)kCacheThreads)));
    if (m.dtype == STC_F32) {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_transform_cached<float>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      k_transform_cached<float><<<g, kCacheThreads, lds, c.stream>>>(m.indices.as<int32_t>(), m.values.as<float>(),
                                                                     m.nnz, d_idf, cval, ctag, zero_floor);
    } else {
      HIP_CHECK(hipFuncSetAttribute((const void*)k_transform_cached<double>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      k_transform_cached<double><<<g, kCacheThreads, lds, c.stream>>>(m.indices.as<int32_t>(), m.values.as<double>(),
                                                                      m.nnz, d_idf, cval, ctag, zero_floor);
    }
    KERNEL_CHECK();
    return;
  }
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
