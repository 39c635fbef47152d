// hashing_tf.hip — K1 (MurmurHash3_x86_32 + nonNegativeMod) and K2 (per-document bucket
// counting into a sorted CSR) for gfx950.
//
// Replaces [U] mllib.feature.HashingTF.transform / murmur3Hash (Spark 2.4.3, build.sbt:10), i.e.
// the reference's vocab-indexed counting slot LDAClustering.scala:154-167.  Bit-exact.
//
// Layout: the corpus arrives as ONE UTF-8 byte blob + int64 token offsets + int64 doc offsets
// (plain arrays a JNI caller can hand over without per-string objects).  K1 is one lane per token
// (byte-wise reads: tokens are 1–20 bytes, the blob is read once, HBM-bound).  K2 sorts each
// document's bucket ids with a segmented radix sort, flags run heads, scans them, and emits the
// sorted distinct ids + run lengths — no atomics, so hot terms ("the") cost nothing extra.
#include <hipcub/hipcub.hpp>

#include "stc_internal.h"

namespace stc {
namespace hashing {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mix_k1(uint32_t k1) {
  k1 *= 0xCC9E2D51u;
  k1 = rotl32(k1, 15);
  return k1 * 0x1B873593u;
}
__device__ __forceinline__ uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = rotl32(h1, 13);
  return h1 * 5u + 0xE6546B64u;
}
__device__ __forceinline__ uint32_t fmix(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16;
  h1 *= 0x85EBCA6Bu;
  h1 ^= h1 >> 13;
  h1 *= 0xC2B2AE35u;
  h1 ^= h1 >> 16;
  return h1;
}

// MurmurHash3_x86_32(seed 42).  SPARK24 = Spark 2.4 hashUnsafeBytes (each tail byte
// sign-extended and mixed as a block); otherwise the standard tail (Spark 3 hashUnsafeBytes2).
template <bool SPARK24>
__device__ __forceinline__ int32_t murmur3(const uint8_t* p, uint32_t n) {
  uint32_t h1 = 42u;
  const uint32_t nb = n & ~3u;
  for (uint32_t i = 0; i < nb; i += 4) {
    const uint32_t k1 = (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) |
                        ((uint32_t)p[i + 3] << 24);
    h1 = mix_h1(h1, mix_k1(k1));
  }
  if (SPARK24) {
    for (uint32_t i = nb; i < n; ++i) h1 = mix_h1(h1, mix_k1((uint32_t)(int32_t)(int8_t)p[i]));
  } else {
    const uint32_t tail = n - nb;
    uint32_t k1 = 0;
    if (tail >= 3) k1 ^= (uint32_t)p[nb + 2] << 16;
    if (tail >= 2) k1 ^= (uint32_t)p[nb + 1] << 8;
    if (tail >= 1) {
      k1 ^= (uint32_t)p[nb];
      h1 ^= mix_k1(k1);
    }
  }
  return (int32_t)fmix(h1, n);
}

template <bool SPARK24>
__global__ __launch_bounds__(256) void k_hash(const uint8_t* __restrict__ utf8,
                                              const int64_t* __restrict__ tok_off, int64_t n_tok,
                                              int32_t num_features, int32_t* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n_tok;
       t += (int64_t)gridDim.x * 256) {
    const int64_t b = tok_off[t];
    const int32_t h = murmur3<SPARK24>(utf8 + b, (uint32_t)(tok_off[t + 1] - b));
    int32_t raw = h % num_features;  // Utils.nonNegativeMod (Java % truncates toward zero)
    out[t] = raw + (raw < 0 ? num_features : 0);
  }
}

static int grid_for(int64_t n, int64_t per_block = 256, int64_t cap = 256 * 16) {
  int64_t g = ceil_div(n, per_block);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

void hash_tokens(Ctx& c, const uint8_t* d_utf8, const int64_t* d_tok_off, int64_t n_tok,
                 int32_t num_features, int variant, int32_t* d_idx) {
  if (n_tok == 0) return;
  if (variant == STC_HASH_SPARK24)
    k_hash<true><<<grid_for(n_tok), 256, 0, c.stream>>>(d_utf8, d_tok_off, n_tok, num_features, d_idx);
  else
    k_hash<false><<<grid_for(n_tok), 256, 0, c.stream>>>(d_utf8, d_tok_off, n_tok, num_features, d_idx);
  KERNEL_CHECK();
}

// head[t] = 1 iff sorted key t starts a run inside its document
__global__ __launch_bounds__(256) void k_mark_doc_starts(const int64_t* __restrict__ doc_off,
                                                         int64_t n_docs, int32_t* __restrict__ head) {
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < n_docs; d += (int64_t)gridDim.x * 256) {
    const int64_t s = doc_off[d];
    if (s < doc_off[d + 1]) head[s] = 1;
  }
}
__global__ __launch_bounds__(256) void k_heads(const int32_t* __restrict__ keys, int64_t n,
                                               int32_t* __restrict__ head) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    if (t == 0 || keys[t] != keys[t - 1]) head[t] = 1;  // doc starts were set before
  }
}
// incl = inclusive scan of head; for head tokens write index + run start
__global__ __launch_bounds__(256) void k_emit(const int32_t* __restrict__ keys,
                                              const int32_t* __restrict__ head,
                                              const int32_t* __restrict__ incl, int64_t n,
                                              int32_t* __restrict__ out_idx,
                                              int64_t* __restrict__ run_start) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    if (head[t]) {
      const int64_t pos = (int64_t)incl[t] - 1;
      out_idx[pos] = keys[t];
      run_start[pos] = t;
    }
  }
}
template <typename V>
__global__ __launch_bounds__(256) void k_counts(const int64_t* __restrict__ run_start, int64_t nnz,
                                                int64_t n_tok, int binary, V* __restrict__ vals) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * 256) {
    const int64_t e = (p + 1 < nnz) ? run_start[p + 1] : n_tok;
    vals[p] = binary ? V(1) : V(e - run_start[p]);
  }
}
__global__ __launch_bounds__(256) void k_indptr(const int64_t* __restrict__ doc_off, int64_t n_docs,
                                                const int32_t* __restrict__ incl,
                                                int64_t* __restrict__ indptr) {
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d <= n_docs; d += (int64_t)gridDim.x * 256) {
    const int64_t s = doc_off[d];
    indptr[d] = s > 0 ? (int64_t)incl[s - 1] : 0;
  }
}

static int bits_for(int64_t n) {
  int b = 1;
  while ((int64_t(1) << b) < n) ++b;
  return b;
}

void build_csr(Ctx& c, const uint8_t* d_utf8, const int64_t* d_tok_off, int64_t n_tok,
               const int64_t* d_doc_off, int64_t n_docs, int32_t num_features, int binary,
               int variant, int value_dtype, DCsr& out) {
  STC_REQUIRE(n_tok < (int64_t(1) << 31), "at most 2^31-1 tokens per call (split the corpus)");
  out.rows = n_docs;
  out.cols = num_features;
  out.dtype = value_dtype;
  out.indptr.reserve(sizeof(int64_t) * (n_docs + 1));
  if (n_tok == 0) {
    HIP_CHECK(hipMemsetAsync(out.indptr.p, 0, sizeof(int64_t) * (n_docs + 1), c.stream));
    out.nnz = 0;
    return;
  }
  DevBuf keys, sorted, head, incl, runs, tmp;
  keys.reserve(sizeof(int32_t) * n_tok);
  sorted.reserve(sizeof(int32_t) * n_tok);
  head.reserve(sizeof(int32_t) * n_tok);
  incl.reserve(sizeof(int32_t) * n_tok);
  hash_tokens(c, d_utf8, d_tok_off, n_tok, num_features, variant, keys.as<int32_t>());

  const int nbits = bits_for(num_features);
  size_t tb = 0;
  HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortKeys(
      nullptr, tb, keys.as<int32_t>(), sorted.as<int32_t>(), (int)n_tok, (int)n_docs, d_doc_off,
      d_doc_off + 1, 0, nbits, c.stream));
  size_t tb2 = 0;
  HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tb2, head.as<int32_t>(), incl.as<int32_t>(),
                                             (int)n_tok, c.stream));
  tmp.reserve(tb > tb2 ? tb : tb2);
  HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortKeys(
      tmp.p, tb, keys.as<int32_t>(), sorted.as<int32_t>(), (int)n_tok, (int)n_docs, d_doc_off,
      d_doc_off + 1, 0, nbits, c.stream));

  HIP_CHECK(hipMemsetAsync(head.p, 0, sizeof(int32_t) * n_tok, c.stream));
  k_mark_doc_starts<<<grid_for(n_docs), 256, 0, c.stream>>>(d_doc_off, n_docs, head.as<int32_t>());
  KERNEL_CHECK();
  k_heads<<<grid_for(n_tok), 256, 0, c.stream>>>(sorted.as<int32_t>(), n_tok, head.as<int32_t>());
  KERNEL_CHECK();
  HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp.p, tb2, head.as<int32_t>(), incl.as<int32_t>(),
                                             (int)n_tok, c.stream));
  int32_t nnz32 = 0;
  HIP_CHECK(hipMemcpyAsync(&nnz32, incl.as<int32_t>() + (n_tok - 1), sizeof(int32_t),
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  const int64_t nnz = nnz32;
  out.nnz = nnz;
  out.indices.reserve(sizeof(int32_t) * nnz);
  out.values.reserve((value_dtype == STC_F32 ? 4 : 8) * nnz);
  runs.reserve(sizeof(int64_t) * nnz);
  k_emit<<<grid_for(n_tok), 256, 0, c.stream>>>(sorted.as<int32_t>(), head.as<int32_t>(),
                                                incl.as<int32_t>(), n_tok, out.indices.as<int32_t>(),
                                                runs.as<int64_t>());
  KERNEL_CHECK();
  if (value_dtype == STC_F32)
    k_counts<float><<<grid_for(nnz), 256, 0, c.stream>>>(runs.as<int64_t>(), nnz, n_tok, binary,
                                                         out.values.as<float>());
  else
    k_counts<double><<<grid_for(nnz), 256, 0, c.stream>>>(runs.as<int64_t>(), nnz, n_tok, binary,
                                                          out.values.as<double>());
  KERNEL_CHECK();
  k_indptr<<<grid_for(n_docs + 1), 256, 0, c.stream>>>(d_doc_off, n_docs, incl.as<int32_t>(),
                                                       out.indptr.as<int64_t>());
  KERNEL_CHECK();
  HIP_CHECK(hipStreamSynchronize(c.stream));  // scratch buffers die at scope exit
}

}  // namespace hashing
}  // namespace stc
