// tokenizer.hip — K0: Spark ML Tokenizer (`text.toLowerCase.split("\\s")`) on gfx950, the step
// in front of HashingTF.
//
// Replaces [U] org.apache.spark.ml.feature.Tokenizer.createTransformFunc (Spark 2.4.3,
// build.sbt:10): lower-case the document, split on every single Java `\s` character
// ([ \t\n\x0B\f\r]), keep interior empty tokens, drop trailing empty tokens (String.split with
// limit 0), and return the whole string as one token when it holds no separator ("" → [""]).
// The reference's own CoreNLP/OpenNLP front-end (LDAClustering.scala:116-139) stays out of scope.
//
// Lower-casing as Java 8's String.toLowerCase (root locale) — the JVM Spark 2.4.3 runs on — for every
// code point: ASCII inline, the BMP through the generated two-level table case_table.h (Unicode 6.2
// semantics: characters assigned later pass through, as Java 8 leaves them), Deseret (the one cased
// supplementary block in 6.2) inline, everything else passed through.  Every mapping kept keeps its
// UTF-8 length, so output byte i is a function of the character that contains byte i.  Characters whose
// Java mapping is not such a map (U+0130 İ → "i̇", U+03A3 Σ with its Final_Sigma context rule, and the
// capitals whose lower case changes UTF-8 length: U+023A/U+023E, U+1E9E ẞ, U+2126 Ω, U+212A K, U+212B Å,
// U+2C62…, U+A78D, U+A7AA — 18 code points) are REJECTED loudly (STC_ERR_INVALID_ARG with the byte
// position), never silently mis-cased.
//
// Layout: in = one UTF-8 blob + int64 text offsets per document.  Out = the lower-cased blob with
// the separator bytes removed, so token t is the contiguous out[tok_off[t] .. tok_off[t+1]) and
// document d owns tokens [doc_off[d], doc_off[d+1]) — exactly stc_hashing_tf's input.
// One wave per document (k_count: 256 bytes per step as aligned dword lane loads; k_emit: 64); a ballot of the
// separator flags gives each lane its separator rank, from which both the compacted byte position
// and the token starts follow without atomics.  Two passes (count, emit) around one device scan.
// HBM-bound: 2 reads + 1 write of the blob.
#include <hipcub/hipcub.hpp>

#include "case_table.h"
#include "stc_internal.h"

namespace stc {
namespace tokenizer {

constexpr int kWaves = 4;  // waves (documents) per 256-thread workgroup

__device__ __forceinline__ bool is_java_space(uint32_t b) {
  return b == 0x20u || (b >= 0x09u && b <= 0x0Du);  // \t \n \x0B \f \r and ' '
}

// UTF-8 length from the lead byte (0: a continuation byte)
__device__ __forceinline__ int utf8_len(uint32_t b) { return b < 0x80u ? 1 : b < 0xC0u ? 0 : b < 0xE0u ? 2 : b < 0xF0u ? 3 : 4; }

// Java 8 lower case of a BMP code point (0: rejected — see case_table.h)
__device__ __forceinline__ uint32_t lower_bmp(uint32_t cp) {
  const uint32_t pg = kCasePage[cp >> 8];
  return pg ? kCasePages[pg - 1][cp & 0xFFu] : cp;
}
// ... of any code point: the BMP table, Deseret U+10400–U+10427 → +0x28, the rest unchanged
__device__ __forceinline__ uint32_t lower_cp(uint32_t cp) {
  if (cp < 0x10000u) return lower_bmp(cp);
  return (cp >= 0x10400u && cp <= 0x10427u) ? cp + 0x28u : cp;
}
// the code point of the n-byte UTF-8 sequence at text[j] (j + n <= e), or ~0 when malformed
__device__ __forceinline__ uint32_t decode_at(const uint8_t* __restrict__ text, int64_t j, int n) {
  uint32_t cp = text[j] & (0xFFu >> (n + 1));
  for (int q = 1; q < n; ++q) {
    const uint32_t c = text[j + q];
    if ((c & 0xC0u) != 0x80u) return ~0u;
    cp = (cp << 6) | (c & 0x3Fu);
  }
  return cp;
}
// byte `pos` (0 = lead) of code point cp's n-byte UTF-8 form
__device__ __forceinline__ uint32_t utf8_byte(uint32_t cp, int n, int pos) {
  if (pos == 0) return n == 2 ? (0xC0u | (cp >> 6)) : n == 3 ? (0xE0u | (cp >> 12)) : (0xF0u | (cp >> 18));
  return 0x80u | ((cp >> (6 * (n - 1 - pos))) & 0x3Fu);
}

// true when the lead byte at text[i] starts a character the kernel must reject (see the header)
__device__ __forceinline__ bool unsupported_at(const uint8_t* __restrict__ text, int64_t i, int64_t e) {
  const int n = utf8_len(text[i]);
  if (n < 2 || n > 3 || i + n > e) return false;  // ASCII, continuation, 4-byte, truncated: pass through
  const uint32_t cp = decode_at(text, i, n);
  return cp != ~0u && lower_bmp(cp) == 0u;
}

// output byte for input byte b = text[i] of the document [s, e) (same-length mappings only)
__device__ __forceinline__ uint32_t to_lower_at(const uint8_t* __restrict__ text, int64_t s, int64_t e, int64_t i,
                                                uint32_t b) {
  if (b < 0x80u) return (b >= 0x41u && b <= 0x5Au) ? b + 0x20u : b;  // ASCII: A–Z
  // the character holding byte i: its lead at i − pos (malformed sequences pass through unchanged)
  int pos = 0;
  int64_t j = i;
  while (utf8_len(text[j]) == 0) {
    if (pos == 3 || j == s) return b;
    --j;
    ++pos;
  }
  const int n = utf8_len(text[j]);
  if (n < 2 || pos >= n || j + n > e) return b;
  const uint32_t cp = decode_at(text, j, n);
  if (cp == ~0u) return b;
  const uint32_t lc = lower_cp(cp);
  return lc == 0u ? b : utf8_byte(lc, n, pos);
}

__device__ __forceinline__ int64_t lanes_below(uint64_t m, int lane) {
  return __popcll(m & ((lane ? (~0ull >> (64 - lane)) : 0ull)));
}

// pass 1: per document, token count and kept (non-separator) byte count; first bad byte position.
// Each lane reads one aligned dword (the caller pads the blob by >= 4 bytes), so a wave step covers
// 256 bytes; the four per-byte ballots give the separator count and the last kept byte.
__global__ __launch_bounds__(64 * kWaves) void k_count(const uint8_t* __restrict__ text,
                                                       const int64_t* __restrict__ text_off,
                                                       int64_t n_docs, int64_t* __restrict__ ntok,
                                                       int64_t* __restrict__ nkeep,
                                                       unsigned long long* __restrict__ bad) {
  const int lane = threadIdx.x & 63;
  for (int64_t d = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); d < n_docs;
       d += (int64_t)gridDim.x * kWaves) {
    const int64_t s = text_off[d], e = text_off[d + 1];
    int64_t seps = 0, last_keep = -1;
    for (int64_t c = s & ~int64_t(3); c < e; c += 256) {
      const int64_t w = c + 4 * lane;
      const uint32_t word = (w < e) ? *reinterpret_cast<const uint32_t*>(text + w) : 0x20202020u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t i = w + j;
        const bool in = i >= s && i < e;
        const uint32_t b = (word >> (8 * j)) & 0xFFu;
        const bool sep = is_java_space(b);
        if (in && b >= 0xC4u && unsupported_at(text, i, e)) atomicMin(bad, (unsigned long long)i);
        const uint64_t sm = __ballot(in && sep), km = __ballot(in && !sep);
        seps += __popcll(sm);
        if (km) {
          const int64_t lk = c + 4 * (63 - __clzll(km)) + j;
          last_keep = lk > last_keep ? lk : last_keep;
        }
      }
    }
    if (lane == 0) {
      const int64_t len = e - s;
      int64_t t;
      if (seps == 0) t = 1;                      // no match: the whole string ("" included)
      else if (last_keep < 0) t = 0;             // only separators: every piece is a trailing empty
      else t = seps + 1 - (e - 1 - last_keep);   // drop the trailing empty pieces
      ntok[d] = t;
      nkeep[d] = len - seps;
    }
  }
}

// pass 2: lower-case + compact the kept bytes, write each token's start
__global__ __launch_bounds__(64 * kWaves) void k_emit(const uint8_t* __restrict__ text,
                                                      const int64_t* __restrict__ text_off,
                                                      int64_t n_docs,
                                                      const int64_t* __restrict__ doc_off,
                                                      const int64_t* __restrict__ byte_off,
                                                      uint8_t* __restrict__ out,
                                                      int64_t* __restrict__ tok_off) {
  const int lane = threadIdx.x & 63;
  for (int64_t d = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); d < n_docs;
       d += (int64_t)gridDim.x * kWaves) {
    const int64_t s = text_off[d], e = text_off[d + 1];
    const int64_t base = byte_off[d], tb = doc_off[d], nt = doc_off[d + 1] - tb;
    if (nt > 0 && lane == 0) tok_off[tb] = base;
    int64_t seps = 0;
    for (int64_t c = s; c < e; c += 64) {
      const int64_t i = c + lane;
      const bool in = i < e;
      const uint32_t b = in ? text[i] : 0x20u;
      const bool sep = is_java_space(b);
      const uint64_t sm = __ballot(in && sep);
      const int64_t j = seps + lanes_below(sm, lane);  // separators before byte i in this doc
      if (in) {
        if (!sep) out[base + (i - s) - j] = (uint8_t)to_lower_at(text, s, e, i, b);
        else if (j + 1 < nt) tok_off[tb + j + 1] = base + (i - s) - j;
      }
      seps += __popcll(sm);
    }
  }
}

static int grid_docs(int64_t n_docs) {
  int64_t g = ceil_div(n_docs, kWaves);
  if (g < 1) g = 1;
  if (g > 256 * 32) g = 256 * 32;
  return (int)g;
}

void tokenize(Ctx& c, const uint8_t* d_text, const int64_t* d_text_off, int64_t n_docs,
              DevBuf& out_utf8, DevBuf& out_tok_off, DevBuf& out_doc_off, int64_t& n_tok,
              int64_t& n_out_bytes, int64_t& bad_pos) {
  hipStream_t s = c.stream;
  DevBuf cnt, keep, byte_off, badb, tmp;
  cnt.reserve(8 * (n_docs + 1));
  keep.reserve(8 * (n_docs + 1));
  byte_off.reserve(8 * (n_docs + 1));
  badb.reserve(8);
  out_doc_off.reserve(8 * (n_docs + 1));
  HIP_CHECK(hipMemsetAsync(cnt.p, 0, 8 * (n_docs + 1), s));
  HIP_CHECK(hipMemsetAsync(keep.p, 0, 8 * (n_docs + 1), s));
  HIP_CHECK(hipMemsetAsync(badb.p, 0xFF, 8, s));
  if (n_docs > 0) {
    k_count<<<grid_docs(n_docs), 64 * kWaves, 0, s>>>(d_text, d_text_off, n_docs, cnt.as<int64_t>(),
                                                      keep.as<int64_t>(), badb.as<unsigned long long>());
    KERNEL_CHECK();
  }
  size_t tb = 0;
  HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt.as<int64_t>(), out_doc_off.as<int64_t>(),
                                             (int)(n_docs + 1), s));
  tmp.reserve(tb);
  HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, cnt.as<int64_t>(), out_doc_off.as<int64_t>(),
                                             (int)(n_docs + 1), s));
  HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, keep.as<int64_t>(), byte_off.as<int64_t>(),
                                             (int)(n_docs + 1), s));
  int64_t h[3];
  HIP_CHECK(hipMemcpyAsync(&h[0], out_doc_off.as<int64_t>() + n_docs, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(&h[1], byte_off.as<int64_t>() + n_docs, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(&h[2], badb.p, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  n_tok = h[0];
  n_out_bytes = h[1];
  bad_pos = h[2];  // -1 (all ones) when every character is supported
  if (bad_pos >= 0) return;
  out_utf8.reserve(n_out_bytes + 16);  // k_hash reads whole aligned dwords past a token
  out_tok_off.reserve(8 * (n_tok + 1));
  if (n_docs > 0) {
    k_emit<<<grid_docs(n_docs), 64 * kWaves, 0, s>>>(d_text, d_text_off, n_docs,
                                                     out_doc_off.as<int64_t>(), byte_off.as<int64_t>(),
                                                     out_utf8.as<uint8_t>(), out_tok_off.as<int64_t>());
    KERNEL_CHECK();
  }
  HIP_CHECK(hipMemcpyAsync(out_tok_off.as<int64_t>() + n_tok, byte_off.as<int64_t>() + n_docs, 8,
                           hipMemcpyDeviceToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));  // scratch buffers die at scope exit
}

}  // namespace tokenizer
}  // namespace stc
