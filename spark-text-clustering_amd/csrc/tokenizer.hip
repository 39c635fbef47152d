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
// supplementary block in 6.2) inline, everything else passed through.  The 18 code points whose mapping is
// not a same-length 1:1 map are applied by rule: U+0130 İ → "i̇" (SpecialCasing, 2 → 3 bytes), U+03A3 Σ →
// ς or σ by the Final_Sigma context (a cased letter before it, case-ignorables between, and no cased
// letter after it past case-ignorables — classes from case_table.h's kSig tables), and 16 capitals whose
// lower case has another UTF-8 length (U+023A → U+2C65, ẞ → ß, Ω → ω, K → k, …).  Output byte positions
// shift by those characters' length changes: a wave-prefix over the rare lanes that hold one.
//
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

// the Final_Sigma class of cp: 0 other, 1 case-ignorable, 2 cased (case_table.h kSig*)
__device__ __forceinline__ int sigma_class(uint32_t cp) {
  const uint32_t pg = cp < 0x110000u ? kSigPage[cp >> 8] : 0u;
  return pg ? (kSigPages[pg - 1][(cp & 0xFFu) >> 2] >> (2 * (cp & 3u))) & 3 : 0;
}
// the code point of the character at text[j] (its length in *n), or ~0 when malformed / truncated at e
__device__ __forceinline__ uint32_t cp_at(const uint8_t* __restrict__ text, int64_t j, int64_t e, int* n) {
  const uint32_t b = text[j];
  *n = utf8_len(b);
  if (*n == 1) return b;
  if (*n == 0 || j + *n > e) {
    *n = 1;
    return ~0u;
  }
  return decode_at(text, j, *n);
}
// Final_Sigma for the Σ at text[i] (2 bytes) of the document [s, e): preceded by a cased letter with only
// case-ignorables between, and not followed by case-ignorables then a cased letter (the Unicode rule, as the
// oracle's str.lower() applies it).  A malformed byte ends a scan as a non-cased character.
// KNOWN DIVERGENCE from Spark's JVM (parity unpinned: no artefact or test of the reference holds it): Java
// 8's ConditionalSpecialCasing.isFinalCased scans the whole BreakIterator word instead, where letters AND
// digits belong to one word, so a digit between Σ and a cased letter changes the answer — "Α1Σ" gives Java
// ς but this rule σ, "ΑΣ1Β" Java σ but this rule ς.  Letters, marks, spaces and punctuation around Σ agree.
__device__ bool final_sigma(const uint8_t* __restrict__ text, int64_t s, int64_t e, int64_t i) {
  bool pre = false;
  for (int64_t j = i; j > s;) {  // backwards, one character at a time
    int64_t p = j - 1;
    while (p > s && j - p < 4 && (text[p] & 0xC0u) == 0x80u) --p;
    int n = 0;
    const uint32_t cp = cp_at(text, p, j, &n);
    if (cp == ~0u || p + n != j) break;
    const int c = sigma_class(cp);
    if (c == 1) {
      j = p;
      continue;
    }
    pre = c == 2;
    break;
  }
  if (!pre) return false;
  for (int64_t j = i + 2; j < e;) {
    int n = 0;
    const uint32_t cp = cp_at(text, j, e, &n);
    if (cp == ~0u) return true;
    const int c = sigma_class(cp);
    if (c != 1) return c != 2;
    j += n;
  }
  return true;
}
__device__ __forceinline__ int utf8_size(uint32_t cp) { return cp < 0x80u ? 1 : cp < 0x800u ? 2 : 3; }
// the lower case of a character the table leaves to rule (kCasePages entry 0): its UTF-8 bytes packed
// little-endian into *out, their count returned
__device__ int special_lower(const uint8_t* __restrict__ text, int64_t s, int64_t e, int64_t i, uint32_t cp,
                             uint32_t* out) {
  if (cp == 0x130u) {  // İ → i + U+0307 COMBINING DOT ABOVE
    *out = 0x69u | (0xCCu << 8) | (0x87u << 16);
    return 3;
  }
  uint32_t lc = cp;
  if (cp == 0x3A3u) {
    lc = final_sigma(text, s, e, i) ? 0x3C2u : 0x3C3u;
  } else {
    for (int q = 0; q < kSpecialN; ++q)
      if (kSpecialFrom[q] == cp) lc = kSpecialTo[q];
  }
  const int n = utf8_size(lc);
  uint32_t w = 0;
  for (int q = 0; q < n; ++q) w |= (n == 1 ? lc : utf8_byte(lc, n, q)) << (8 * q);
  *out = w;
  return n;
}
// the lead byte at text[i] (i < e) starts a character the table leaves to rule: its code point, else 0
__device__ __forceinline__ uint32_t special_at(const uint8_t* __restrict__ text, int64_t i, int64_t e) {
  const int n = utf8_len(text[i]);
  if (n < 2 || n > 3 || i + n > e) return 0u;
  const uint32_t cp = decode_at(text, i, n);
  return (cp != ~0u && lower_bmp(cp) == 0u) ? cp : 0u;
}
// its UTF-8 length change (Σ keeps its length; İ and U+023A / U+023E grow by one; the rest shrink)
__device__ __forceinline__ int special_delta(uint32_t cp, int n_in) {
  if (cp == 0x130u) return 1;
  if (cp == 0x3A3u) return 0;
  for (int q = 0; q < kSpecialN; ++q)
    if (kSpecialFrom[q] == cp) return utf8_size(kSpecialTo[q]) - n_in;
  return 0;
}

// output byte for input byte b = text[i] of the document [s, e) (same-length mappings); 0x100: the byte
// belongs to a character applied by rule, whose lead lane writes it
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
  return lc == 0u ? 0x100u : utf8_byte(lc, n, pos);
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
                                                       int64_t* __restrict__ nkeep) {
  const int lane = threadIdx.x & 63;
  for (int64_t d = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); d < n_docs;
       d += (int64_t)gridDim.x * kWaves) {
    const int64_t s = text_off[d], e = text_off[d + 1];
    int64_t seps = 0, last_keep = -1;
    int delta = 0;  // this lane's UTF-8 length changes (characters applied by rule)
    for (int64_t c = s & ~int64_t(3); c < e; c += 256) {
      const int64_t w = c + 4 * lane;
      const uint32_t word = (w < e) ? *reinterpret_cast<const uint32_t*>(text + w) : 0x20202020u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t i = w + j;
        const bool in = i >= s && i < e;
        const uint32_t b = (word >> (8 * j)) & 0xFFu;
        const bool sep = is_java_space(b);
        if (in && b >= 0xC4u) {
          const uint32_t cp = special_at(text, i, e);
          if (cp) delta += special_delta(cp, utf8_len(b));
        }
        const uint64_t sm = __ballot(in && sep), km = __ballot(in && !sep);
        seps += __popcll(sm);
        if (km) {
          const int64_t lk = c + 4 * (63 - __clzll(km)) + j;
          last_keep = lk > last_keep ? lk : last_keep;
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) delta += __shfl_xor(delta, o, 64);
    if (lane == 0) {
      const int64_t len = e - s;
      int64_t t;
      if (seps == 0) t = 1;                      // no match: the whole string ("" included)
      else if (last_keep < 0) t = 0;             // only separators: every piece is a trailing empty
      else t = seps + 1 - (e - 1 - last_keep);   // drop the trailing empty pieces
      ntok[d] = t;
      nkeep[d] = len - seps + delta;
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
    int64_t seps = 0, shift = 0;  // separators, and length changes of rule-applied characters, so far
    for (int64_t c = s; c < e; c += 64) {
      const int64_t i = c + lane;
      const bool in = i < e;
      const uint32_t b = in ? text[i] : 0x20u;
      const bool sep = is_java_space(b);
      const uint64_t sm = __ballot(in && sep);
      const int64_t j = seps + lanes_below(sm, lane);  // separators before byte i in this doc
      // a character applied by rule starting at byte i: its lane writes all of its output bytes
      uint32_t sp = 0, sw = 0;
      int sn = 0, dl = 0;
      if (in && b >= 0xC4u) {
        sp = special_at(text, i, e);
        if (sp) {
          sn = special_lower(text, s, e, i, sp, &sw);
          dl = sn - utf8_len(b);
        }
      }
      int64_t pre = shift;  // length changes of the characters before byte i
      if (__ballot(dl != 0) != 0) {  // rare: an inclusive lane scan of the changes
        int x = dl;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(x, o, 64);
          if (lane >= o) x += y;
        }
        pre += x - dl;
        shift += __shfl(x, 63, 64);
      }
      if (in) {
        const int64_t o = base + (i - s) - j + pre;
        if (sp) {
          for (int q = 0; q < sn; ++q) out[o + q] = (uint8_t)(sw >> (8 * q));
        } else if (!sep) {
          const uint32_t lb = to_lower_at(text, s, e, i, b);
          if (lb < 0x100u) out[o] = (uint8_t)lb;
        } else if (j + 1 < nt) {
          tok_off[tb + j + 1] = o;
        }
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
              int64_t& n_out_bytes) {
  hipStream_t s = c.stream;
  DevBuf cnt, keep, byte_off, tmp;
  cnt.reserve(8 * (n_docs + 1));
  keep.reserve(8 * (n_docs + 1));
  byte_off.reserve(8 * (n_docs + 1));
  out_doc_off.reserve(8 * (n_docs + 1));
  HIP_CHECK(hipMemsetAsync(cnt.p, 0, 8 * (n_docs + 1), s));
  HIP_CHECK(hipMemsetAsync(keep.p, 0, 8 * (n_docs + 1), s));
  if (n_docs > 0) {
    k_count<<<grid_docs(n_docs), 64 * kWaves, 0, s>>>(d_text, d_text_off, n_docs, cnt.as<int64_t>(),
                                                      keep.as<int64_t>());
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
  int64_t h[2];
  HIP_CHECK(hipMemcpyAsync(&h[0], out_doc_off.as<int64_t>() + n_docs, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(&h[1], byte_off.as<int64_t>() + n_docs, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  n_tok = h[0];
  n_out_bytes = h[1];
  out_utf8.reserve(n_out_bytes + kHashPad);  // the hash reads 32-byte windows of whole aligned dwords
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
