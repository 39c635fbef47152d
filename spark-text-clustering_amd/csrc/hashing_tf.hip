// hashing_tf.hip — K1 (MurmurHash3_x86_32 + nonNegativeMod) and K2 (per-document bucket
// counting into a sorted CSR) for gfx950.
//
// Replaces [U] mllib.feature.HashingTF.transform / murmur3Hash (Spark 2.4.3, build.sbt:10), i.e.
// the reference's vocab-indexed counting slot LDAClustering.scala:154-167.  Bit-exact.
//
// Layout: the corpus arrives as ONE UTF-8 byte blob + int64 token offsets + int64 doc offsets
// (plain arrays a JNI caller can hand over without per-string objects).  One wave per document hashes
// its tokens (K1, aligned dword reads) straight into registers and sorts them there (K2 pass A; hipcub's
// segmented sort only for documents past 1024 tokens, hashed to memory first); pass B emits the sorted
// distinct ids + run lengths — no atomics on the CSR, so hot terms ("the") cost nothing extra.
#include <hipcub/hipcub.hpp>

#include <map>
#include <mutex>

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

// MurmurHash3_x86_32(seed 42) of n bytes at p.  SPARK24 = Spark 2.4 hashUnsafeBytes (each tail
// byte sign-extended and mixed as a block); otherwise the standard tail (Spark 3 hashUnsafeBytes2).
// The bytes are read as whole aligned dwords and realigned with v_alignbyte (a byte load per character
// was the kernel's issue bottleneck).  Round 4: the first 8 dwords of a token arrive as one window of
// two 16-byte loads issued together (load_win, before the hash needs them) — tokens of ≤ 27 bytes hash
// from registers with no dependent load; longer ones read their remaining dwords one by one.  The
// buffers carry ≥ kHashPad bytes of padding, so a window never leaves the allocation.
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
struct Win {
  u32x4a lo, hi;
};
__device__ __forceinline__ Win load_win(const uint8_t* p) {
  // (pointer arithmetic, not an integer round trip: the loads stay global_load, not flat_load)
  const u32x4a* w = reinterpret_cast<const u32x4a*>(p - (reinterpret_cast<uintptr_t>(p) & 3));
  return Win{w[0], w[1]};
}

template <bool SPARK24>
__device__ __forceinline__ int32_t murmur3_win(const uint8_t* p, uint32_t n, const Win& W) {
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p - sh);
  const uint32_t d[8] = {W.lo.x, W.lo.y, W.lo.z, W.lo.w, W.hi.x, W.hi.y, W.hi.z, W.hi.w};
  uint32_t h1 = 42u;
  const uint32_t nb = n & ~3u;
#pragma unroll
  for (uint32_t k = 0; k < 7; ++k)  // blocks inside the window (bytes 4k..4k+3 use dwords k, k+1)
    if (4 * k + 4 <= nb) h1 = mix_h1(h1, mix_k1(__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh)));
  for (uint32_t i = 28; i < nb; i += 4)  // past the window
    h1 = mix_h1(h1, mix_k1(__builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], sh)));
  const uint32_t tail = n - nb;
  if (tail) {
    const uint32_t kk = nb >> 2;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t k = 0; k < 7; ++k)
      if (kk == k) {
        lo = d[k];
        hi = d[k + 1];
      }
    if (kk >= 7) {
      lo = w[kk];
      hi = w[kk + 1];
    }
    const uint32_t t = __builtin_amdgcn_alignbyte(hi, lo, sh);  // bytes nb.. in order
    if (SPARK24) {
#pragma unroll
      for (uint32_t i = 0; i < 3; ++i)
        if (i < tail) h1 = mix_h1(h1, mix_k1((uint32_t)(int32_t)(int8_t)(t >> (8 * i))));
    } else {
      h1 ^= mix_k1(t & (0xFFFFFFFFu >> (8 * (4 - tail))));
    }
  }
  return (int32_t)fmix(h1, n);
}
template <bool SPARK24>
__device__ __forceinline__ int32_t murmur3(const uint8_t* p, uint32_t n) {
  return murmur3_win<SPARK24>(p, n, load_win(p));
}

// four tokens per thread and step, a grid stride apart (neighbouring lanes keep neighbouring tokens,
// so the byte loads stay coalesced) — four independent offset → window → hash chains in flight, every
// window issued before the first hash
template <bool SPARK24, typename O>
__global__ __launch_bounds__(256) void k_hash(const uint8_t* __restrict__ utf8,
                                              const O* __restrict__ tok_off, int64_t n_tok,
                                              int32_t num_features, int32_t* __restrict__ out) {
  const int64_t S = (int64_t)gridDim.x * 256;
  for (int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x; t0 < n_tok; t0 += 4 * S) {
    O b[4], e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t t = t0 + q * S < n_tok ? t0 + q * S : n_tok - 1;
      b[q] = tok_off[t];
      e[q] = tok_off[t + 1];
    }
    Win w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = load_win(utf8 + b[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int32_t h = murmur3_win<SPARK24>(utf8 + b[q], (uint32_t)(e[q] - b[q]), w[q]);
      if (t0 + q * S < n_tok) {
        const int32_t raw = h % num_features;  // Utils.nonNegativeMod (Java % truncates toward zero)
        out[t0 + q * S] = raw + (raw < 0 ? num_features : 0);
      }
    }
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
  const int g = grid_for(ceil_div(n_tok, (int64_t)4), 256, 256 * 32);
  if (variant == STC_HASH_SPARK24)
    k_hash<true><<<g, 256, 0, c.stream>>>(d_utf8, d_tok_off, n_tok, num_features, d_idx);
  else
    k_hash<false><<<g, 256, 0, c.stream>>>(d_utf8, d_tok_off, n_tok, num_features, d_idx);
  KERNEL_CHECK();
}
template <typename O>
static void hash_tokens_t(Ctx& c, const uint8_t* d_utf8, const O* d_tok_off, int64_t n_tok, int32_t num_features,
                          int variant, int32_t* d_idx) {
  const int g = grid_for(ceil_div(n_tok, (int64_t)4), 256, 256 * 32);
  if (variant == STC_HASH_SPARK24)
    k_hash<true><<<g, 256, 0, c.stream>>>(d_utf8, d_tok_off, n_tok, num_features, d_idx);
  else
    k_hash<false><<<g, 256, 0, c.stream>>>(d_utf8, d_tok_off, n_tok, num_features, d_idx);
  KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------
// K2: per-document sort + run-length count → CSR.  One wave per document.
//  pass A (k_doc_hash_sort, then k_doc_sort for 257–1024 tokens): documents of ≤ kSortCap tokens are
//    bitonic-sorted in registers (≤ 256 tokens hashed straight into them) (P = m/64 keys per lane, m = the next power of two ≥ max(n, 64); partners
//    j ≥ P across lanes by __shfl_xor, j < P inside the lane), written back sorted, and their distinct
//    ids counted into nnz[d].  Longer documents are hashed to memory and appended to a list for the
//    segmented radix sort (hipcub), then counted by k_doc_runs<COUNT>.
//  scan nnz → indptr; pass B (k_doc_runs<EMIT>): each document's sorted keys in 64-key chunks; run
//    heads by ballot, output slots by mbcnt, run lengths from the next head in the chunk, or, for a
//    chunk's last run, when the next chunk's first head (or the document end) arrives.
// No atomics on the output; the large-document list is an atomic append whose order only permutes
// hipcub's segments, so the CSR is bit-identical run to run.
// ---------------------------------------------------------------------------------------
constexpr int kSortCap = 1024;  // ≤ 16 keys per lane
#ifndef TF_DPP
#define TF_DPP 1  // the sort's cross-lane exchanges by DPP / swizzle (0: ds_bpermute throughout)
#endif

// x from lane ^ lx without the LDS crossbar where a DPP pattern exists (round 4: every shuffle of the
// network was a ds_bpermute, ~60 % of the sort): xor 1 / 2 quad_perm, xor 4 = half-row mirror (xor 7)
// after quad_perm xor 3, xor 8 = row rotate by 8; xor 16 ds_swizzle (no address VGPR); xor 32 bpermute.
__device__ __forceinline__ int32_t shfl_xor_dpp(int32_t v, int lx) {
  switch (lx) {
    case 1: return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    case 2: return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    case 4: return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(v, 0x1B, 0xF, 0xF, false),  // [3,2,1,0]
                                            0x141, 0xF, 0xF, false);     // row_half_mirror
    case 8: return __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);  // row_ror:8
    case 16: return __builtin_amdgcn_ds_swizzle(v, 0x401F);              // and 0x1F, xor 0x10
    default: return __shfl_xor(v, lx, 64);
  }
}

// Σ over the wave of a per-lane count in [0, P] from bit-sliced ballots (scalar popcounts, no shuffles)
template <int P>
__device__ __forceinline__ int wave_sum_small(int v) {
  int tot = 0;
#pragma unroll
  for (int b = 0; (1 << b) <= P; ++b) tot += __popcll(__ballot((v >> b) & 1)) << b;
  return tot;
}
// the exclusive prefix of such a count over the lanes below this one
template <int P>
__device__ __forceinline__ int wave_excl_small(int v) {
  int pre = 0;
#pragma unroll
  for (int b = 0; (1 << b) <= P; ++b) {
    const uint64_t m = __ballot((v >> b) & 1);
    pre += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
  }
  return pre;
}

template <int P>
__device__ __forceinline__ void bitonic_regs(int32_t (&x)[P], int lane) {
  constexpr int m = 64 * P;  // fully unrolled: every partner distance is a constant
#pragma unroll
  for (int k = 2; k <= m; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= P) {  // partner in lane ^ (j / P), same register
        const int lx = j / P;
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const int e = lane * P + p;
          const int32_t o = TF_DPP ? shfl_xor_dpp(x[p], lx) : __shfl_xor(x[p], lx, 64);
          const bool lower = (e & j) == 0, asc = (e & k) == 0;
          x[p] = (lower == asc) ? min(x[p], o) : max(x[p], o);
        }
      } else {
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const int q = p ^ j;
          if (q > p) {
            const int e = lane * P + p;
            const bool asc = (e & k) == 0;
            const int32_t a = x[p], b = x[q];
            x[p] = asc ? min(a, b) : max(a, b);
            x[q] = asc ? max(a, b) : min(a, b);
          }
        }
      }
    }
  }
}

template <int P>
__device__ __forceinline__ int64_t sort_doc(const int32_t* __restrict__ keys, int32_t* __restrict__ sorted,
                                            int64_t s, int n, int lane) {
  int32_t x[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int e = lane * P + p;
    x[p] = e < n ? keys[s + e] : INT32_MAX;  // pads sort last (bucket ids < numFeatures ≤ 2^31 − 1)
  }
  bitonic_regs<P>(x, lane);
  const int32_t prev_last = __shfl_up(x[P - 1], 1, 64);
  int heads = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int e = lane * P + p;
    if (e < n) {
      sorted[s + e] = x[p];
      const int32_t prev = p == 0 ? prev_last : x[p - 1];
      heads += (e == 0 || x[p] != prev) ? 1 : 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) heads += __shfl_xor(heads, o, 64);
  return heads;
}

constexpr int kDocWaves = 4;  // documents in flight per workgroup (one per wave)
constexpr int kFusedCap = 256;  // documents up to this many tokens are hashed and sorted in one pass

// K1 fused into K2's pass A: the document's bucket ids never round-trip through HBM.  Token p·64 + lane
// of the document goes to register p of the lane (coalesced offset and byte loads; the bitonic network
// sorts any starting order), is hashed there, and the P registers are sorted and their distinct ids
// counted exactly as sort_doc does.
template <bool SPARK24, int P, typename O>
__device__ __forceinline__ int hash_sort_regs(const uint8_t* __restrict__ utf8, const O* __restrict__ tok_off,
                                              int64_t s, int n, int32_t nf, int32_t (&x)[P], int lane) {
  O b[P], e[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int q = p * 64 + lane;
    b[p] = q < n ? tok_off[s + q] : 0;
    e[p] = q < n ? tok_off[s + q + 1] : 0;
  }
  Win cur = load_win(utf8 + b[0]);  // pad lanes read the blob's first bytes (b = 0), unused
#pragma unroll
  for (int p = 0; p < P; ++p) {
    Win nxt;
    if (p + 1 < P) nxt = load_win(utf8 + b[p + 1]);  // the next token's window in flight while this one hashes
    const int q = p * 64 + lane;
    if (q < n) {
      const int32_t raw = murmur3_win<SPARK24>(utf8 + b[p], (uint32_t)(e[p] - b[p]), cur) % nf;  // Utils.nonNegativeMod
      x[p] = raw + (raw < 0 ? nf : 0);
    } else {
      x[p] = INT32_MAX;  // pads sort last
    }
    if (p + 1 < P) cur = nxt;
  }
  bitonic_regs<P>(x, lane);
  const int32_t prev_last = __shfl_up(x[P - 1], 1, 64);
  int heads = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int q = lane * P + p;
    const int32_t prev = p == 0 ? prev_last : x[p - 1];
    heads += (q < n && (q == 0 || x[p] != prev)) ? 1 : 0;
  }
  return wave_sum_small<P>(heads);  // distinct ids (wave total)
}

// the same from bucket ids already hashed into `keys` (token order): load, sort, count distinct
template <int P>
__device__ __forceinline__ int keys_sort_regs(const int32_t* __restrict__ keys, int64_t s, int n, int32_t (&x)[P],
                                              int lane) {
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int q = p * 64 + lane;
    x[p] = q < n ? keys[s + q] : INT32_MAX;  // pads sort last
  }
  bitonic_regs<P>(x, lane);
  const int32_t prev_last = __shfl_up(x[P - 1], 1, 64);
  int heads = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int q = lane * P + p;
    const int32_t prev = p == 0 ? prev_last : x[p - 1];
    heads += (q < n && (q == 0 || x[p] != prev)) ? 1 : 0;
  }
  return wave_sum_small<P>(heads);
}

template <bool SPARK24, int P, typename O>
__device__ __forceinline__ int64_t hash_sort_doc(const uint8_t* __restrict__ utf8, const O* __restrict__ tok_off,
                                                 int64_t s, int n, int32_t nf, int32_t* __restrict__ sorted,
                                                 int lane) {
  int32_t x[P];
  const int heads = hash_sort_regs<SPARK24, P, O>(utf8, tok_off, s, n, nf, x, lane);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int q = lane * P + p;
    if (q < n) sorted[s + q] = x[p];
  }
  return heads;
}

// one wave per document: ≤ kFusedCap tokens hashed, sorted and counted in registers (nnz[d]); longer
// documents hashed into `keys` — ≤ kSortCap tokens for k_doc_sort (counted in *n_medium), the rest for the
// segmented radix sort (appended to `large`).  Capping the fused path at 4 keys per lane keeps the kernel
// at ~50 VGPRs: the hashing's dependent offset → byte loads need the occupancy (the P = 16 form held 132).
template <bool SPARK24, typename O>
__global__ __launch_bounds__(64 * kDocWaves, 8) void k_doc_hash_sort(const uint8_t* __restrict__ utf8,
                                                                 const O* __restrict__ tok_off,
                                                                 const int64_t* __restrict__ doc_off, int64_t n_docs,
                                                                 int32_t nf, int32_t* __restrict__ keys,
                                                                 int32_t* __restrict__ sorted,
                                                                 int64_t* __restrict__ nnz, int32_t* __restrict__ large,
                                                                 int32_t* __restrict__ n_large,
                                                                 int32_t* __restrict__ n_medium) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar doc_off loads
  for (int64_t d = (int64_t)blockIdx.x * kDocWaves + wv; d < n_docs; d += (int64_t)gridDim.x * kDocWaves) {
    const int64_t s = doc_off[d], n64 = doc_off[d + 1] - s;
    if (n64 > kFusedCap) {
      for (int64_t q = lane; q < n64; q += 64) {
        const int64_t t = s + q;
        const int32_t raw = murmur3<SPARK24>(utf8 + tok_off[t], (uint32_t)(tok_off[t + 1] - tok_off[t])) % nf;
        keys[t] = raw + (raw < 0 ? nf : 0);
      }
      if (lane == 0) {
        if (n64 > kSortCap) large[atomicAdd(n_large, 1)] = (int32_t)d;
        else atomicAdd(n_medium, 1);
      }
      continue;
    }
    const int n = (int)n64;
    int64_t h = 0;
    if (n <= 64) h = hash_sort_doc<SPARK24, 1, O>(utf8, tok_off, s, n, nf, sorted, lane);
    else if (n <= 128) h = hash_sort_doc<SPARK24, 2, O>(utf8, tok_off, s, n, nf, sorted, lane);
    else h = hash_sort_doc<SPARK24, 4, O>(utf8, tok_off, s, n, nf, sorted, lane);
    if (lane == 0) nnz[d] = h;
  }
}

// ---- single pass (round 4) for corpora whose documents all hold ≤ kFusedCap tokens (known at upload):
// hash + register sort + CSR emission in one kernel, the row offsets from a decoupled look-back over
// tiles of kDocWaves documents — no sorted-key array, no nnz scan, no second pass over the keys.
// Workgroups take tiles in ticket order — eight counters, one per XCD, counter c handing out tiles
// c, c + 8, … in order — so every tile a look-back waits on is held by a running workgroup, or is the
// next one its counter hands out to a workgroup whose own look-back waits only on lower tiles (the
// lowest unpublished tile always makes progress): no dependence on dispatch order or residency.  A look-back that waits past its poll bound sets the fault word; the host then rebuilds
// the CSR with the sorted-key passes (mode 0).  Measured without gain: batching tickets (2–8 consecutive
// tiles per atomic: 1.2× to 300× slower, a batch's later tiles publish their counts an iteration late)
// and a static tile order over a resident grid (tile = step·grid + blockIdx: 2.89 vs 2.11 ms, a slow
// workgroup stalls every later tile; and with the flat-hash mode the grid was not all resident).  status[t] = flag << 62 | value
// (flag 1: the tile's own entry count, 2: the inclusive count of tiles 0..t), written by one lane with
// agent-scope atomic stores and read with agent-scope atomic loads (vector memory, L2-coherent).
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbVal = kLbAgg - 1;
// the ticket counters: one per XCD, each on its own 128-byte line (one word takes ≈ 88 returning atomics
// per µs — MI355X_MICROARCH.md "dequeue" — against 125 k tiles per launch at config 2)
constexpr int kTicketPitch = 16;                       // u64 words between counters
constexpr int kTicketWords = kTicketPitch * 9;         // fault word's line + 8 counters

// the exclusive entry count before `tile` (wave 0 of the workgroup; every lane returns it)
// A bounded wait: a predecessor silent for ~2^20 polls (far beyond any tile's run time) sets *fault and the
// look-back ends, so the grid always drains; the host then fails the call (STC_ERR_HIP).
constexpr int kLbMaxPolls = 1 << 20;

// publish a tile's own entry count (tile 0: its inclusive count) — never waits
__device__ __forceinline__ void tile_publish(uint64_t* status, int64_t tile, int64_t agg) {
  __hip_atomic_store(&status[tile], (tile == 0 ? kLbInc : kLbAgg) | (uint64_t)agg, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// the exclusive entry count before `tile` (one wave; every lane returns it), then the tile's inclusive
// count published.  Waits only for predecessors' own counts, which tile_publish writes unconditionally.
__device__ __forceinline__ int64_t tile_lookback(uint64_t* status, int64_t tile, int64_t agg, int lane,
                                                 uint64_t* fault, int max_polls) {
  if (tile == 0) return 0;
  int64_t excl = 0;
  for (int64_t j = tile - 1;; j -= 64) {  // a window of 64 predecessors, closest in lane 0
    const int64_t k = j - lane;
    uint64_t v = k >= 0 ? __hip_atomic_load(&status[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbInc;
    for (int polls = 0; __ballot((v >> 62) == 0); ++polls) {  // a predecessor not yet published: it is running
      if (polls >= max_polls) {
        if (lane == 0) __hip_atomic_store(fault, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v = kLbInc;  // give up (the output is discarded)
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      if ((v >> 62) == 0) v = __hip_atomic_load(&status[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint64_t inc = __ballot((v >> 62) == 2);
    const int lp = inc ? __ffsll((unsigned long long)inc) - 1 : 63;  // the closest inclusive count
    int64_t sum = lane <= lp ? (int64_t)(v & kLbVal) : 0;
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    excl += sum;
    if (inc) break;
  }
  if (lane == 0) __hip_atomic_store(&status[tile], kLbInc | (uint64_t)(excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// one document's sorted keys (x[p] = element lane·P + p) → its distinct ids and run lengths at out0
template <int P, typename V>
__device__ __forceinline__ void emit_runs(const int32_t (&x)[4], int n, int lane, int64_t out0, int binary,
                                          int32_t* __restrict__ idx, V* __restrict__ vals) {
  const int32_t prev_last = __shfl_up(x[P - 1], 1, 64);
  bool hd[P];
  int hc = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int q = lane * P + p;
    const int32_t prev = p == 0 ? prev_last : x[p - 1];
    hd[p] = q < n && (q == 0 || x[p] != prev);
    hc += hd[p] ? 1 : 0;
  }
  const int excl = wave_excl_small<P>(hc);  // head slots before this lane
  int first = n;  // this lane's first head position
#pragma unroll
  for (int p = P - 1; p >= 0; --p)
    if (hd[p]) first = lane * P + p;
  // the first head after this lane: the next lane holding one (ballot), its `first`
  const uint64_t has = __ballot(hc > 0);
  const uint64_t after = lane == 63 ? 0ull : has >> (lane + 1);
  const int nl = after ? lane + 1 + __builtin_ctzll(after) : lane;
  const int nf = __shfl(first, nl, 64);
  int nx = after ? nf : n;
  int nxt[P];
#pragma unroll
  for (int p = P - 1; p >= 0; --p) {
    nxt[p] = nx;
    if (hd[p]) nx = lane * P + p;
  }
  int64_t r = out0 + excl;
#pragma unroll
  for (int p = 0; p < P; ++p)
    if (hd[p]) {
      idx[r] = x[p];
      vals[r] = binary ? V(1) : V(nxt[p] - (lane * P + p));
      ++r;
    }
}

// Pipelined one tile deep: a workgroup publishes tile t's count as soon as its documents are sorted, hashes
// and sorts its next tile, and only then resolves t's offset and emits t — by then t's predecessors have
// published, so the look-back seldom waits (the unpipelined form idled ~40 % of the time there).
#ifndef TF_EMIT_OCC
#define TF_EMIT_OCC 7  // waves per SIMD: 72 VGPRs; 8 spills two
#endif
#ifndef TF_EMIT_WAVES
#define TF_EMIT_WAVES 8  // documents per tile (one per wave): one ticket and one look-back per tile (4: +30 %)
#endif
constexpr int kEmitWaves = TF_EMIT_WAVES;

template <int P>
__device__ __forceinline__ void take(int32_t (&x)[4], const int32_t (&xp)[P]) {
#pragma unroll
  for (int p = 0; p < P; ++p) x[p] = xp[p];
}

template <bool SPARK24, bool KEYS, typename V, typename O>
__global__ __launch_bounds__(64 * kEmitWaves, TF_EMIT_OCC) void k_doc_hash_emit(
    const int32_t* __restrict__ keys /* KEYS: the hashed ids, token order */,
    const uint8_t* __restrict__ utf8, const O* __restrict__ tok_off, const int64_t* __restrict__ doc_off,
    int64_t n_docs, int32_t nf, int binary, int64_t* __restrict__ indptr, int32_t* __restrict__ idx,
    V* __restrict__ vals, uint64_t* __restrict__ status, unsigned long long* __restrict__ ticket, int max_polls) {
  __shared__ int tile_s;
  __shared__ int wn[kEmitWaves];
  __shared__ int64_t base_s;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tiles = (n_docs + kEmitWaves - 1) / kEmitWaves;
  // the previous tile, sorted and published, awaiting its offset
  int64_t tp = -1;
  int32_t xq[4];
  int nq = 0, hq = 0, preq = 0, aggq = 0;
  for (;;) {
    if (threadIdx.x == 0)  // counter c hands out tiles c, c + 8, … (one counter per XCD: blockIdx % 8)
      tile_s = (int)(atomicAdd(ticket + kTicketPitch * (blockIdx.x & 7), 1ull) * 8 + (blockIdx.x & 7));
    __syncthreads();
    const int64_t tile = __builtin_amdgcn_readfirstlane(tile_s);
    const bool have = tile < tiles;  // the tickets only grow: once past the end, the loop drains tp and exits
    if (!have && tp < 0) break;
    int32_t x[4] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MAX};
    int n = 0, h = 0, pre = 0, agg = 0;
    if (have) {
      const int64_t d = tile * kEmitWaves + wv;
      if (d < n_docs) {
        const int64_t s = doc_off[d];
        n = (int)(doc_off[d + 1] - s);
        if (n <= 64) {
          int32_t xp[1];
          h = KEYS ? keys_sort_regs<1>(keys, s, n, xp, lane) : hash_sort_regs<SPARK24, 1, O>(utf8, tok_off, s, n, nf, xp, lane);
          take<1>(x, xp);
        } else if (n <= 128) {
          int32_t xp[2];
          h = KEYS ? keys_sort_regs<2>(keys, s, n, xp, lane) : hash_sort_regs<SPARK24, 2, O>(utf8, tok_off, s, n, nf, xp, lane);
          take<2>(x, xp);
        } else {
          int32_t xp[4];
          h = KEYS ? keys_sort_regs<4>(keys, s, n, xp, lane) : hash_sort_regs<SPARK24, 4, O>(utf8, tok_off, s, n, nf, xp, lane);
          take<4>(x, xp);
        }
      }
      if (lane == 0) wn[wv] = h;
    }
    __syncthreads();
    if (have) {
#pragma unroll
      for (int w = 0; w < kEmitWaves; ++w) {
        const int c = wn[w];
        pre += w < wv ? c : 0;
        agg += c;
      }
      if (threadIdx.x == 0) tile_publish(status, tile, agg);
    }
    if (tp >= 0) {
      if (wv == 0) {
        const int64_t ex = tile_lookback(status, tp, aggq, lane, status + tiles, max_polls);
        if (lane == 0) base_s = ex;
      }
      __syncthreads();
      const int64_t d = tp * kEmitWaves + wv;
      if (d < n_docs) {
        const int64_t out0 = base_s + preq;
        if (nq <= 64) emit_runs<1, V>(xq, nq, lane, out0, binary, idx, vals);
        else if (nq <= 128) emit_runs<2, V>(xq, nq, lane, out0, binary, idx, vals);
        else emit_runs<4, V>(xq, nq, lane, out0, binary, idx, vals);
        if (lane == 0) indptr[d + 1] = out0 + hq;
      }
    }
    tp = have ? tile : -1;
#pragma unroll
    for (int p = 0; p < 4; ++p) xq[p] = x[p];
    nq = n;
    hq = h;
    preq = pre;
    aggq = agg;
  }
}

// the documents of kFusedCap < n ≤ kSortCap tokens, hashed by k_doc_hash_sort: sorted in registers from
// `keys` (8 or 16 keys per lane) and counted
__global__ __launch_bounds__(64 * kDocWaves) void k_doc_sort(const int32_t* __restrict__ keys,
                                                            const int64_t* __restrict__ doc_off, int64_t n_docs,
                                                            int32_t* __restrict__ sorted, int64_t* __restrict__ nnz) {
  const int lane = threadIdx.x & 63;
  for (int64_t d = (int64_t)blockIdx.x * kDocWaves + (threadIdx.x >> 6); d < n_docs;
       d += (int64_t)gridDim.x * kDocWaves) {
    const int64_t s = doc_off[d], n64 = doc_off[d + 1] - s;
    if (n64 <= kFusedCap || n64 > kSortCap) continue;
    const int n = (int)n64;
    const int64_t h = n <= 512 ? sort_doc<8>(keys, sorted, s, n, lane) : sort_doc<16>(keys, sorted, s, n, lane);
    if (lane == 0) nnz[d] = h;
  }
}

// segment bounds of the listed long documents (for hipcub's segmented sort) and their flags
__global__ __launch_bounds__(256) void k_large_segments(const int32_t* __restrict__ large, int32_t n_large,
                                                        const int64_t* __restrict__ doc_off,
                                                        int64_t* __restrict__ beg, int64_t* __restrict__ end,
                                                        uint8_t* __restrict__ is_large) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n_large) {
    const int32_t d = large[i];
    beg[i] = doc_off[d];
    end[i] = doc_off[d + 1];
    is_large[d] = 1;
  }
}

// the runs of one document's sorted keys, 64 at a time: COUNT → nnz[d]; EMIT → ids + run lengths at
// indptr[d] (the value is 1 when binary)
template <bool EMIT, typename V>
__device__ __forceinline__ void doc_runs(const int32_t* __restrict__ src, int64_t s, int64_t n, int lane,
                                         int64_t out0, int binary, int32_t* __restrict__ idx,
                                         V* __restrict__ vals, int64_t* nnz_out) {
  int64_t done = 0;                  // runs started so far (wave-uniform)
  int64_t pend_start = -1, pend_slot = 0;
  int32_t last = 0;                  // the previous chunk's last key
  int32_t key_n = lane < n ? src[s + lane] : 0;  // one chunk ahead: its load overlaps this chunk's work
  for (int64_t c0 = 0; c0 < n; c0 += 64) {
    const int64_t i = c0 + lane;
    const bool valid = i < n;
    const int32_t key = key_n;
    if (c0 + 64 < n) key_n = i + 64 < n ? src[s + i + 64] : 0;
    int32_t prev = __shfl_up(key, 1, 64);
    if (lane == 0) prev = last;
    const bool head = valid && (i == 0 || key != prev);
    const uint64_t mask = __ballot(head);
    const int nh = __popcll(mask);
    if (EMIT) {
      if (mask != 0 && pend_start >= 0 && lane == 0)  // the open run ends at this chunk's first head
        vals[out0 + pend_slot] = binary ? V(1) : V(c0 + __ffsll((unsigned long long)mask) - 1 - pend_start);
      if (head) {
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        const int64_t slot = done + rank;
        idx[out0 + slot] = key;
        const uint64_t after = lane == 63 ? 0ull : (mask >> (lane + 1));
        if (after) vals[out0 + slot] = binary ? V(1) : V(__ffsll((unsigned long long)after));
      }
      if (mask != 0) {
        const int lh = 63 - __clzll((long long)mask);
        pend_start = c0 + lh;
        pend_slot = done + nh - 1;
      }
    }
    done += nh;
    last = __shfl(key, 63, 64);
  }
  if (EMIT) {
    if (pend_start >= 0 && lane == 0) vals[out0 + pend_slot] = binary ? V(1) : V(n - pend_start);
  } else if (lane == 0) {
    *nnz_out = done;
  }
}

template <bool EMIT, typename V>
__global__ __launch_bounds__(64 * kDocWaves) void k_doc_runs(const int32_t* __restrict__ sorted,
                                                 const int32_t* __restrict__ sorted_l,
                                                 const uint8_t* __restrict__ is_large,
                                                 const int32_t* __restrict__ large, int32_t n_large,
                                                 const int64_t* __restrict__ doc_off, int64_t n_docs,
                                                 const int64_t* __restrict__ indptr, int binary,
                                                 int32_t* __restrict__ idx, V* __restrict__ vals,
                                                 int64_t* __restrict__ nnz) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar offset loads
  const int64_t count = EMIT ? n_docs : n_large;  // COUNT runs over the long documents only
  for (int64_t w = (int64_t)blockIdx.x * kDocWaves + wv; w < count; w += (int64_t)gridDim.x * kDocWaves) {
    const int64_t d = EMIT ? w : large[w];
    const int64_t s = doc_off[d], n = doc_off[d + 1] - s;
    const int32_t* src = (is_large && is_large[d]) ? sorted_l : sorted;
    doc_runs<EMIT, V>(src, s, n, lane, EMIT ? indptr[d] : 0, binary, idx, vals, nnz + d);
  }
}

// order[s + i] = the in-row position of row d's i-th rarest term (df ascending, ties by position):
// the E-step row order of lda_wide.hip.  Rows past kSortCap keep CSR order.
template <int P>
__device__ __forceinline__ void order_row(const int32_t* __restrict__ idx, const int64_t* __restrict__ df,
                                          int32_t* __restrict__ order, int64_t s, int n, int lane) {
  int32_t x[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int e = lane * P + p;
    const int64_t f = e < n ? df[idx[s + e]] : 0;
    x[p] = e < n ? (int32_t)((f < (1 << 21) - 1 ? f : (1 << 21) - 1) << 10 | e) : INT32_MAX;
  }
  bitonic_regs<P>(x, lane);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int e = lane * P + p;
    if (e < n) order[s + e] = x[p] & 1023;
  }
}

__global__ __launch_bounds__(64 * kDocWaves) void k_row_order(const int64_t* __restrict__ indptr, int64_t rows,
                                                             const int32_t* __restrict__ idx,
                                                             const int64_t* __restrict__ df,
                                                             int32_t* __restrict__ order) {
  const int lane = threadIdx.x & 63;
  for (int64_t d = (int64_t)blockIdx.x * kDocWaves + (threadIdx.x >> 6); d < rows;
       d += (int64_t)gridDim.x * kDocWaves) {
    const int64_t s = indptr[d], n64 = indptr[d + 1] - s;
    if (n64 > kSortCap) {
      for (int64_t e = lane; e < n64; e += 64) order[s + e] = (int32_t)e;
      continue;
    }
    const int n = (int)n64;
    if (n <= 64) order_row<1>(idx, df, order, s, n, lane);
    else if (n <= 128) order_row<2>(idx, df, order, s, n, lane);
    else if (n <= 256) order_row<4>(idx, df, order, s, n, lane);
    else if (n <= 512) order_row<8>(idx, df, order, s, n, lane);
    else order_row<16>(idx, df, order, s, n, lane);
  }
}

void row_order_by_df(Ctx& c, const DCsr& m, const int64_t* d_df, int32_t* d_order) {
  if (m.rows == 0 || m.nnz == 0) return;
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(ceil_div(m.rows, kDocWaves), 1), 1 << 14);
  k_row_order<<<g, 64 * kDocWaves, 0, c.stream>>>(m.indptr.as<int64_t>(), m.rows, m.indices.as<int32_t>(), d_df,
                                                  d_order);
  KERNEL_CHECK();
}

// resident token corpora keep their token offsets as u32 when the blob allows (stc_tokens_upload): the
// offsets are 8 of the ~16 bytes HashingTF reads per token
__global__ __launch_bounds__(256) void k_narrow(const int64_t* __restrict__ src, int64_t n, uint32_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dst[i] = (uint32_t)src[i];
}
void narrow_offsets(Ctx& c, const int64_t* d_src, int64_t n, uint32_t* d_dst) {
  if (n == 0) return;
  k_narrow<<<grid_for(n, 256, 256 * 32), 256, 0, c.stream>>>(d_src, n, d_dst);
  KERNEL_CHECK();
}

// the look-back single pass (modes 1 / 2); false: a look-back timed out, the caller runs the passes
static bool single_pass(Ctx& c, const uint8_t* d_utf8, const int64_t* d_tok_off64, const uint32_t* d_tok_off32,
                        int64_t n_tok, const int64_t* d_doc_off, int64_t n_docs, int32_t num_features, int binary,
                        int variant, int value_dtype, DCsr& out) {
  hipStream_t st = c.stream;
  const int64_t tiles = ceil_div(n_docs, (int64_t)kEmitWaves);
  DevBuf& lb = c.scratch[2];
  lb.reserve(sizeof(uint64_t) * (tiles + kTicketWords));
  uint64_t* status = lb.as<uint64_t>();  // [tiles] look-back words, the fault word, 8 ticket counters
  HIP_CHECK(hipMemsetAsync(status, 0, sizeof(uint64_t) * (tiles + kTicketWords), st));
  HIP_CHECK(hipMemsetAsync(out.indptr.p, 0, sizeof(int64_t), st));
  // nnz ≤ n_tok: the output is sized before the counts exist
  c.recycle.take(out.indices, sizeof(int32_t) * n_tok);
  c.recycle.take(out.values, (value_dtype == STC_F32 ? 4 : 8) * n_tok);
  // mode 1 (default): hashed inside the per-document pass; mode 2: the tokens hashed flat first (k_hash,
  // four independent chains per lane), the per-document pass then loads, sorts and emits
  const bool flat = c.tf_mode == 2;
  int32_t* keys = nullptr;
  if (flat) {
    DevBuf& kb = c.scratch[0];
    kb.reserve(sizeof(int32_t) * n_tok);
    keys = kb.as<int32_t>();
    if (d_tok_off32) hash_tokens_t(c, d_utf8, d_tok_off32, n_tok, num_features, variant, keys);
    else hash_tokens_t(c, d_utf8, d_tok_off64, n_tok, num_features, variant, keys);
  }
  int max_polls = c.tf_force_fault ? 0 : kLbMaxPolls;
  auto go = [&](auto spark, auto* vals) {
    constexpr bool S24 = decltype(spark)::value;
    using V = std::remove_pointer_t<decltype(vals)>;
    auto launch = [&](const void* kern, auto tok_off) {
      // a grid of what is resident (more workgroups would only take tickets past the end); the occupancy
      // query once per kernel and process
      static std::mutex mu;
      static std::map<const void*, int> occ;
      int per_cu = 0;
      {
        std::lock_guard<std::mutex> lk(mu);
        auto it = occ.find(kern);
        if (it == occ.end()) {
          HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kEmitWaves, 0));
          occ[kern] = per_cu;
        } else {
          per_cu = it->second;
        }
      }
      const int64_t resident = (int64_t)std::max(per_cu, 1) * c.cus;
      const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(tiles, resident));
      unsigned long long* ticket = reinterpret_cast<unsigned long long*>(status + tiles + kTicketPitch);
      const uint8_t* u8 = d_utf8;
      const int64_t* doff = d_doc_off;
      int64_t nd = n_docs;
      int32_t nf = num_features;
      int bin = binary;
      int64_t* ip = out.indptr.as<int64_t>();
      int32_t* ix = out.indices.as<int32_t>();
      V* vv = vals;
      uint64_t* stp = status;
      void* args[] = {&keys, &u8, &tok_off, &doff, &nd, &nf, &bin, &ip, &ix, &vv, &stp, &ticket, &max_polls};
      HIP_CHECK(hipLaunchKernel(kern, dim3(g), dim3(64 * kEmitWaves), args, 0, st));
    };
    if (flat) launch((const void*)k_doc_hash_emit<S24, true, V, int64_t>, d_tok_off64);
    else if (d_tok_off32) launch((const void*)k_doc_hash_emit<S24, false, V, uint32_t>, d_tok_off32);
    else launch((const void*)k_doc_hash_emit<S24, false, V, int64_t>, d_tok_off64);
  };
  if (value_dtype == STC_F32) {
    if (variant == STC_HASH_SPARK24) go(std::true_type{}, out.values.as<float>());
    else go(std::false_type{}, out.values.as<float>());
  } else {
    if (variant == STC_HASH_SPARK24) go(std::true_type{}, out.values.as<double>());
    else go(std::false_type{}, out.values.as<double>());
  }
  KERNEL_CHECK();
  int64_t total = 0;
  uint64_t fault = 0;
  HIP_CHECK(hipMemcpyAsync(&total, out.indptr.as<int64_t>() + n_docs, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipMemcpyAsync(&fault, status + tiles, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  if (fault) {
    ++c.tf_fallbacks;
    return false;
  }
  out.nnz = total;
  out.positive = true;
  out.unique_ids = true;
  return true;
}

void build_csr(Ctx& c, const uint8_t* d_utf8, const int64_t* d_tok_off64, const uint32_t* d_tok_off32, int64_t n_tok,
               const int64_t* d_doc_off, int64_t n_docs, int32_t num_features, int binary,
               int variant, int value_dtype, int64_t max_doc, DCsr& out) {
  STC_REQUIRE(n_tok < (int64_t(1) << 31), "at most 2^31-1 tokens per call (split the corpus)");
  hipStream_t st = c.stream;
  out.rows = n_docs;
  out.cols = num_features;
  out.dtype = value_dtype;
  c.recycle.take(out.indptr, sizeof(int64_t) * (n_docs + 1));
  if (n_tok == 0) {
    HIP_CHECK(hipMemsetAsync(out.indptr.p, 0, sizeof(int64_t) * (n_docs + 1), st));
    out.nnz = 0;
    return;
  }
  if (max_doc >= 0 && max_doc <= kFusedCap && c.tf_mode > 0 &&
      single_pass(c, d_utf8, d_tok_off64, d_tok_off32, n_tok, d_doc_off, n_docs, num_features, binary, variant,
                  value_dtype, out))
    return;
  // grow-only scratch kept on the context (the featurisation of one corpus reuses it): no allocation,
  // and so no implicit device synchronisation of hipFree, per call
  DevBuf& keys = c.scratch[0];
  DevBuf& sorted = c.scratch[1];
  DevBuf& nnz = c.scratch[2];
  DevBuf& small = c.scratch[3];
  DevBuf& stmp = c.scratch[4];
  nnz.reserve(sizeof(int64_t) * (n_docs + 1));
  small.reserve(sizeof(int32_t) * (n_docs + 16));
  sorted.reserve(sizeof(int32_t) * n_tok);
  int32_t* n_large_d = small.as<int32_t>();  // word 0: long documents, word 1: medium ones
  int32_t* large = small.as<int32_t>() + 16;
  HIP_CHECK(hipMemsetAsync(n_large_d, 0, 2 * sizeof(int32_t), st));
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(ceil_div(n_docs, kDocWaves), 1), 1 << 14);
  keys.reserve(sizeof(int32_t) * n_tok);  // the long documents' bucket ids, at their token positions
  auto pass_a = [&](auto spark, const auto* tok_off) {
    constexpr bool S24 = decltype(spark)::value;
    k_doc_hash_sort<S24><<<g, 64 * kDocWaves, 0, st>>>(d_utf8, tok_off, d_doc_off, n_docs, num_features,
                                                       keys.as<int32_t>(), sorted.as<int32_t>(), nnz.as<int64_t>() + 1,
                                                       large, n_large_d, n_large_d + 1);
  };
  if (variant == STC_HASH_SPARK24) {
    if (d_tok_off32) pass_a(std::true_type{}, d_tok_off32);
    else pass_a(std::true_type{}, d_tok_off64);
  } else {
    if (d_tok_off32) pass_a(std::false_type{}, d_tok_off32);
    else pass_a(std::false_type{}, d_tok_off64);
  }
  KERNEL_CHECK();
  int32_t counts[2] = {0, 0};
  HIP_CHECK(hipMemcpyAsync(counts, n_large_d, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  const int32_t n_large = counts[0];
  if (counts[1] > 0) {
    k_doc_sort<<<g, 64 * kDocWaves, 0, st>>>(keys.as<int32_t>(), d_doc_off, n_docs, sorted.as<int32_t>(),
                                             nnz.as<int64_t>() + 1);
    KERNEL_CHECK();
  }
  DevBuf& sorted_l = c.scratch[5];
  DevBuf& seg = c.scratch[6];
  DevBuf& flags = c.scratch[7];
  DevBuf& tmp = c.scratch[8];
  if (n_large > 0) {  // long documents: hipcub segmented radix sort, then their run counts
    sorted_l.reserve(sizeof(int32_t) * n_tok);
    seg.reserve(sizeof(int64_t) * 2 * n_large);
    flags.reserve(n_docs);
    HIP_CHECK(hipMemsetAsync(flags.p, 0, n_docs, st));
    int64_t* beg = seg.as<int64_t>();
    int64_t* end = beg + n_large;
    k_large_segments<<<(unsigned)ceil_div(n_large, 256), 256, 0, st>>>(large, n_large, d_doc_off, beg, end,
                                                                       flags.as<uint8_t>());
    KERNEL_CHECK();
    int nbits = 1;  // bucket ids < numFeatures
    while ((int64_t(1) << nbits) < num_features) ++nbits;
    size_t tb = 0;
    HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tb, keys.as<int32_t>(), sorted_l.as<int32_t>(),
                                                         (int)n_tok, n_large, beg, end, 0, nbits, st));
    tmp.reserve(tb);
    HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortKeys(tmp.p, tb, keys.as<int32_t>(), sorted_l.as<int32_t>(),
                                                         (int)n_tok, n_large, beg, end, 0, nbits, st));
    k_doc_runs<false, float><<<(unsigned)std::min<int64_t>(ceil_div((int64_t)n_large, (int64_t)kDocWaves), 1 << 14), 64 * kDocWaves, 0, st>>>(
        sorted.as<int32_t>(), sorted_l.as<int32_t>(), flags.as<uint8_t>(), large, n_large, d_doc_off, n_docs,
        nullptr, binary, nullptr, nullptr, nnz.as<int64_t>() + 1);
    KERNEL_CHECK();
  }
  // indptr = [0, inclusive scan of nnz]
  HIP_CHECK(hipMemsetAsync(out.indptr.p, 0, sizeof(int64_t), st));
  size_t sb = 0;
  HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, sb, nnz.as<int64_t>() + 1, out.indptr.as<int64_t>() + 1,
                                             (int)n_docs, st));
  stmp.reserve(sb);
  HIP_CHECK(hipcub::DeviceScan::InclusiveSum(stmp.p, sb, nnz.as<int64_t>() + 1, out.indptr.as<int64_t>() + 1,
                                             (int)n_docs, st));
  int64_t total = 0;
  HIP_CHECK(hipMemcpyAsync(&total, out.indptr.as<int64_t>() + n_docs, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  out.nnz = total;
  out.positive = true;  // counts ≥ 1 (binary: 1)
  out.unique_ids = true;  // one entry per distinct id
  c.recycle.take(out.indices, sizeof(int32_t) * std::max<int64_t>(total, 1));
  c.recycle.take(out.values, (value_dtype == STC_F32 ? 4 : 8) * std::max<int64_t>(total, 1));
  const uint8_t* fl = n_large > 0 ? flags.as<uint8_t>() : nullptr;
  if (value_dtype == STC_F32)
    k_doc_runs<true, float><<<g, 64 * kDocWaves, 0, st>>>(sorted.as<int32_t>(), sorted_l.as<int32_t>(), fl, large, n_large,
                                              d_doc_off, n_docs, out.indptr.as<int64_t>(), binary,
                                              out.indices.as<int32_t>(), out.values.as<float>(), nullptr);
  else
    k_doc_runs<true, double><<<g, 64 * kDocWaves, 0, st>>>(sorted.as<int32_t>(), sorted_l.as<int32_t>(), fl, large, n_large,
                                               d_doc_off, n_docs, out.indptr.as<int64_t>(), binary,
                                               out.indices.as<int32_t>(), out.values.as<double>(), nullptr);
  KERNEL_CHECK();
}

}  // namespace hashing
}  // namespace stc
