// inflate_split.hip -- one LARGE member decoded by many workgroups at once.
//
// The lane path (inflate_lane.hip) and the wave path (inflate_wave.hip) give a
// member one lane / one wave: a member's decode is one serial chain of Huffman
// lookups, so one large member in a batch -- C5-ii's 2.19 MB deflate64 fixture
// (SURVEY.md 8(d)), 75 ms in one wave -- sets the whole batch's time.  Here a
// member is cut at its block boundaries and the pieces decode in parallel:
//
//  1. zs_k_split_find: the member's bits are divided into ZS_SPLIT_MAX ranges;
//     one workgroup per range tests every bit offset of its range (32 at a
//     time per thread, candidates queued for the full check) for the start of a
//     dynamic-Huffman block header that zlib would
//     accept (zs_split_header_rest: a complete code-length code, code lengths
//     that decode without overrunning, an end-of-block code, complete lit/len
//     and distance codes -- stricter than inflate_table, which only costs a
//     missed boundary), and keeps the first.
//  2. zs_k_split_decode: one workgroup per found start (a "piece"; the first
//     piece starts at bit 0) decodes blocks wave-uniformly, like
//     zs_k_inflate_wave, until it closes a block at or past the next piece's
//     start.  The history before a piece's start is unknown: a copy reaching
//     back before it produces MARKERS -- the ring and the piece's output hold
//     u16 values, a byte below 256, and 255 + k for "the byte k positions
//     before the piece" (k <= 65280) -- which copies propagate like bytes.
//  3. zs_k_split_resolve: one workgroup per member checks that the pieces
//     chain (each ended exactly where the next one starts, without an error,
//     the last one with the final block), places them by a prefix sum of their
//     lengths and, piece by piece in order, writes each byte or looks its
//     marker up in the bytes already written.
//
// Any doubt -- an error in a piece, pieces that do not chain (a header found at
// a bit offset that is not a real block start), a marker further back than a
// u16 can say, a piece over its scratch -- sets the member's bail, and the exact
// kernel (zs_k_inflate) decodes it, so statuses and messages stay exact.
// Semantics: inffast.ts:5-228 without call boundaries, i.e. deflate64 (which
// the reference never decodes with inflate_fast, inflate.ts:841) and raw
// deflate with inflate_ref_wrap = 0; the host routes only those here.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_inflate.h"
#include "zs_inftab.h"
#include "zs_wave.h"
#include "zs_split.h"

// ------------------------------------------------------------ header check
// The candidate's bits: words of the member read aligned (w4: the aligned
// words holding it, sh: its offset in the first, last: the last word's index).
// The candidate's bits: the aligned words holding the member (w4; sh: its
// offset in the first, last: the last word's index, reads clamped to it).
// (pointers typed by address space: generic ones let the compiler fold word()'s two loads into one
// flat load of a selected pointer)
typedef const __attribute__((address_space(1))) uint32_t zs_gc_u32;
typedef const __attribute__((address_space(3))) uint32_t zs_lc_u32;
struct zs_hdr_src {
  zs_gc_u32* w4;
  uint32_t sh, last;
  zs_lc_u32* lw;  // a window of the aligned words staged in LDS: [lq0, lq0 + ln)
  uint32_t lq0, ln;
  __device__ __forceinline__ uint32_t word(uint32_t q) const {
    return q - lq0 < ln ? lw[q - lq0] : w4[min(q, last)];
  }
  __device__ __forceinline__ uint32_t load4(uint64_t at) const {  // bytes [at, at + 4)
    const uint64_t cb = at + sh;
    const uint32_t q = (uint32_t)(cb >> 2);
    return __builtin_amdgcn_alignbyte(word(q + 1u), word(q), (uint32_t)(cb & 3u));
  }
};

// The rest of a dynamic header that inflate (inflate.ts:662-836) accepts, for
// a candidate that passed the finder's quick tests: the code lengths decode (repeat 16
// never first, no run past HLIT + HDIST), the end-of-block code has a length,
// and -- stricter than inflate_table, which only costs a missed boundary --
// the lit/len code is complete and the distance code complete or one 1-bit
// code.  Kraft sums scaled to 2^15 replace per-length counts, and the
// code-length code decodes from registers (no tables: any thread may run it).
// (kBlPos: each code-length symbol's place in the header's order, ZS_BL_ORDER inverted)
static constexpr uint8_t kBlPos[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};

static __device__ bool zs_split_header_rest(const zs_hdr_src S, uint64_t bit, uint64_t nbits, uint64_t a,
                                            uint64_t b) {
  const uint32_t nlen = (uint32_t)((a >> 3) & 31u) + 257, ndist = (uint32_t)((a >> 8) & 31u) + 1;
  const uint32_t ncode = (uint32_t)((a >> 13) & 15u) + 4u;
  // the code-length code's canonical codes (RFC 1951 3.2.2), in symbol order per length
  uint32_t cl[19];
#pragma unroll
  for (uint32_t i = 0; i < 19; i++) {
    const uint32_t pos = 17u + 3u * i;
    uint32_t v;
    if (pos + 3u <= 64u) v = (uint32_t)(a >> pos) & 7u;
    else if (pos >= 64u) v = (uint32_t)(b >> (pos - 64u)) & 7u;
    else v = (uint32_t)((a >> pos) | (b << (64u - pos))) & 7u;
    cl[i] = i < ncode ? v : 0u;
  }
  // the canonical code (RFC 1951 3.2.2) in registers: with the next 7 bits
  // read MSB first (r), a code's length is 1 + #{l < 7 : r >= lim[l]} (lim[l]:
  // the end of the length-l codes, left-justified to 7 bits), its rank
  // (r >> (7 - L)) + base[L], and the symbols by rank are 5-bit fields of sy
  uint32_t lim[8], base[8];
  uint64_t sy0 = 0, sy1 = 0;  // ranks 0..11, 12..18
  {
    uint32_t code = 0, rank = 0;
#pragma unroll
    for (uint32_t len = 1; len <= 7; len++) {
      uint32_t c = 0;
#pragma unroll
      for (uint32_t sym = 0; sym < 19; sym++) {
        const bool hit = cl[kBlPos[sym]] == len;
        const uint32_t k = rank + c;
        if (hit) {
          if (k < 12) sy0 |= (uint64_t)sym << (5u * k);
          else sy1 |= (uint64_t)sym << (5u * (k - 12u));
        }
        c += hit ? 1u : 0u;
      }
      base[len] = rank - code;
      lim[len] = (code + c) << (7u - len);
      rank += c;
      code = (code + c) << 1;
    }
  }
  // the bit reader, past the 17 + 3 ncode header bits
  uint64_t at = (bit + 17u + 3u * ncode) >> 3;
  uint64_t hold = (uint64_t)S.load4(at) | ((uint64_t)S.load4(at + 4) << 32);
  uint32_t bits = 64u - (uint32_t)((bit + 17u + 3u * ncode) & 7u);
  hold >>= 64u - bits;
  at += 8;
  uint64_t used = bit + 17u + 3u * ncode;  // stream bits consumed
  auto need = [&](uint32_t k) {
    if (bits < k) {
      hold |= (uint64_t)S.load4(at) << bits;
      at += 4;
      bits += 32;
    }
  };
  auto take = [&](uint32_t k) -> uint32_t {
    need(k);
    const uint32_t v = (uint32_t)hold & ((1u << k) - 1u);
    hold >>= k;
    bits -= k;
    used += k;
    return v;
  };
  uint32_t kl = 0, kd = 0, dn = 0, i = 0, prev = 0;
  bool eob = false;
  while (i < nlen + ndist) {
    // one code-length symbol
    need(7);
    const uint32_t r = __builtin_bitreverse32((uint32_t)hold) >> 25;
    uint32_t L = 1;
#pragma unroll
    for (uint32_t len = 1; len < 7; len++) L += r >= lim[len] ? 1u : 0u;
    uint32_t bs = base[1];
#pragma unroll
    for (uint32_t len = 2; len <= 7; len++) bs = L == len ? base[len] : bs;
    const uint32_t k = (r >> (7u - L)) + bs;
    const uint32_t v = (uint32_t)((k < 12 ? sy0 >> (5u * k) : sy1 >> (5u * (k - 12u))) & 31u);
    hold >>= L;
    bits -= L;
    used += L;
    uint32_t rep = 1, val = v;
    if (v == 16) {
      if (i == 0) return false;
      rep = 3 + take(2);
      val = prev;
    } else if (v == 17) {
      rep = 3 + take(3);
      val = 0;
    } else if (v == 18) {
      rep = 11 + take(7);
      val = 0;
    }
    if (i + rep > nlen + ndist || used > nbits) return false;
    const uint32_t w = val ? 32768u >> val : 0u;
    // the run's part in each code
    const uint32_t nl = i < nlen ? min(rep, nlen - i) : 0u;
    kl += nl * w;
    kd += (rep - nl) * w;
    dn += val ? rep - nl : 0u;
    if (i <= 256u && 256u < i + rep) eob = val != 0;
    if (kl > 32768u || kd > 32768u) return false;  // over-subscribed
    i += rep;
    prev = val;
  }
  return eob && kl == 32768u && (kd == 32768u || (dn == 1 && kd == 16384u));
}

// ----------------------------------------------------------------- finder
// The code-length code's Kraft sum from a candidate's bits (a: 0..63, b:
// 64..127): CODES must be complete (inftrees.ts:128-139).
static __device__ __forceinline__ bool zs_split_kraft(uint64_t a, uint64_t b) {
  const uint32_t ncode = (uint32_t)((a >> 13) & 15u) + 4u;
  uint32_t kraft = 0;
#pragma unroll
  for (uint32_t i = 0; i < 19; i++) {
    const uint32_t pos = 17u + 3u * i;
    uint32_t v;
    if (pos + 3u <= 64u) v = (uint32_t)(a >> pos) & 7u;
    else if (pos >= 64u) v = (uint32_t)(b >> (pos - 64u)) & 7u;
    else v = (uint32_t)((a >> pos) | (b << (64u - pos))) & 7u;
    kraft += (i < ncode && v) ? (128u >> v) : 0u;
  }
  return kraft == 128u;
}

// One workgroup per (member, range): ranges r = 1 .. ZS_SPLIT_MAX-1 of
// span = max(16384, nbits / ZS_SPLIT_MAX) bits (range 0 is the member's start);
// found[m * ZS_SPLIT_MAX + r] = the first header start in the range, or ~0.
// A thread tests the 32 bit offsets of one member word at a time: BTYPE = 2
// and HLIT / HDIST in range for all 32 at once on shifted words (about one
// offset in five passes), the code-length code's Kraft sum for those, and the
// survivors (~1 %) queue in LDS; the full header check (zs_split_header_rest)
// then runs one candidate per thread, so a wave's lanes share the long checks
// instead of waiting on one.  Chunks of 8,192 offsets in order: the first chunk
// with an accepted candidate holds the range's first.
#define ZS_FIND_T 256u
#define ZS_FIND_Q 1024u
#ifndef ZS_FIND_EXP
#define ZS_FIND_EXP 0  // timing experiments (0 in the product): 1 no full checks, 2 no Kraft test, 4 staging only, 8 counters
#endif
#if ZS_FIND_EXP & 8
__device__ unsigned long long zs_find_stat[4];  // chunks, queued, checked, clock cycles in the checks
extern "C" int zs_find_stats(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_find_stat), sizeof(zs_find_stat));
}
#endif
__global__ __launch_bounds__(256) void zs_k_split_find(const uint8_t* __restrict__ in,
                                                     const uint64_t* __restrict__ in_off,
                                                     const uint32_t* __restrict__ in_len,
                                                     const uint32_t* __restrict__ list, int wbits,
                                                     uint64_t* __restrict__ found) {
  __shared__ unsigned long long best;
  __shared__ uint32_t nq;
  __shared__ uint32_t qoff[ZS_FIND_Q];       // queued candidates, bits past the range's start
  __shared__ uint32_t stage[2 * ZS_FIND_T];  // the chunk's aligned words and as many after (the headers' bits)
  const uint32_t m = blockIdx.x / ZS_SPLIT_MAX, r = blockIdx.x % ZS_SPLIT_MAX, t = threadIdx.x;
  const uint32_t s = list[m];
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  const uint64_t nbits = 8ull * n;
  const uint64_t span = zs_split_span(n);
  const uint64_t lo = span * r, hi = min(nbits, lo + span);
  if (t == 0) {
    best = ~0ull;
    nq = 0;
  }
  __syncthreads();
  if (r == 0 || lo >= hi) {
    if (t == 0) found[blockIdx.x] = r == 0 ? 0ull : ~0ull;
    return;
  }
  const bool d64 = wbits == -16;
  zs_hdr_src S;
  S.sh = (uint32_t)((uintptr_t)src & 3u);
  S.w4 = (zs_gc_u32*)(src - S.sh);
  S.last = (S.sh + n - 1u) >> 2;
  S.lw = (zs_lc_u32*)stage;
  S.ln = 0;
  S.lq0 = 0;
  const uint64_t w_lo = lo >> 5, w_hi = (hi + 31u) >> 5;
  for (uint64_t wc = w_lo; wc < w_hi; wc += ZS_FIND_T) {
    // stage the chunk's words (and 1 KiB after): the quick tests and most header checks read LDS
    S.ln = 0;
    for (uint32_t i = t; i < 2 * ZS_FIND_T; i += ZS_FIND_T) stage[i] = S.word((uint32_t)wc + i);
    __syncthreads();
    S.lq0 = (uint32_t)wc;
    S.ln = 2 * ZS_FIND_T;
    const uint64_t w = wc + t;
    if (!(ZS_FIND_EXP & 4) && w < w_hi) {
      // member words w .. w+4 (member bit 32 w on), from the aligned words
      uint32_t mw[5];
      {
        uint32_t aw[6];
#pragma unroll
        for (uint32_t k = 0; k < 6; k++) aw[k] = S.word((uint32_t)w + k);
#pragma unroll
        for (uint32_t k = 0; k < 5; k++) mw[k] = __builtin_amdgcn_alignbyte(aw[k + 1], aw[k], S.sh);
      }
      const uint64_t x0 = ((uint64_t)mw[1] << 32) | mw[0], x1 = ((uint64_t)mw[3] << 32) | mw[2], x2 = mw[4];
#define ZS_SB(k) ((uint32_t)(x0 >> (k)))  // bit o + k of the candidate at offset o, for o = 0..31
      uint32_t c = ~ZS_SB(1) & ZS_SB(2) & ~(ZS_SB(4) & ZS_SB(5) & ZS_SB(6) & ZS_SB(7));
      if (!d64) c &= ~(ZS_SB(9) & ZS_SB(10) & ZS_SB(11) & ZS_SB(12));
#undef ZS_SB
      const uint64_t b0 = 32ull * w;
      if (b0 < lo) c &= ~0u << (uint32_t)(lo - b0);
      if (b0 + 32u > hi) c &= (1u << (uint32_t)(hi - b0)) - 1u;
      while (c) {
        const uint32_t o = (uint32_t)__builtin_ctz(c);
        c &= c - 1u;
        const uint64_t a = o ? (x0 >> o) | (x1 << (64u - o)) : x0;
        const uint64_t bb = o ? (x1 >> o) | (x2 << (64u - o)) : x1;
        if (!(ZS_FIND_EXP & 2) && zs_split_kraft(a, bb)) {
          const uint32_t qi = atomicAdd(&nq, 1u);
          if (qi < ZS_FIND_Q) qoff[qi] = (uint32_t)(b0 + o - lo);
          else if (zs_split_header_rest(S, b0 + o, nbits, a, bb)) atomicMin(&best, (unsigned long long)(b0 + o));
        }
      }
    }
    __syncthreads();
    const uint32_t cnt = (ZS_FIND_EXP & 1) ? 0u : min(nq, ZS_FIND_Q);
#if ZS_FIND_EXP & 8
    if (t == 0) {
      atomicAdd(&zs_find_stat[0], 1ull);
      atomicAdd(&zs_find_stat[1], (unsigned long long)cnt);
    }
    const unsigned long long tc0 = clock64();
#endif
    for (uint32_t i = t; i < cnt; i += ZS_FIND_T) {
      const uint64_t bit = lo + qoff[i];
      if (bit >= best) continue;
#if ZS_FIND_EXP & 8
      atomicAdd(&zs_find_stat[2], 1ull);
#endif
      uint64_t a, bb;
      {
        const uint64_t cb = (bit >> 3) + S.sh;
        const uint32_t q = (uint32_t)(cb >> 2);
        const uint32_t off = (uint32_t)((cb & 3u) * 8u + (bit & 7u));
        const uint64_t l0 = ((uint64_t)S.word(q + 1u) << 32) | S.word(q),
                       h0 = ((uint64_t)S.word(q + 3u) << 32) | S.word(q + 2u);
        a = off ? (l0 >> off) | (h0 << (64u - off)) : l0;
        bb = h0 >> off;
      }
      if (zs_split_header_rest(S, bit, nbits, a, bb)) atomicMin(&best, (unsigned long long)bit);
    }
#if ZS_FIND_EXP & 8
    if ((t & 63) == 0) atomicAdd(&zs_find_stat[3], clock64() - tc0);
#endif
    __syncthreads();
    if (best != ~0ull) break;
    if (t == 0) nq = 0;
    __syncthreads();  // (also: the stage is rewritten next)
  }
  if (t == 0) found[blockIdx.x] = best;
}

// the member's found starts in order (piece order; piece 0 starts at bit 0)
static __device__ __forceinline__ uint32_t zs_split_starts(const uint64_t* found, uint32_t m, uint64_t* starts) {
  uint32_t c = 0;
  for (uint32_t r = 0; r < ZS_SPLIT_MAX; r++) {
    const uint64_t f = found[m * ZS_SPLIT_MAX + r];
    if (f != ~0ull) starts[c++] = f;
  }
  return c;
}

// ----------------------------------------------------------------- decoder
// u16 history ring (the window: 32 KiB; deflate64 64 KiB) first in the dynamic LDS
struct zs_split_tabs {
  uint32_t inw[ZS_WIN_IN];
  zcode codes[ENOUGH_LENS + ENOUGH_DISTS_9];
  uint16_t lens[320];
  uint16_t work[288];
};

__global__ __launch_bounds__(64) void zs_k_split_decode(const uint8_t* __restrict__ in,
                                                       const uint64_t* __restrict__ in_off,
                                                       const uint32_t* __restrict__ in_len,
                                                       const uint32_t* __restrict__ list, int wbits,
                                                       const uint64_t* __restrict__ found,
                                                       zs_split_piece_res* __restrict__ pres,
                                                       uint16_t* __restrict__ scratch, uint32_t piece_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t zs_ssm[];
  const bool d64 = wbits == -16;
  const uint32_t wsize = d64 ? 65536u : 32768u;
  const uint32_t rmask = wsize - 1u;
  uint16_t* ring = reinterpret_cast<uint16_t*>(zs_ssm);
  zs_split_tabs& W = *reinterpret_cast<zs_split_tabs*>(zs_ssm + 2u * wsize);
  const uint32_t m = blockIdx.x / ZS_SPLIT_MAX, k = blockIdx.x % ZS_SPLIT_MAX;
  const uint32_t lane = threadIdx.x;
  const uint32_t s = zs_u(list[m]);
  const uint32_t n = zs_u(in_len[s]);
  __shared__ uint64_t starts[ZS_SPLIT_MAX];
  uint32_t npieces = 0;
  if (lane == 0) npieces = zs_split_starts(found, m, starts);
  npieces = zs_u(npieces);
  if (k >= npieces) return;
  const uint64_t start = starts[k];
  const uint8_t* src = in + in_off[s];
  zs_wave_reader R;
  R.n = n;
  R.sh = (uint32_t)((uintptr_t)src & 3u);
  R.w4 = reinterpret_cast<const uint32_t*>(src - R.sh);
  R.last = (R.sh + n - 1u) >> 2;
  R.inw = W.inw;
  const uint32_t at0 = (uint32_t)(start >> 3);
  zs_wr_stage(R, (at0 + R.sh) >> 2);
  zs_wr_seek(R, at0);
  zs_wr_take(R, (uint32_t)(start & 7u));
  uint16_t* dst = scratch + (size_t)blockIdx.x * piece_cap;
  uint32_t* dstw = reinterpret_cast<uint32_t*>(dst);
  const uint32_t* ringw = reinterpret_cast<const uint32_t*>(ring);
  const uint32_t lmask = d64 ? 31u : 15u;
  const bool first = k == 0;
  uint32_t total = 0, flushed = 0, next = ZS_SPLIT_MAX, nblk = 0;
  bool bail = false, last = false;
  // output leaves the ring 128 entries (one dword per lane) at a time
  auto flush = [&]() {
    while (total - flushed >= 128u) {
      dstw[(flushed >> 1) + lane] = ringw[((flushed & rmask) >> 1) + lane];
      flushed += 128u;
    }
  };
  // the value at piece position x = total + i - dist (signed): the ring, or a marker
  auto hist = [&](uint32_t t, uint32_t dist, bool& bad) -> uint32_t {
    if (t >= dist) return ring[(t - dist) & rmask];
    const uint32_t back = dist - t;  // 1 .. 65536 before the piece
    if (first || back > ZS_SPLIT_MARK_MAX) { bad = true; return 0u; }
    return 255u + back;
  };
  while (!bail && !last) {
    // A block closed exactly where a later piece starts: the piece ends (a
    // start that is no real block boundary -- a header-like bit pattern inside
    // a block -- is passed over, and its piece falls off the chain)
    if (nblk++) {
      const uint64_t b = zs_wr_bitpos(R);
      uint32_t q = k + 1;
      while (q < npieces && starts[q] < b) q++;
      if (q < npieces && starts[q] == b) { next = q; break; }
    }
    last = zs_wr_take(R, 1) != 0;
    const uint32_t type = zs_wr_take(R, 2);
    uint32_t lbits, dbits, lused;
    if (type == 0) {  // stored
      zs_wr_align(R);
      const uint32_t len = zs_wr_take(R, 16), nlen = zs_wr_take(R, 16);
      const uint32_t at = (uint32_t)(zs_wr_bitpos(R) >> 3);
      if (len != (nlen ^ 0xffffu) || zs_wr_over(R) || at + len > R.n || total + len > piece_cap) { bail = true; break; }
      for (uint32_t i = 0; i < len; i += 64) {
        const uint32_t j = i + lane;
        if (j < len) ring[(total + lane) & rmask] = src[at + j];
        total += min(64u, len - i);
        flush();
      }
      zs_wr_seek(R, at + len);
      continue;
    }
    if (type == 1) {
      uint32_t sym;
      for (sym = 0; sym < 144; sym++) W.lens[sym] = 8;
      for (; sym < 256; sym++) W.lens[sym] = 9;
      for (; sym < 280; sym++) W.lens[sym] = 7;
      for (; sym < 288; sym++) W.lens[sym] = 8;
      lbits = 9;
      zs_inflate_table(LENS, W.lens, 288, W.codes, &lbits, W.work, d64, &lused);
      for (sym = 0; sym < 32; sym++) W.lens[sym] = 5;
      dbits = 5;
      zs_inflate_table(DISTS, W.lens, 32, W.codes + lused, &dbits, W.work, d64, &sym);
    } else if (type == 2) {
      const uint32_t nlen = zs_wr_take(R, 5) + 257, ndist = zs_wr_take(R, 5) + 1, ncode = zs_wr_take(R, 4) + 4;
      if (nlen > 286 || (!d64 && ndist > 30)) { bail = true; break; }
      uint32_t i;
      for (i = 0; i < ncode; i++) W.lens[ZS_BL_ORDER[i]] = (uint16_t)zs_wr_take(R, 3);
      for (; i < 19; i++) W.lens[ZS_BL_ORDER[i]] = 0;
      uint32_t cbits = 7, used;
      if (zs_inflate_table(CODES, W.lens, 19, W.codes, &cbits, W.work, d64, &used)) { bail = true; break; }
      i = 0;
      while (i < nlen + ndist) {
        const zcode here = zs_wr_decode(R, W.codes, cbits);
        const uint32_t v = C_VAL(here);
        if (v < 16) { W.lens[i++] = (uint16_t)v; continue; }
        uint32_t rep, val = 0;
        if (v == 16) {
          if (i == 0) { bail = true; break; }
          val = zs_u(W.lens[i - 1]);
          rep = 3 + zs_wr_take(R, 2);
        } else if (v == 17) {
          rep = 3 + zs_wr_take(R, 3);
        } else {
          rep = 11 + zs_wr_take(R, 7);
        }
        if (i + rep > nlen + ndist) { bail = true; break; }
        while (rep--) W.lens[i++] = (uint16_t)val;
      }
      if (bail || zs_wr_over(R) || zs_u(W.lens[256]) == 0) { bail = true; break; }
      lbits = 9;
      uint32_t dused;
      if (zs_inflate_table(LENS, W.lens, nlen, W.codes, &lbits, W.work, d64, &lused)) { bail = true; break; }
      dbits = 6;
      if (zs_inflate_table(DISTS, W.lens + nlen, ndist, W.codes + lused, &dbits, W.work, d64, &dused)) {
        bail = true;
        break;
      }
    } else {
      bail = true;
      break;
    }
    lbits = zs_u(lbits);
    dbits = zs_u(dbits);
    const zcode* lt = W.codes;
    const zcode* dt = W.codes + zs_u(lused);
    for (;;) {
      zcode here = zs_wr_decode(R, lt, lbits);
      uint32_t op = C_OP(here);
      if (op == 0) {
        if (total >= piece_cap) { bail = true; break; }
        if (lane == 0) ring[total & rmask] = (uint16_t)C_VAL(here);
        total++;
        flush();
        continue;
      }
      if (op & 32) break;                   // end of block
      if (op & 64) { bail = true; break; }  // invalid literal/length code
      const uint32_t len = C_VAL(here) + zs_wr_take(R, op & lmask);
      here = zs_wr_decode(R, dt, dbits);
      op = C_OP(here);
      if (op & 64) { bail = true; break; }  // invalid distance code
      const uint32_t dist = C_VAL(here) + zs_wr_take(R, op & 15u);
      if (dist > wsize || total + len > piece_cap) { bail = true; break; }
      bool bad = false;
      // in pieces of at most half the ring, each flushed before the next (a
      // deflate64 length-285 copy is up to 65,538 values: longer than the ring)
      for (uint32_t left = len; left;) {
        const uint32_t pn = min(left, 32768u);
        if (dist >= 64 || dist >= pn) {
          for (uint32_t i = 0; i < pn; i += 64) {
            const uint32_t j = i + lane;
            if (j < pn) ring[(total + j) & rmask] = (uint16_t)hist(total + j, dist, bad);
          }
        } else {
          // period dist < 64: lane j < step (a multiple of dist) stores the value dist - j % dist back
          const uint32_t per = 64u / dist, step = per * dist;
          const uint32_t mm = lane - (lane / dist) * dist;
          const uint16_t b = (uint16_t)hist(total + mm, dist, bad);
          for (uint32_t i = 0; i < pn; i += step) {
            const uint32_t j = i + lane;
            if (lane < step && j < pn) ring[(total + j) & rmask] = b;
          }
        }
        total += pn;
        left -= pn;
        flush();
      }
      if (__builtin_amdgcn_ballot_w64(bad)) { bail = true; break; }
    }
    if (zs_wr_over(R)) bail = true;
  }
  if (!bail) {
    const uint32_t wend = (total + 1u) >> 1;
    for (uint32_t w = (flushed >> 1) + lane; w < wend; w += 64) dstw[w] = ringw[w & (rmask >> 1)];
  }
  if (lane == 0) {
    zs_split_piece_res r;
    r.end = zs_wr_bitpos(R);
    r.count = total;
    r.flags = (bail ? ZS_SPLIT_BAIL : 0u) | (last && !bail ? ZS_SPLIT_FINAL : 0u);
    r.next = next;
    r.pad = 0;
    pres[blockIdx.x] = r;
  }
}

// ---------------------------------------------------------------- resolver
// zs_k_split_chain (a thread per member): the chain -- piece 0, then the piece
// each one stopped at, to the final block -- and the pieces' places by a prefix
// sum of their lengths.
__global__ void zs_k_split_chain(const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ out_cap,
                                 const uint32_t* __restrict__ list, uint32_t n_list,
                                 const zs_split_piece_res* __restrict__ pres, zs_split_member* __restrict__ mem) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_list) return;
  const uint32_t s = list[m];
  const uint64_t nbits = 8ull * in_len[s];
  zs_split_member& M = mem[m];
  bool ok = false;
  uint32_t c = 0, j = 0;
  uint64_t tot = 0, end = 0;
  while (c < ZS_SPLIT_MAX) {
    const zs_split_piece_res p = pres[m * ZS_SPLIT_MAX + j];
    if (p.flags & ZS_SPLIT_BAIL) break;
    M.piece[c] = j;
    M.off[c++] = (uint32_t)tot;
    tot += p.count;
    if (p.flags & ZS_SPLIT_FINAL) {
      ok = p.end <= nbits;
      end = p.end;
      break;
    }
    if (p.next <= j || p.next >= ZS_SPLIT_MAX) break;
    j = p.next;
  }
  if (tot > out_cap[s]) ok = false;
  M.nchain = ok ? c : 0u;
  M.total = ok ? (uint32_t)tot : 0u;
  M.consumed = (uint32_t)((end + 7u) >> 3);
  M.bad = ok ? 0u : 1u;
}

// zs_k_split_place (a workgroup per piece): the pieces' values at their
// places in the member's u32 value array -- a byte, or 0x80000000 | the
// absolute position a marker names
__global__ __launch_bounds__(256) void zs_k_split_place(const zs_split_piece_res* __restrict__ pres,
                                                       zs_split_member* __restrict__ mem,
                                                       const uint16_t* __restrict__ scratch, uint32_t piece_cap,
                                                       uint32_t* __restrict__ val, uint64_t val_stride) {
  const uint32_t m = blockIdx.x / ZS_SPLIT_MAX, j = blockIdx.x % ZS_SPLIT_MAX;
  zs_split_member& M = mem[m];
  if (j >= M.nchain) return;
  const uint32_t pj = M.piece[j], o = M.off[j], cnt = pres[m * ZS_SPLIT_MAX + pj].count;
  const uint16_t* v = scratch + (size_t)(m * ZS_SPLIT_MAX + pj) * piece_cap;
  uint32_t* V = val + (size_t)m * val_stride;
  bool bad = false;
  for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
    const uint32_t x = v[i];
    uint32_t y = x;
    if (x >= 256u) {
      const uint32_t back = x - 255u;
      bad |= back > o;  // before the member's start: a real "too far back" (the exact kernel reports it)
      y = 0x80000000u | (o - back);
    }
    V[o + i] = y;
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) M.bad = 1u;
}

// zs_k_split_jump: one round of pointer jumping over every marker (a marker
// names a byte of an earlier piece, which may be a marker itself: chains are at
// most as long as the member has pieces, so log2(ZS_SPLIT_MAX) rounds end them)
__global__ __launch_bounds__(256) void zs_k_split_jump(const zs_split_member* __restrict__ mem,
                                                      uint32_t* __restrict__ val, uint64_t val_stride) {
  const uint32_t m = blockIdx.y;
  const zs_split_member& M = mem[m];
  if (M.bad) return;
  uint32_t* V = val + (size_t)m * val_stride;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < M.total; p += gridDim.x * blockDim.x) {
    const uint32_t x = V[p];
    if (x & 0x80000000u) V[p] = V[x & 0x7fffffffu];
  }
}

// zs_k_split_write: the bytes, four per thread (out_off is 4-aligned and the
// last word's bytes past the end lie inside the capacity), and the outcome
__global__ __launch_bounds__(256) void zs_k_split_write(const uint32_t* __restrict__ list,
                                                       zs_split_member* __restrict__ mem,
                                                       const uint32_t* __restrict__ val, uint64_t val_stride,
                                                       uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off) {
  const uint32_t m = blockIdx.y;
  zs_split_member& M = mem[m];
  if (M.bad) return;
  const uint32_t* V = val + (size_t)m * val_stride;
  uint32_t* dst = reinterpret_cast<uint32_t*>(out + out_off[list[m]]);
  const uint32_t nw = (M.total + 3u) >> 2;
  bool left = false;  // a marker the rounds did not resolve
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
    uint32_t x = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t p = 4u * w + k;
      const uint32_t v = p < M.total ? V[p] : 0u;
      left |= (v & 0x80000000u) != 0;
      x |= (v & 0xffu) << (8u * k);
    }
    dst[w] = x;
  }
  if (__syncthreads_or(left) && threadIdx.x == 0) atomicOr(&M.bad, 1u);
}

__global__ void zs_k_split_final(const uint32_t* __restrict__ list, uint32_t n_list,
                                 const zs_split_member* __restrict__ mem, zs_lane_res* __restrict__ res,
                                 uint32_t* __restrict__ lens_out) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_list) return;
  const zs_split_member& M = mem[m];
  zs_lane_res r = {1u, 0u, 0u, 0u};
  if (!M.bad) {
    r.bail = 0;
    r.out_len = M.total;
    r.consumed = M.consumed;
  }
  res[list[m]] = r;
  lens_out[list[m]] = r.out_len;
}

size_t zs_split_lds_bytes(bool d64) { return (d64 ? 131072u : 65536u) + sizeof(zs_split_tabs); }
