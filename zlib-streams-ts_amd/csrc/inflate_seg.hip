// inflate_seg.hip -- the segmented decode: one member's symbols decoded by many
// LANES at once, for batches whose members are too few to fill the chip one lane
// (inflate_lane.hip) or one wave (inflate_wave.hip) per member -- the per-rank
// shards of the 8-GPU configs (512 x 256 KiB, 1,024 x 64 KiB).
//
// A member's decode is one serial chain of Huffman lookups; three facts cut it:
//  * inside a block, Huffman decoding started at an arbitrary bit falls into
//    step with the true symbol stream after a few symbols (median 100 bits,
//    max ~1,750 over 7,800 trials on the benchmark corpora): a lane decoding
//    from the block's true start reaches, past the next lane's start, a symbol
//    start that lane also visited -- from there both are the true stream;
//  * a copy reaching back before a piece's start can be written as a MARKER
//    (u16 255 + k: "the value k positions before the piece"), propagated by
//    later copies like a byte, and resolved once the earlier pieces are known;
//  * for members too long for one walk, block starts can be found by testing
//    every bit offset (zs_k_split_find), and walks started there.
// The reference's window-wrap copy (inffast.ts:127-147, reproduced by default)
// depends on its inflate() call boundaries (32 KiB input sub-chunks, 64 KiB
// output buffers, streams.ts:78-93): they move only at "events" -- the first
// symbol ending past a sub-chunk end, the first symbol reaching a full buffer
// -- so the call state at every piece start follows from each piece's output
// count, events and last symbol length (tools/emu/emu_seg.py checks this plan
// against the serial bookkeeping and the oracle), and each piece replays the
// bookkeeping (zs_refcalls) from its start.
//
// Kernels, each over the whole batch:
//  zs_k_split_find  (members over ZS_SEG_BIG_BITS only) candidate block starts,
//                   one per bit range (inflate_split.hip)
//  zs_k_seg_walk    one wave per entry (a member's start; a big member's found
//                   block starts): block after block, header and tables, then
//                   spans of 64 lanes, lane j decoding from bit sym0 + j S and
//                   recording the symbol starts of its first ZS_SEG_W bits; it
//                   stops at the first of its positions (past the next lane's
//                   start) that the next lane recorded.  Output counts,
//                   crossing events, the span's end (end of block, or the next
//                   span's start); the walk stops at the final block or at a
//                   later entry's start.
//  zs_k_seg_plan    one wave per member: entries chained by their ends, the
//                   pieces placed (prefix sum), trailer and capacity checked,
//                   call state per piece (REFW)
//  zs_k_seg_decode  one wave per span: each lane decodes its piece into u16
//                   values (bytes or markers) with the window-wrap copy replayed
//  zs_k_seg_resolve one workgroup per member: pieces in order, markers looked up
//                   in the bytes already final (a 64 KiB LDS ring), bytes written
// A stored block is one piece, its bytes copied from the input by the decode.
// Any doubt -- no chain of blocks, a lane that never
// synchronises, an invalid code or "too far back" in a piece, a marker further
// back than a u16 says -- marks the member bad; the host then runs the
// wave kernel over it (and that the exact kernel), so outcomes stay the reference's.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_inflate.h"
#include "zs_inftab.h"
#include "zs_wave.h"
#include "zs_refcalls.h"
#include "zs_seg.h"

#ifndef ZS_SEG_EXP
#define ZS_SEG_EXP 0  // instrumentation (timing experiments only; 0 in the product): 1 per-span decode clocks,
                      // 2 per-entry walk clocks (tools/dbg/seg_walk_clock.py)
#endif
#if ZS_SEG_EXP & 2
#define ZS_SEG_WDBG_N 65536u
// per entry: header cycles, span phase-1 cycles (lanes decoding alone), span sync + record cycles, blocks,
// spans, phase-1 symbols of the busiest lane (summed over spans), all cycles, bad-code reseeks
__device__ unsigned long long zs_seg_wdbg[ZS_SEG_WDBG_N][8];
extern "C" int zs_seg_wdbg_fetch(void* out, unsigned long long bytes) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_seg_wdbg),
                                  bytes < sizeof(zs_seg_wdbg) ? bytes : sizeof(zs_seg_wdbg));
}
#endif

#if ZS_SEG_EXP & 16
// header sub-phases, summed over all headers: code-length table, code-length decode, lit/len table, dist table, headers
__device__ unsigned long long zs_seg_hdbg[8];
extern "C" int zs_seg_hdbg_fetch(void* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_seg_hdbg), sizeof(zs_seg_hdbg));
}
#define HD_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define HD_ADD(i, a, b) do { if ((threadIdx.x & 63u) == 0) atomicAdd(&zs_seg_hdbg[i], (b) - (a)); } while (0)
#else
#define HD_T(v) do { } while (0)
#define HD_ADD(i, a, b) do { } while (0)
#endif

// ------------------------------------------------------------- lane reader
// One lane's bit reader (the lane kernel's scheme: clamped aligned words, one
// refill ahead, zero past the end), started at any bit; member bit positions
// fit 32 bits (the host sends members under 512 MB here).
struct zs_sg_reader {
  const uint32_t* w4;
  uint32_t sh, last, n;
  uint32_t pos;  // bytes moved into hold (a multiple of 4)
  uint64_t hold;
  uint32_t bits;
  uint32_t pf;
};
static __device__ __forceinline__ uint32_t zs_sg_load4(const zs_sg_reader& R, uint32_t at) {
#if ZS_SEG_EXP & 4  // (timing: input words made up in registers instead of loaded -- garbage decodes)
  return at * 2654435761u;
#endif
  const uint32_t q = (at + R.sh) >> 2;
  const uint32_t lo = R.w4[min(q, R.last)], hi = R.w4[min(q + 1u, R.last)];
  const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, R.sh);
  const uint32_t valid = at < R.n ? R.n - at : 0u;
  return valid >= 4u ? v : v & ((1u << (8u * valid)) - 1u);
}
static __device__ __forceinline__ void zs_sg_fill(zs_sg_reader& R) {
  R.hold |= (uint64_t)R.pf << R.bits;
  R.bits += 32;
  R.pos += 4;
  R.pf = zs_sg_load4(R, R.pos);
}
static __device__ __forceinline__ void zs_sg_drop(zs_sg_reader& R, uint32_t k) {
  R.hold >>= k;
  R.bits -= k;
}
static __device__ __forceinline__ void zs_sg_seek(zs_sg_reader& R, uint32_t bit) {
  R.pos = (bit >> 5) << 2;
  R.hold = 0;
  R.bits = 0;
  R.pf = zs_sg_load4(R, R.pos);
  zs_sg_fill(R);
  zs_sg_drop(R, bit & 31u);
}
static __device__ __forceinline__ uint32_t zs_sg_bitpos(const zs_sg_reader& R) { return R.pos * 8u - R.bits; }
static __device__ __forceinline__ uint32_t zs_sg_take(zs_sg_reader& R, uint32_t k) {  // k <= 32
  if (R.bits < k) zs_sg_fill(R);
  const uint32_t v = (uint32_t)R.hold & (k == 32 ? 0xffffffffu : ((1u << k) - 1u));
  zs_sg_drop(R, k);
  return v;
}
static __device__ __forceinline__ void zs_sg_init(zs_sg_reader& R, const uint8_t* src, uint32_t n) {
  R.n = n;
  R.sh = (uint32_t)((uintptr_t)src & 3u);
  R.w4 = reinterpret_cast<const uint32_t*>(src - R.sh);
  R.last = (R.sh + n - 1u) >> 2;
}
// a code from a zlib table (second level included); nb: its bits
template <typename TT>
static __device__ __forceinline__ zcode zs_sg_code(zs_sg_reader& R, const TT& t, uint32_t mask, uint32_t& nb) {
  zcode here = t[(uint32_t)R.hold & mask];
  uint32_t b = C_BITS(here);
  if (C_OP(here) && (C_OP(here) & 0xf0) == 0) {
    const uint32_t rb = b;
    here = t[C_VAL(here) + (((uint32_t)R.hold & ((1u << (rb + C_OP(here))) - 1u)) >> rb)];
    b = rb + C_BITS(here);
  }
  zs_sg_drop(R, b);
  nb = b;
  return here;
}
// one symbol (inffast.ts:5-228 decode, inflate.ts LEN..DISTEXT for deflate64)
#define ZS_SG_LIT 0u
#define ZS_SG_COPY 1u
#define ZS_SG_EOB 2u
#define ZS_SG_BAD 3u
struct zs_sg_sym {
  uint32_t kind, val, len;  // literal: val; copy: len, val = distance
  uint32_t l1, e1, l2, e2;  // the bit fields (zs_refcalls)
};
template <typename TD>
static __device__ __forceinline__ zs_sg_sym zs_sg_decode(zs_sg_reader& R, const zcode* lt, uint32_t lmask,
                                                        const TD& dt, uint32_t dmask, uint32_t emask) {
  zs_sg_sym y = {ZS_SG_BAD, 0u, 0u, 0u, 0u, 0u, 0u};
  if (R.bits < 32) zs_sg_fill(R);
  zcode here = zs_sg_code(R, lt, lmask, y.l1);
  uint32_t op = C_OP(here);
  if (op == 0) {
    y.kind = ZS_SG_LIT;
    y.val = C_VAL(here);
    y.len = 1;
    return y;
  }
  if (op & 32) {
    y.kind = ZS_SG_EOB;
    return y;
  }
  if (op & 64) return y;  // "invalid literal/length code"
  y.e1 = op & emask;
  y.len = C_VAL(here) + zs_sg_take(R, y.e1);
  if (R.bits < 32) zs_sg_fill(R);
  here = zs_sg_code(R, dt, dmask, y.l2);
  op = C_OP(here);
  if (op & 64) return y;  // "invalid distance code"
  y.e2 = op & 15u;
  y.val = C_VAL(here) + zs_sg_take(R, y.e2);
  y.kind = ZS_SG_COPY;
  return y;
}

// The block header at the wave reader's position (inflate.ts:600-836) into
// zlib's tables (inflate_table) in LDS, as zs_k_inflate_wave; a stored block's
// length (inflate.ts:631-672: LEN and NLEN at the next byte boundary, the reader
// left at its first byte) in slen, else ZS_SEG_NONE; false for anything invalid
// (the member then takes the other paths).
static __device__ bool zs_sg_header(zs_wave_reader& R, zcode* codes, uint16_t* lens, uint16_t* work, bool d64,
                                    uint32_t& last, uint32_t& lbits, uint32_t& dbits, uint32_t& dofs,
                                    uint32_t& ntab, uint32_t& slen) {
  last = zs_wr_take(R, 1);
  const uint32_t type = zs_wr_take(R, 2);
  uint32_t lused = 0, dused = 0;
  slen = ZS_SEG_NONE;
  if (type == 0) {
    zs_wr_align(R);
    const uint32_t len = zs_wr_take(R, 16), nlen = zs_wr_take(R, 16);
    if (len != (nlen ^ 0xffffu) || zs_wr_over(R)) return false;  // "invalid stored block lengths", or past the input
    slen = len;
    return true;
  }
  if (type == 1) {  // fixed tables (inflate.ts:218-280)
    uint32_t sym;
    for (sym = 0; sym < 144; sym++) lens[sym] = 8;
    for (; sym < 256; sym++) lens[sym] = 9;
    for (; sym < 280; sym++) lens[sym] = 7;
    for (; sym < 288; sym++) lens[sym] = 8;
    lbits = 9;
    zs_inflate_table_wave<false>(LENS, lens, 288, codes, &lbits, work, d64, &lused);
    for (sym = 0; sym < 32; sym++) lens[sym] = 5;
    dbits = 5;
    zs_inflate_table_wave<false>(DISTS, lens, 32, codes + lused, &dbits, work, d64, &dused);
  } else if (type == 2) {  // dynamic (inflate.ts:662-836)
    const uint32_t nlen = zs_wr_take(R, 5) + 257, ndist = zs_wr_take(R, 5) + 1, ncode = zs_wr_take(R, 4) + 4;
    if (nlen > 286 || (!d64 && ndist > 30)) return false;
    uint32_t i;
    for (i = 0; i < ncode; i++) lens[ZS_BL_ORDER[i]] = (uint16_t)zs_wr_take(R, 3);
    for (; i < 19; i++) lens[ZS_BL_ORDER[i]] = 0;
    uint32_t cbits = 7, used;
    HD_T(t0);
    if (zs_inflate_table_wave<false>(CODES, lens, 19, codes, &cbits, work, d64, &used)) return false;
    HD_T(t1);
    // The code lengths (inflate.ts:702-778), one symbol at a time but with no
    // memory round trip per symbol: the code-length code's table (<= 128
    // entries of bits << 8 | symbol) sits in a VGPR, lane l holding entries l
    // and l + 64, read with v_readlane at the input's next cbits bits; a repeat
    // is stored by up to 138 lanes at once; the previous length stays in a
    // register.  (Was an LDS lookup and readfirstlane per symbol and a store
    // per repeated length: ~44k core cycles per header, profiles/r06/hdr/.)
    const uint32_t lane = threadIdx.x & 63u, csz = 1u << cbits, cmask = csz - 1u, N = nlen + ndist;
    const zcode c0 = lane < csz ? codes[lane] : 0u, c1 = lane + 64u < csz ? codes[lane + 64u] : 0u;
    const uint32_t tv = ((C_BITS(c0) << 8) | C_VAL(c0)) | (((C_BITS(c1) << 8) | C_VAL(c1)) << 16);
    uint32_t prev = 0;
    i = 0;
    while (i < N) {
      if (R.bits < 32) zs_wr_fill(R);
      const uint32_t idx = (uint32_t)R.hold & cmask;
      const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)tv, (int)(idx & 63u));
      const uint32_t e = (idx & 64u) ? e2 >> 16 : e2 & 0xffffu;
      const uint32_t nb = e >> 8, v = e & 0xffu;
      R.hold >>= nb;
      R.bits -= nb;
      if (v < 16) {
        lens[i++] = (uint16_t)v;
        prev = v;
        continue;
      }
      uint32_t rep, val = 0;
      if (v == 16) {
        if (i == 0) return false;
        val = prev;
        rep = 3 + zs_wr_take(R, 2);
      } else if (v == 17) {
        rep = 3 + zs_wr_take(R, 3);
      } else {
        rep = 11 + zs_wr_take(R, 7);
      }
      if (i + rep > N) return false;
      for (uint32_t j = lane; j < rep; j += 64u) lens[i + j] = (uint16_t)val;
      i += rep;
      prev = val;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // (the lengths visible to this wave's table builds)
    __builtin_amdgcn_wave_barrier();
    if (zs_wr_over(R) || zs_u(lens[256]) == 0) return false;
    HD_T(t2);
    lbits = 9;
    if (zs_inflate_table_wave<false>(LENS, lens, nlen, codes, &lbits, work, d64, &lused)) return false;
    HD_T(t3);
    dbits = 6;
    if (zs_inflate_table_wave<false>(DISTS, lens + nlen, ndist, codes + lused, &dbits, work, d64, &dused)) return false;
    HD_T(t4);
    HD_ADD(0, t0, t1);
    HD_ADD(1, t1, t2);
    HD_ADD(2, t2, t3);
    HD_ADD(3, t3, t4);
    HD_ADD(4, 0ull, 1ull);
    HD_ADD(5, 0ull, (unsigned long long)(nlen + ndist));
  } else {
    return false;  // "invalid block type"
  }
  lbits = zs_u(lbits);
  dbits = zs_u(dbits);
  dofs = zs_u(lused);
  ntab = zs_u(lused + dused);
  return true;
}

// ------------------------------------------------------------------- walk
// One wave per ENTRY: entry 0 of every member is its first bit; a member with
// more than ZS_SEG_BIG_BITS input bits also has the block starts the finder
// found (zs_k_split_find, one per bit range) as entries 1 ..  An entry's wave
// walks the blocks from its start in order -- header and tables, then the
// block's symbols in SPANS of 64 lanes, lane j decoding from sym0 + j S -- until
// a block ends at a later entry's start (the plan links them there) or the final
// block ends.  Within a span, lane j records the symbol starts of the first
// ZS_SEG_W bits of its range and stops at the first of its positions, past the
// next lane's start, that the next lane recorded: from there both decode the
// true stream (the lane before is confirmed, so is it).  The span ends at the
// end-of-block code of a confirmed lane, or -- its last lane confirmed past the
// span's nominal end -- at a symbol start, where the next span continues.
// (a checkpoint: the position's offset in its window | the lane's output count << 12;
// a count past 2^20 -- garbage only -- comes out wrong, which the decode's count check catches)
#define ZS_SG_CK(off, cum) ((off) | ((cum) << 12))
template <uint32_t W>
struct zs_sg_walk_lds {
  zcode codes[ZS_SEG_TAB];
  union {
    struct {  // a block header (between spans)
      uint32_t inw[ZS_WIN_IN];
      uint16_t lens[320];
      uint16_t work[288];
    } h;
    struct {  // a span
      uint32_t own[ZS_SEG_LANES][W / 32];   // each lane's symbol starts in [q, q + W)
      uint32_t tail[ZS_SEG_LANES][W / 32];  // ... and in [q + S, q + S + W): the next lane's window
      uint32_t ock[ZS_SEG_LANES][W / ZS_SEG_CKB];  // checkpoints in each (ZS_SG_CK)
      uint32_t tck[ZS_SEG_LANES][W / ZS_SEG_CKB];
    } s;
  };
#if ZS_SEG_EXP & 2
  unsigned long long dbg[4];  // phase-1 cycles, rest cycles, busiest lane's symbols, reseeks (this span)
#endif
  uint32_t sync[ZS_SEG_LANES];  // lane j's start on the true stream: the first start it shares with lane j - 1
  uint32_t odone[ZS_SEG_LANES];  // words of own[j] complete (lane j has moved past them)
  uint32_t send;
};

// One span of a block whose tables are in L.codes: lanes j < nl decode from
// q_j = sym0 + j S; pe0 is the end of the symbol before sym0 (sub-chunk events).
//  1. every lane decodes on its own -- no barrier, no exchange -- from q_j to
//     the first symbol start at or past q_{j+1} + W (the last lane: past the
//     span's nominal end, or to the input's end when the span reaches it),
//     recording its symbol starts in [q_j, q_j + W) and in [q_{j+1}, q_{j+1} + W),
//     with checkpoints of its output count, its end-of-block / invalid codes
//     and its sub-chunk crossings;
//  2. lane j's true start is the first symbol start lane j - 1 recorded in
//     [q_j, q_j + W) that lane j recorded too (lane 0 starts on the true stream,
//     so by induction each lane from its start does);
//  3. the chain is lanes 0 .. J - 1 (J: the first lane without a shared start);
//     the first of them whose piece holds an end-of-block code ends the block
//     there (BEND); else the span ends at the last chain lane's stop, a true
//     symbol start where the next span continues (CONT) -- past the nominal end,
//     or, the chain broken at J, past q_J + W.
// Writes the span's lane records; returns BEND / CONT, or NONE for a span that
// cannot go on (past the input without an end of block).
#define ZS_SG_K_NONE 0u
#define ZS_SG_K_BEND 2u
#define ZS_SG_K_CONT 4u
template <bool D64, uint32_t W, bool ST>
static __device__ uint32_t zs_sg_span(zs_sg_walk_lds<W>& L, const uint8_t* src, uint32_t n, uint32_t sym0, uint32_t pe0,
                                      uint32_t nl, uint32_t S, uint32_t lbits, uint32_t dbits, uint32_t dofs,
                                      zs_seg_lane* __restrict__ recs, uint32_t& send, bool& bad_out, bool split) {
  const uint32_t lane = threadIdx.x;
#if ZS_SEG_EXP & 2
  const unsigned long long dbg_t0 = __builtin_readcyclecounter();
  uint32_t dbg_sym = 0, dbg_seek = 0;
#endif
  const uint32_t nbits = 8u * n;
  const uint32_t nend = sym0 + nl * S;  // the nominal end
  const bool cont_ok = nend < nbits;    // (else the block must end in this span)
  const uint32_t lmask = (1u << lbits) - 1u, dmask = (1u << dbits) - 1u, emask = D64 ? 31u : 15u;
  const zcode* lt = L.codes;
  const zcode* dt = L.codes + dofs;
  const bool on = lane < nl;
  const bool lastl = lane + 1u == nl;
  const uint32_t q = sym0 + lane * S, qn = q + S;
  const uint32_t lim = !on ? q : !lastl ? qn + W : cont_ok ? nend : nbits + 64u;
  for (uint32_t i = 0; i < W / 32; i++) {
    L.s.own[lane][i] = 0;
    L.s.tail[lane][i] = 0;
  }
  for (uint32_t i = 0; i < (W / ZS_SEG_CKB); i++) {
    L.s.ock[lane][i] = ZS_SEG_NONE;
    L.s.tck[lane][i] = ZS_SEG_NONE;
  }
  L.odone[lane] = 0;
  // (LDS-typed: through a generic pointer a volatile access is a flat one, waited for with vmcnt(0) -- the
  // input prefetch included)
  typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
  lds_vu32* const vodone = (lds_vu32*)L.odone;
  lds_vu32* const vown_next = (lds_vu32*)(lane + 1u < nl ? L.s.own[lane + 1u] : L.s.own[lane]);
  bool left_own = false;
  // ---- 1. the lane's own decode
  zs_sg_reader G;
  zs_sg_init(G, src, n);
  if (on) zs_sg_seek(G, q);
  uint32_t pos = q, cum = 0, last_len = 0;
  uint32_t pe = lane == 0 ? pe0 : q;  // the end of the symbol before (events)
  uint32_t nev = 0, ev_k[ZS_SEG_NEV], ev_sb[ZS_SEG_NEV], ev_c[ZS_SEG_NEV];
  // end-of-block and invalid codes: those in [q, q + W) (where the garbage before
  // the lane's true start is) in rings of the last ZS_SEG_NEOB, and the first one
  // past it (in the true stream once the lane is on the chain)
  uint32_t neob = 0, eob_sb[ZS_SEG_NEOB], eob_end[ZS_SEG_NEOB], eob_cum[ZS_SEG_NEOB];
  uint32_t xeob_sb = ZS_SEG_NONE, xeob_end = 0, xeob_cum = 0;
  uint32_t nbad = 0, bad_sb[ZS_SEG_NEOB], xbad = ZS_SEG_NONE;
#pragma unroll
  for (uint32_t e = 0; e < ZS_SEG_NEV; e++) ev_k[e] = ev_sb[e] = ev_c[e] = 0;
#pragma unroll
  for (uint32_t e = 0; e < ZS_SEG_NEOB; e++) eob_sb[e] = eob_end[e] = eob_cum[e] = bad_sb[e] = 0;
  uint32_t ock = 0, tck = 0;  // checkpoint buckets filled
  // split mode: the first symbol start at or past the lane's middle, the output count there, the symbol before's
  const uint32_t qm = split ? q + S / 2u : ZS_SEG_NONE;
  uint32_t mid_sb = ZS_SEG_NONE, mid_cum = 0, mid_ll = 0;
  // the bitmaps' current word (own words 0 .., tail words W / 32 ..) collects
  // in a register: positions only grow, so each word is stored once
  constexpr uint32_t NW = W / 32u;
  uint32_t aw = ZS_SEG_NONE, acc = 0;
  auto put_word = [&]() {
    if (aw < NW) L.s.own[lane][aw] = acc;
    else if (aw != ZS_SEG_NONE) L.s.tail[lane][aw - NW] = acc;
  };
  auto mark = [&](uint32_t w, uint32_t bit) {
    if (w != aw) {
      put_word();
      if (w < NW) {  // own words below w are final: the lane before may stop on them
        asm volatile("" ::: "memory");
        vodone[lane] = w;
      }
      aw = w;
      acc = 0;
    }
    acc |= 1u << bit;
  };
  bool nofast = false;  // the stretch below stopped at this lane's end-of-block / invalid code
  // (ST: the walk instance for large members -- the 4,096 x 256 KiB walk 5.96 -> 5.49 ms; C5-i's 64 KiB
  // members, 2,048-bit spans, lose 4 % with this code in the loop at all: their instance has none)
  constexpr bool stretches = ST;
  while (pos < lim) {
#if !(ZS_SEG_EXP & 32)
    // The stretch between a lane's two windows: no marks, no checkpoints and --
    // 64 bits (more than a symbol) short of the tail window, the split point and
    // the next sub-chunk boundary -- no events.  When EVERY running lane is in its
    // stretch, the wave decodes literals and copies without that bookkeeping until
    // one of them leaves it (an end-of-block or invalid code seeks back and leaves
    // that symbol to the loop below).  The extra bits need no refill: >= 32 bits
    // are held before a code of <= 15 bits and <= 16 extra bits.
    if (stretches && __builtin_amdgcn_ballot_w64(left_own && !nofast) == __builtin_amdgcn_read_exec()) {
      uint32_t bdn = (pos + 262143u) & ~262143u;
      if (bdn == 0) bdn = 262144u;
      uint32_t fe = min(min(qn, lim), bdn);
      if (mid_sb == ZS_SEG_NONE) fe = min(fe, qm);
      const bool in = fe > pos + 64u;
      const uint64_t run = __builtin_amdgcn_read_exec();
      if (__builtin_amdgcn_ballot_w64(in) == run) {
        const uint32_t fend = fe - 64u;
        bool stay;
        do {
          if (G.bits < 32) zs_sg_fill(G);
          uint32_t nb;
          zcode here = zs_sg_code(G, lt, lmask, nb);
          uint32_t op = C_OP(here), len = 1u;
          bool stop = false;
          if (op) {
            if (op & 96u) {  // end of block / invalid
              stop = true;
            } else {
              const uint32_t e1 = op & emask;
              len = C_VAL(here) + ((uint32_t)G.hold & ((1u << e1) - 1u));
              zs_sg_drop(G, e1);
              if (G.bits < 32) zs_sg_fill(G);
              here = zs_sg_code(G, dt, dmask, nb);
              op = C_OP(here);
              stop = (op & 64u) != 0;  // invalid distance
              zs_sg_drop(G, op & 15u);
            }
          }
          if (stop) {
            zs_sg_seek(G, pos);
            nofast = true;
          } else {
#if ZS_SEG_EXP & 2
            dbg_sym++;
#endif
            cum += len;
            last_len = len;
            pos = zs_sg_bitpos(G);
          }
          stay = !stop && pos < fend;
        } while (__builtin_amdgcn_ballot_w64(stay) == run);
        pe = pos;
        continue;
      }
    }
    nofast = false;
#endif
    const uint32_t off = pos - q, toff = pos - qn;
    if (pos >= qm && mid_sb == ZS_SEG_NONE) {
      mid_sb = pos;
      mid_cum = cum;
      mid_ll = last_len;
    }
    if (off < W) {
      mark(off >> 5, off & 31u);
      if (off >= ock * ZS_SEG_CKB) {
        L.s.ock[lane][off / ZS_SEG_CKB] = ZS_SG_CK(off, cum);
        ock = off / ZS_SEG_CKB + 1u;
      }
    } else {
      if (!left_own) {  // own[] complete
        put_word();
        aw = ZS_SEG_NONE;
        asm volatile("" ::: "memory");
        vodone[lane] = NW;
        left_own = true;
      }
      if (toff < W) {
        mark(NW + (toff >> 5), toff & 31u);
        if (toff >= tck * ZS_SEG_CKB) {
          L.s.tck[lane][toff / ZS_SEG_CKB] = ZS_SG_CK(toff, cum);
          tck = toff / ZS_SEG_CKB + 1u;
        }
        // a start the next lane has recorded (its window complete): the two meet here
        // or earlier (step 2 finds the first), the rest of the tail is not needed
        if (lane + 1u < nl && (toff >> 5) < vodone[lane + 1u] && ((vown_next[toff >> 5] >> (toff & 31u)) & 1u)) break;
      }
    }
    const uint32_t sb = pos;
    const zs_sg_sym y = zs_sg_decode(G, lt, lmask, dt, dmask, emask);
#if ZS_SEG_EXP & 2
    dbg_sym++;
    dbg_seek += y.kind == ZS_SG_BAD ? 1u : 0u;
#endif
    if (y.kind == ZS_SG_BAD) {
      if (sb - q < W) {
#pragma unroll
        for (uint32_t e = 0; e < ZS_SEG_NEOB; e++)
          if (e == (nbad & (ZS_SEG_NEOB - 1u))) bad_sb[e] = sb;
        nbad++;
      } else if (xbad == ZS_SEG_NONE) {
        xbad = sb;
      }
      pos = sb + 1u;
      zs_sg_seek(G, pos);
      pe = pos;
      last_len = 0;
      continue;
    }
    const uint32_t se = zs_sg_bitpos(G);
    // sub-chunk crossing events: boundaries 262144 k (k >= 1) with pe <= b < se
    uint32_t bd = (pe + 262143u) & ~262143u;
    if (bd == 0) bd = 262144u;
    while (bd < se) {
#pragma unroll
      for (uint32_t e = 0; e < ZS_SEG_NEV; e++)
        if (e == nev) {
          ev_k[e] = bd >> 18;
          ev_sb[e] = sb;
          ev_c[e] = cum;
        }
      nev++;
      bd += 262144u;
    }
    if (y.kind == ZS_SG_EOB) {
      // (an end of block running past the input is never the true one: the last lane
      // decodes on past the end, where a 1-bit code's zeros would fill the ring --
      // the deflate64 fixture payload_63k)
      if (se > nbits) {
      } else if (sb - q < W) {
#pragma unroll
        for (uint32_t e = 0; e < ZS_SEG_NEOB; e++)
          if (e == (neob & (ZS_SEG_NEOB - 1u))) {
            eob_sb[e] = sb;
            eob_end[e] = se;
            eob_cum[e] = cum;
          }
        neob = min(neob + 1u, 2u * ZS_SEG_NEOB);  // (a ring: the last ZS_SEG_NEOB)
      } else if (xeob_sb == ZS_SEG_NONE) {
        xeob_sb = sb;
        xeob_end = se;
        xeob_cum = cum;
      }
      last_len = 0;
    } else {
      cum += y.len;
      last_len = y.len;
    }
    pe = se;
    pos = se;
  }
  put_word();
  __syncthreads();
#if ZS_SEG_EXP & 2
  const unsigned long long dbg_t1 = __builtin_readcyclecounter();
  if (lane == 0) {
    L.dbg[0] = dbg_t1 - dbg_t0;
    L.dbg[2] = 0;
    L.dbg[3] = 0;
  }
  __syncthreads();
  atomicMax(&L.dbg[2], (unsigned long long)dbg_sym);
  atomicAdd(&L.dbg[3], (unsigned long long)dbg_seek);
#endif
  // ---- 2. each lane's true start: the first start in its window lane - 1 shares
  uint32_t sp = lane == 0 ? sym0 : ZS_SEG_NONE;
  if (on && lane) {
    for (uint32_t i = 0; i < W / 32; i++) {
      const uint32_t x = L.s.tail[lane - 1u][i] & L.s.own[lane][i];
      if (x) {
        sp = q + 32u * i + (uint32_t)__builtin_ctz(x);
        break;
      }
    }
  }
  L.sync[lane] = sp;
  __syncthreads();
  // ---- 3. the chain: lanes 0 .. J - 1
  const uint64_t nos = __builtin_amdgcn_ballot_w64(on && sp == ZS_SEG_NONE);
  const uint32_t J = nos ? (uint32_t)__builtin_ctzll(nos) : nl;
  const bool chain = lane < J;
  const uint32_t start = sp;
  // the piece's end before any end of block: the next lane's start, or (the chain's
  // last lane) its stop
  const uint32_t nxs = lane + 1u < J ? L.sync[lane + 1u] : pos;
  // the first end-of-block code at or past the start (the chain's lanes are on the true
  // stream from there), if before the piece's end
  uint32_t hs = ZS_SEG_NONE, eend = 0, ecum = 0;
#pragma unroll
  for (uint32_t e = 0; e < ZS_SEG_NEOB; e++)
    if (e < neob && eob_sb[e] >= start && eob_sb[e] < hs) {
      hs = eob_sb[e];
      eend = eob_end[e];
      ecum = eob_cum[e];
    }
  if (hs == ZS_SEG_NONE && xeob_sb != ZS_SEG_NONE) {
    hs = xeob_sb;
    eend = xeob_end;
    ecum = xeob_cum;
  }
  const bool has_eob = chain && hs < nxs;
  const uint64_t eobm = __builtin_amdgcn_ballot_w64(has_eob);
  const uint32_t JE = eobm ? (uint32_t)__builtin_ctzll(eobm) : ZS_SEG_NONE;  // the lane ending the block
  const uint32_t jlast = eobm ? JE : J - 1u;
  uint32_t kind = eobm ? ZS_SG_K_BEND : ZS_SG_K_CONT;
  // a chain that reaches the input's end needs its end of block; a chain broken at J
  // continues from its last lane's stop (a true symbol start)
  if (!eobm && J == nl && !cont_ok) kind = ZS_SG_K_NONE;
  const bool mine = chain && lane <= jlast;
  bool bad = false;
  zs_seg_lane& P = recs[lane];
  P.act = 0;
  if (mine && kind != ZS_SG_K_NONE) {
    const uint32_t end = lane == JE ? eend : nxs;
    // the output count at the start: from the last own checkpoint at or before it
    uint32_t cp = q, cc = 0;
    for (uint32_t c = 0; c < (W / ZS_SEG_CKB); c++) {
      const uint32_t v = L.s.ock[lane][c], p = q + (v & 0xfffu);
      if (v != ZS_SEG_NONE && p <= start) {
        cp = p;
        cc = v >> 12;
      }
    }
    // ... and at the end: the end-of-block code's, the stop's, or from the last tail
    // checkpoint at or before the next lane's start (with the last symbol's length)
    uint32_t ce = cum, ll = last_len;
    if (lane == JE) {
      ce = ecum;
      ll = 0;
    }
    const bool redo_end = lane != JE && lane + 1u < J;
    uint32_t tp = qn, tc = 0;
    bool tfound = false;
    if (redo_end)
      for (uint32_t c = 0; c < (W / ZS_SEG_CKB); c++) {
        const uint32_t v = L.s.tck[lane][c], p = qn + (v & 0xfffu);
        if (v != ZS_SEG_NONE && p <= end) {
          tp = p;
          tc = v >> 12;
          tfound = true;
        }
      }
    bad |= redo_end && !tfound;
    // re-decode the stretches [cp, start) and (redo_end) [tp, end)
    for (uint32_t pass = 0; pass < 2; pass++) {
      if (pass == 1 && !redo_end) break;
      uint32_t p = pass ? tp : cp, c = pass ? tc : cc, lp = 0;
      const uint32_t to = pass ? end : start;
      zs_sg_seek(G, p);
      while (p < to) {
        const zs_sg_sym y = zs_sg_decode(G, lt, lmask, dt, dmask, emask);
        if (y.kind == ZS_SG_BAD) {
          p = p + 1u;
          zs_sg_seek(G, p);
          lp = 0;
          continue;
        }
        lp = y.kind == ZS_SG_EOB ? 0u : y.len;
        c += lp;
        p = zs_sg_bitpos(G);
      }
      bad |= p != to;
      if (pass) {
        ce = c;
        ll = lp;
      } else {
        cc = c;
      }
    }
    // the piece's own events, consecutive sub-chunks
    uint32_t k0 = 0, ne = 0;
    uint32_t eo[ZS_SEG_NEV];
#pragma unroll
    for (uint32_t e = 0; e < ZS_SEG_NEV; e++) {
      eo[e] = 0;
      if (e < nev && ev_sb[e] >= start && ev_sb[e] < end) {
        if (ne == 0) k0 = ev_k[e];
        bad |= ev_k[e] != k0 + ne;
#pragma unroll
        for (uint32_t g = 0; g < ZS_SEG_NEV; g++)
          if (g == ne) eo[g] = ev_c[e] - cc;
        ne++;
      }
    }
    bad |= nev > ZS_SEG_NEV;
    // an invalid code in the true stream
#pragma unroll
    for (uint32_t e = 0; e < ZS_SEG_NEOB; e++) bad |= e < nbad && bad_sb[e] >= start && bad_sb[e] < end;
    bad |= xbad < end;
    P.start = start;
    P.end = end;
    P.cnt = ce - cc;
    P.last_len = ll;
    // a split point strictly inside the piece, on the true stream (past its start)
    const bool cut = mid_sb != ZS_SEG_NONE && mid_sb > start && mid_sb < end && mid_cum > cc && mid_cum < ce;
    P.mb = cut ? mid_sb : ZS_SEG_NONE;
    P.mc = cut ? mid_cum - cc : 0u;
    P.mll = cut ? mid_ll : 0u;
    P.nev = ne;
    P.ev_k0 = k0;
#pragma unroll
    for (uint32_t e = 0; e < ZS_SEG_NEV; e++) P.ev_o[e] = eo[e];
    if (lane == jlast) L.send = end;
  } else {
    P.start = ZS_SEG_NONE;
  }
  bad_out = __syncthreads_or(bad);
  send = L.send;
#if ZS_SEG_EXP & 2
  if (lane == 0) L.dbg[1] = __builtin_readcyclecounter() - dbg_t1;
  __syncthreads();
#endif
  return kind;
}

template <bool D64, uint32_t W, bool ST>
__global__ __launch_bounds__(64) void zs_k_seg_walk(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint32_t* __restrict__ in_len,
                                                    const uint32_t* __restrict__ list, uint32_t n_list,
                                                    const uint32_t* __restrict__ big, uint32_t n_big, int wbits,
                                                    const uint64_t* __restrict__ found,
                                                    const uint32_t* __restrict__ spb, zs_seg_blk* __restrict__ blk,
                                                    zs_seg_lane* __restrict__ lanes, zcode* __restrict__ tcache,
                                                    zs_seg_ent* __restrict__ ents, zs_seg_mem* __restrict__ mem,
                                                    uint32_t* __restrict__ nspan, uint32_t* __restrict__ spans,
                                                    uint32_t sbits, int split) {
  __shared__ zs_sg_walk_lds<W> L;
  const uint32_t lane = threadIdx.x;
  // the entry: blocks [0, n_list): entry 0 of list member blockIdx.x; then
  // (ZS_SPLIT_MAX - 1) entries per big member
  uint32_t m, e, bi = ZS_SEG_NONE;
  if (blockIdx.x < n_list) {
    m = blockIdx.x;
    e = 0;
  } else {
    const uint32_t x = blockIdx.x - n_list;
    bi = x / (ZS_SPLIT_MAX - 1u);
    if (bi >= n_big) return;
    e = 1u + x % (ZS_SPLIT_MAX - 1u);
    m = big[bi];
  }
  zs_seg_ent& E = ents[(size_t)m * ZS_SPLIT_MAX + e];
  uint32_t start = 0;
  if (e) {
    const uint64_t f = found[(size_t)bi * ZS_SPLIT_MAX + e];
    if (f == ~0ull) return;  // (no candidate in this range: the entry record is never read)
    start = (uint32_t)f;
  }
  if (lane == 0) {
    E.start = start;
    E.first = ZS_SEG_NONE;
    E.end = 0;
    E.flags = 0;
  }
  // where the walk may stop: the later entries' starts (a big member's), found
  // in order of their ranges, so in order of position
  uint32_t later = ZS_SEG_NONE;  // this lane's: the start of entry `lane` if later than e
  if (bi != ZS_SEG_NONE && lane > e && lane < ZS_SPLIT_MAX) {
    const uint64_t f = found[(size_t)bi * ZS_SPLIT_MAX + lane];
    if (f != ~0ull) later = (uint32_t)f;
  }
  const uint32_t s = list[m];
  const uint32_t n = in_len[s];
  const uint32_t nbits = 8u * n;
  const uint8_t* src = in + in_off[s];
  const uint32_t sb0 = spb[m], cap = spb[m + 1] - sb0;
  zs_seg_mem& M = mem[m];
  zs_wave_reader R;
  R.n = n;
  R.sh = (uint32_t)((uintptr_t)src & 3u);
  R.w4 = reinterpret_cast<const uint32_t*>(src - R.sh);
  R.last = (R.sh + n - 1u) >> 2;
  R.inw = L.h.inw;
  zs_wr_stage(R, ((start >> 3) + R.sh) >> 2);
  zs_wr_seek(R, start >> 3);
  zs_wr_take(R, start & 7u);
  bool good = true;
  const int wrap = wbits < 0 ? 0 : (wbits >> 4) + 5;  // inflate.ts:152-160
  if (e == 0 && wrap) {  // plain zlib / gzip headers only (inflate.ts:377-580), as the lane path
    const uint32_t b0 = zs_wr_take(R, 8), b1 = zs_wr_take(R, 8);
    if ((wrap & 2) && b0 == 0x1f && b1 == 0x8b) {
      const uint32_t cm = zs_wr_take(R, 8), flg = zs_wr_take(R, 8);
      zs_wr_take(R, 32);
      zs_wr_take(R, 16);
      good = cm == 8 && flg == 0;
    } else if (wrap & 1) {
      good = !(((b0 << 8) | b1) % 31 || (b0 & 15) != 8 || (b0 >> 4) + 8 > 15 || (b1 & 0x20));
    } else {
      good = false;
    }
  }
  uint32_t hdr = (uint32_t)zs_wr_bitpos(R);
  uint32_t pe0 = e == 0 ? 0u : start;  // sub-chunk events before the first symbol go to it
  uint32_t prevb = ZS_SEG_NONE;       // the entry's last span
  uint32_t flags_e = 0;
  // bits per lane: seg_bits for the entry's first block, then from the size of the
  // block before (a zlib stream's blocks are alike): the block in one span of
  // about 60 lanes, S >= ZS_SEG_W (a lane's window ends before the next lane's start)
  uint32_t S = sbits;
#if ZS_SEG_EXP & 2
  unsigned long long wd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long wd_start = __builtin_readcyclecounter();
#endif
  while (good) {
    // ---- a block: its header (wave-uniform) and tables
    if (prevb != ZS_SEG_NONE || hdr != (uint32_t)zs_wr_bitpos(R)) {  // (a span has reused the staging LDS)
      zs_wr_stage(R, ((hdr >> 3) + R.sh) >> 2);
      zs_wr_seek(R, hdr >> 3);
      zs_wr_take(R, hdr & 7u);
    }
    uint32_t last = 0, lbits = 0, dbits = 0, dofs = 0, ntab = 0, slen = ZS_SEG_NONE;
#if ZS_SEG_EXP & 2
    const unsigned long long wd_h = __builtin_readcyclecounter();
#endif
    good = zs_sg_header(R, L.codes, L.h.lens, L.h.work, D64, last, lbits, dbits, dofs, ntab, slen);
#if ZS_SEG_EXP & 2
    wd[0] += __builtin_readcyclecounter() - wd_h;
    wd[3]++;
#endif
    const uint32_t sym0 = (uint32_t)zs_wr_bitpos(R);
    if (good && sym0 > nbits) good = false;
    if (good && slen != ZS_SEG_NONE && (uint64_t)sym0 + 8ull * slen > nbits) good = false;  // (the exact path reports it)
    if (!good) break;
    __syncthreads();
    uint32_t tab = ZS_SEG_NONE, cur = sym0;
    bool first = true;
    if (slen != ZS_SEG_NONE) {
      // ---- a stored block: one span of one piece (lane 0), the bytes at sym0 / 8
      uint32_t b = 0;
      if (lane == 0) b = atomicAdd(&M.nalloc, 1u);
      b = zs_u(__shfl(b, 0));
      if (b >= cap) {
        good = false;
        break;
      }
      b += sb0;
      cur = sym0 + 8u * slen;
      zs_seg_lane& P = lanes[(size_t)b * ZS_SEG_LANES + lane];
      P.act = 0;
      P.start = lane == 0 ? sym0 : ZS_SEG_NONE;
      if (lane == 0) {
        spans[atomicAdd(nspan, 1u)] = b;
        P.end = cur;
        P.cnt = slen;
        P.last_len = 0;
        P.nev = 0;  // (crossings inside it: the plan replays the COPY state, zs_sg_calls::stored)
        P.ev_k0 = 0;
        zs_seg_blk& Bk = blk[b];
        Bk.m = m;
        Bk.e = e;
        Bk.hdr = hdr;
        Bk.sym0 = sym0;
        Bk.end = cur;
        Bk.lbits = Bk.dbits = Bk.dofs = 0;
        Bk.tab = ZS_SEG_NONE;
        Bk.pad[0] = 0;
        Bk.nl = 1;
        Bk.S = 0;
        Bk.next = ZS_SEG_NONE;
        Bk.flags = ZS_SEG_B_OK | ZS_SEG_B_FIRST | ZS_SEG_B_EOB | ZS_SEG_B_STORED | (last ? ZS_SEG_B_FINAL : 0u);
        if (prevb == ZS_SEG_NONE) E.first = b;
        else blk[prevb].next = b;
      }
      prevb = b;
      pe0 = cur;
    }
    while (slen == ZS_SEG_NONE) {  // (a coded block's spans; left by break)
      // ---- a span
      // (split mode: two slots, the second for the pieces' second halves, which the plan writes)
      const uint32_t nsl = split ? 2u : 1u;
      uint32_t b = 0;
      if (lane == 0) b = atomicAdd(&M.nalloc, nsl);
      b = zs_u(__shfl(b, 0));
      if (b + nsl > cap) {
        good = false;
        break;
      }
      b += sb0;
      if (lane == 0) {  // (the decode's work list)
        const uint32_t at = atomicAdd(nspan, nsl);
        spans[at] = b;
        if (split) spans[at + 1u] = b + 1u;
      }
      if (split) {
        zs_seg_lane& P2 = lanes[(size_t)(b + 1u) * ZS_SEG_LANES + lane];
        P2.act = 0;
        P2.start = ZS_SEG_NONE;
      }
      if (first) {
        tab = b;
        for (uint32_t i = lane; i < ntab; i += 64) tcache[(size_t)b * ZS_SEG_TAB + i] = L.codes[i];
      }
      if (cur >= nbits) {
        good = false;
        break;
      }
      const uint32_t nl = max(1u, min(ZS_SEG_LANES, (nbits - cur + S - 1u) / S));
      uint32_t send = 0;
      bool sbad = false;
      const uint32_t k = zs_sg_span<D64, W, ST>(L, src, n, cur, pe0, nl, S, lbits, dbits, dofs,
                                         lanes + (size_t)b * ZS_SEG_LANES, send, sbad, split != 0);
#if ZS_SEG_EXP & 2
      wd[1] += L.dbg[0];
      wd[2] += L.dbg[1];
      wd[4]++;
      wd[5] += L.dbg[2];
      wd[7] += L.dbg[3];
#endif
      if (lane == 0) {
        zs_seg_blk& Bk = blk[b];
        Bk.m = m;
        Bk.e = e;
        Bk.hdr = first ? hdr : cur;
        Bk.sym0 = cur;
        Bk.end = send;
        Bk.lbits = lbits;
        Bk.dbits = dbits;
        Bk.dofs = dofs;
        Bk.tab = tab;
        Bk.pad[0] = ntab;  // (the decode's table size)
        Bk.nl = nl;
        Bk.S = S;
        Bk.next = ZS_SEG_NONE;
        Bk.flags = (k && !sbad ? ZS_SEG_B_OK : 0u) | (first ? ZS_SEG_B_FIRST : 0u) |
                   (k == ZS_SG_K_BEND ? ZS_SEG_B_EOB : 0u) | (k == ZS_SG_K_BEND && last ? ZS_SEG_B_FINAL : 0u) |
                   (split ? ZS_SEG_B_SPLIT : 0u);
        if (prevb == ZS_SEG_NONE) E.first = b;
        else blk[prevb].next = b;
        if (split) {  // the second halves' slot: the same block and tables, off the entry's chain
          zs_seg_blk& B2 = blk[b + 1u];
          B2 = Bk;
          B2.next = ZS_SEG_NONE;
          B2.flags = Bk.flags & ZS_SEG_B_OK;
        }
      }
      prevb = b;
      if (!k || sbad) {
        good = false;
        break;
      }
      first = false;
      pe0 = send;
      cur = send;
      if (k == ZS_SG_K_BEND) break;
    }
    if (!good) break;
    // ---- the block ended at cur: the final one, or at a later entry's start
    if (slen == ZS_SEG_NONE) S = min(ZS_SEG_SMAX, max(W, (cur - hdr) / 60u));
    hdr = cur;
    if (last) {
      flags_e = 3u;
      break;
    }
    if (__builtin_amdgcn_ballot_w64(later == cur)) {
      flags_e = 1u;
      break;
    }
    if (cur >= nbits) {
      good = false;
      break;
    }
  }
  if (lane == 0) {
    E.end = hdr;
    E.flags = good ? flags_e : 0u;
  }
#if ZS_SEG_EXP & 2
  wd[6] = __builtin_readcyclecounter() - wd_start;
  if (lane == 0 && blockIdx.x < ZS_SEG_WDBG_N)
    for (int i = 0; i < 8; i++) zs_seg_wdbg[blockIdx.x][i] = wd[i];
#endif
}

// ------------------------------------------------------------------- plan
// One wave per member: its entries chained from entry 0 (each walk ended where
// the next one starts), their spans in order, the pieces placed, the trailer
// and the capacity checked, and (REFW) the reference's call state at each piece
// start -- tools/emu/emu_seg.py models exactly this walk.
struct zs_sg_calls {
  uint32_t B, wn, wh, cend;
  __device__ void end_call(uint32_t at) {  // zs_refcalls_t::end_call
    const uint32_t produced = at - B;
    if (produced >= 32768u) {
      wn = 0;
      wh = 32768u;
    } else if (produced) {
      const uint32_t d = min(32768u - wn, produced), rest = produced - d;
      if (rest) {
        wn = rest;
        wh = 32768u;
      } else {
        wn += d;
        if (wn == 32768u) wn = 0;
        wh = min(wh + d, 32768u);
      }
    }
    B = at;
  }
  __device__ void fills(uint32_t o) {  // the buffer fills a symbol at output position o has triggered
    while (o >= B + 65536u) end_call(B + 65536u);
  }
  // zs_refcalls_t::stored (the COPY state); the calls ending before its end -- sub-chunk ends below in + len,
  // the header's ones too: no piece has them as events (the next piece's start at in + len)
  __device__ void stored(uint32_t in, uint32_t o, uint32_t len) {
    if (o > B + 65536u) end_call(B + 65536u);
    while (len == 0 && cend < in) {  // (an empty block: the sub-chunks its header read past)
      end_call(o);
      cend += 32768u;
    }
    while (len) {
      while (in >= cend) {
        end_call(o);
        cend += 32768u;
      }
      if (o >= B + 65536u) end_call(B + 65536u);
      const uint32_t take = min(len, min(cend - in, B + 65536u - o));
      in += take;
      o += take;
      len -= take;
    }
  }
};

__global__ __launch_bounds__(64) void zs_k_seg_plan(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint32_t* __restrict__ in_len,
                                                    const uint32_t* __restrict__ out_cap,
                                                    const uint32_t* __restrict__ list, uint32_t n_list, int wbits,
                                                    int refw, const zs_seg_blk* __restrict__ blk,
                                                    zs_seg_lane* __restrict__ lanes, const zs_seg_ent* __restrict__ ents,
                                                    zs_seg_mem* __restrict__ mem, const uint32_t* __restrict__ pbase,
                                                    uint4* __restrict__ ptab) {
  __shared__ zs_seg_lane P[ZS_SEG_LANES];
  __shared__ zs_seg_lane Q[ZS_SEG_LANES];  // (split mode) the second halves, for the span's next slot
  __shared__ uint32_t s_bad, s_O, s_k, s_plen, s_first, s_prevg;
  __shared__ zs_sg_calls s_C;
  const uint32_t m = blockIdx.x, lane = threadIdx.x;
  if (m >= n_list) return;
  zs_seg_mem& M = mem[m];
  const uint32_t s = list[m];
  const zs_seg_ent* E = ents + (size_t)m * ZS_SPLIT_MAX;
  const uint32_t e_start = E[lane].start;  // (lane < ZS_SPLIT_MAX = 64)
  if (lane == 0) {
    s_bad = 0;
    s_O = 0;
    s_k = 0;
    s_prevg = ZS_SEG_NONE;
    s_plen = 0;
    s_first = 1;
    s_C.B = 0;
    s_C.wn = 0;
    s_C.wh = 0;
    s_C.cend = 32768u;
  }
  __syncthreads();
  const uint32_t pb = pbase[m], pmax = pbase[m + 1] - pb;
  uint32_t e = 0, guard = 0, fin_end = 0;
  bool fin = false;
  while (!s_bad) {
    const zs_seg_ent En = E[e];
    if (!(En.flags & 1u) || guard++ > ZS_SPLIT_MAX) {
      s_bad = 1;
      break;
    }
    for (uint32_t b = En.first; b != ZS_SEG_NONE && !s_bad;) {
      const zs_seg_blk Bk = blk[b];
      if (!(Bk.flags & ZS_SEG_B_OK)) {
        s_bad = 1;
        break;
      }
      P[lane] = lanes[(size_t)b * ZS_SEG_LANES + lane];
      const bool split = (Bk.flags & ZS_SEG_B_SPLIT) != 0;
      if (split) {
        Q[lane].start = ZS_SEG_NONE;
        Q[lane].act = 0;
      }
      __syncthreads();
      if (lane == 0) {
        zs_sg_calls C = s_C;
        uint32_t O = s_O, k = s_k, prevg = s_prevg, plen = s_plen;
        bool first = s_first != 0, bad = false;
        const bool newblk = (Bk.flags & ZS_SEG_B_FIRST) != 0;
        if (Bk.flags & ZS_SEG_B_STORED) {  // one piece; the reference's COPY state ends calls inside it
          zs_seg_lane& p = P[0];
          if (refw) C.stored(p.start >> 3, O, p.cnt);
          p.O = O;
          p.off = ((O + 7u) & ~7u) + ZS_SEG_PAD * k;
          p.dend = p.end;
          p.dcnt = p.cnt;
          p.B = C.B;
          p.wn = C.wn;
          p.wh = C.wh;
          p.cend = C.cend;
          p.act = 1u;
          if (k >= pmax) bad = true;
          else ptab[pb + k] = make_uint4(O, p.cnt, p.off, 0u);
          k++;
          prevg = b * ZS_SEG_LANES;
          O += p.cnt;
          plen = 0;
          first = false;
        }
        // one piece (g: its record's global index; l0new: the first of a block)
        auto piece = [&](zs_seg_lane& p, uint32_t g, bool l0new) {
          bool merge = false;
          if (!first && refw) {
            if (l0new) {
              C.fills(O);  // the end-of-block code before it, at output O
            } else {
              C.fills(O - plen);  // the last symbol of the piece before
              // a start within 144 bits before a sub-chunk end: the piece before decodes this one too
              merge = p.start + 144u > 8u * C.cend;
            }
          }
          if (merge) {
            // the piece before is in this block: in this span (or its second halves), or the entry's span before
            const uint32_t ps = prevg / ZS_SEG_LANES;
            zs_seg_lane& q = ps == b ? P[prevg % ZS_SEG_LANES]
                             : (split && ps == b + 1u) ? Q[prevg % ZS_SEG_LANES] : lanes[prevg];
            q.dend = p.end;
            q.dcnt += p.cnt;
            p.act = 0;
            if (k - 1 < pmax) ptab[pb + k - 1].y = q.dcnt;
          } else {
            p.O = O;
            p.off = ((O + 7u) & ~7u) + ZS_SEG_PAD * k;
            p.dend = p.end;
            p.dcnt = p.cnt;
            p.B = C.B;
            p.wn = C.wn;
            p.wh = C.wh;
            p.cend = C.cend;
            p.act = 1u | (l0new ? 0u : 2u);
            if (k >= pmax) bad = true;
            else ptab[pb + k] = make_uint4(O, p.cnt, p.off, 0u);
            k++;
            prevg = g;
          }
          if (refw) {
            for (uint32_t x = 0; x < p.nev; x++) {
              bad |= 32768u * (p.ev_k0 + x) != C.cend;  // events come one sub-chunk at a time (boundary k: cend = 32768 k)
              const uint32_t o = O + p.ev_o[x];
              C.fills(o);
              C.end_call(o);
              C.cend += 32768u;
            }
          }
          O += p.cnt;
          plen = p.last_len;
          first = false;
        };
        for (uint32_t l = 0; l < ZS_SEG_LANES && !bad && !(Bk.flags & ZS_SEG_B_STORED); l++) {
          zs_seg_lane& p = P[l];
          if (p.start == ZS_SEG_NONE) continue;
          if (split && p.mb != ZS_SEG_NONE) {
            // split mode: the piece as two, cut at its split point (the walk's first symbol start past the
            // lane's middle): the second half into the next slot, with the events after the cut
            zs_seg_lane& h = Q[l];
            h = p;
            h.start = p.mb;
            h.cnt = p.cnt - p.mc;
            uint32_t na = 0;
            for (uint32_t x = 0; x < p.nev; x++) na += p.ev_o[x] < p.mc ? 1u : 0u;
            h.nev = p.nev - na;
            h.ev_k0 = p.ev_k0 + na;
            for (uint32_t x = 0; x < h.nev; x++) h.ev_o[x] = p.ev_o[x + na] - p.mc;
            p.end = p.mb;
            p.cnt = p.mc;
            p.last_len = p.mll;
            p.nev = na;
            piece(p, b * ZS_SEG_LANES + l, l == 0 && newblk);
            if (!bad) piece(h, (b + 1u) * ZS_SEG_LANES + l, false);
          } else {
            piece(p, b * ZS_SEG_LANES + l, l == 0 && newblk);
          }
        }
        s_C = C;
        s_O = O;
        s_k = k;
        s_prevg = prevg;
        s_plen = plen;
        s_first = first ? 1u : 0u;
        if (bad) s_bad = 1;
      }
      __syncthreads();
      // the pieces' plan back to HBM
      if (P[lane].start != ZS_SEG_NONE) lanes[(size_t)b * ZS_SEG_LANES + lane] = P[lane];
      if (split) lanes[(size_t)(b + 1u) * ZS_SEG_LANES + lane] = Q[lane];
      __threadfence_block();
      __syncthreads();
      b = Bk.next;
    }
    __syncthreads();
    if (s_bad) break;
    if (En.flags & 2u) {
      fin = true;
      fin_end = En.end;
      break;
    }
    // the entry whose start is where this walk stopped
    const uint64_t nx = __builtin_amdgcn_ballot_w64(lane > e && e_start == En.end);
    if (!nx) {
      s_bad = 1;
      break;
    }
    e = (uint32_t)__builtin_ctzll(nx);
  }
  __syncthreads();
  if (lane == 0) {
    bool bad = s_bad != 0 || !fin;
    const uint32_t total = s_O;
    const uint32_t n = in_len[s];
    uint32_t consumed = (fin_end + 7u) >> 3, want = 0;
    const int wrap = wbits < 0 ? 0 : (wbits >> 4) + 5;
    if (!bad && wrap) {  // the trailer (inflate.ts:1006-1036); the check value is verified after the checksum pass
      const uint8_t* t = in + in_off[s] + consumed;
      if (wrap & 2 && !(wrap & 1)) {
        if (consumed + 8u > n) bad = true;
        else {
          want = (uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
          const uint32_t isize = (uint32_t)t[4] | (uint32_t)t[5] << 8 | (uint32_t)t[6] << 16 | (uint32_t)t[7] << 24;
          bad |= isize != total;
          consumed += 8u;
        }
      } else {
        if (consumed + 4u > n) bad = true;
        else {
          want = (uint32_t)t[0] << 24 | (uint32_t)t[1] << 16 | (uint32_t)t[2] << 8 | (uint32_t)t[3];
          consumed += 4u;
        }
      }
    }
    if (!bad && consumed > n) bad = true;
    if (total > out_cap[s]) bad = true;  // the exact path reports the capacity
    M.bad = bad ? 1u : 0u;
    M.total = total;
    M.consumed = consumed;
    M.want = want;
    M.npieces = s_k;
  }
}

// ----------------------------------------------------------------- decode
// The decode's LDS table: the first ZS_SEG_TAB_DEC entries of a block's tables (inflate_table's
// sizes; text blocks use 600-900), not the ENOUGH bound (1,444): 4 instead of 5.8 KB of LDS per wave,
// 20 waves per CU instead of 16.  The literal/length table always fits (<= 852 entries); distance
// entries past the bound are read from the walk's copy in HBM (zs_sg_dtab)
#ifndef ZS_SEG_TAB_DEC
#define ZS_SEG_TAB_DEC 1024u
#endif
static_assert(ZS_SEG_TAB_DEC > ENOUGH_LENS, "the literal/length table must fit the decode's LDS table");
typedef const __attribute__((address_space(3))) zcode zs_l_zc;
typedef const __attribute__((address_space(1))) zcode zs_g_zc;
struct zs_sg_dtab {  // a distance table: entries below lim in LDS, the rest in HBM
  zs_l_zc* l;
  zs_g_zc* g;
  uint32_t lim;
  __device__ __forceinline__ zcode operator[](uint32_t i) const { return i < lim ? l[i] : g[i]; }
};
#ifndef ZS_SG_RING
#define ZS_SG_RING 32u  // u16 values of a lane's LDS output ring (a power of two; 32 vs 64: 10 instead of 14 KB of
                        // LDS per wave, C5-i 11.0 -> 10.2 ms)
#endif
// room(k) flushes whole 8-value units: up to 7 values stay, so k + 7 must fit (the largest k is 16)
static_assert(ZS_SG_RING >= 16u + 7u && (ZS_SG_RING & (ZS_SG_RING - 1u)) == 0, "decode ring too small");
static_assert(ZS_SG_RING > 28u, "a short-period copy reads up to 2 x 14 values back from the ring (near)");
// One lane's u16 output (bytes, or markers 255 + k: the value k positions
// before the piece): a ZS_SG_RING-value LDS ring, whole 16-byte units to HBM (the
// piece's scratch is 16-byte aligned and padded, so no unit is shared).
// (dst and ring typed by address space: with generic pointers the compiler folds get()'s two
// loads into one flat load of a selected pointer, waited for on both counters)
typedef __attribute__((address_space(1))) uint16_t zs_g_u16;
typedef __attribute__((address_space(3))) uint16_t zs_l_u16;
typedef uint32_t zs_v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) zs_v4u zs_g_u4;
typedef __attribute__((address_space(3))) zs_v4u zs_l_u4;
static __device__ __forceinline__ zs_v4u zs_v4(uint4 a) { return zs_v4u{a.x, a.y, a.z, a.w}; }
struct zs_sg_out {
  zs_g_u16* dst;
  zs_l_u16* ring;
  uint32_t P, F;
  bool ovf;  // a reservation the ring could not hold (guarded statically; a run that sees it bails the member)
  __device__ __forceinline__ void put(uint32_t v) {
    ring[P & (ZS_SG_RING - 1u)] = (uint16_t)v;
    P++;
  }
  __device__ __forceinline__ void flush() {
    while (F + 8u <= P) {
      *reinterpret_cast<zs_g_u4*>(dst + F) = *reinterpret_cast<const zs_l_u4*>(ring + (F & (ZS_SG_RING - 1u)));
      F += 8u;
    }
  }
  __device__ __forceinline__ void room(uint32_t k) {  // room for k more values
    if (P + k - F > ZS_SG_RING) {
      flush();
      ovf |= P + k - F > ZS_SG_RING;
    }
  }
  // the value at piece position x < P: the ring holds the last 64, older ones are stored
#if ZS_SEG_EXP & 1
  uint32_t far = 0;
  __device__ __forceinline__ uint32_t get(uint32_t x) {
    far += x + ZS_SG_RING < P;
    return x + ZS_SG_RING >= P ? ring[x & (ZS_SG_RING - 1u)] : dst[x];
  }
#else
  __device__ __forceinline__ uint32_t get(uint32_t x) const {
    return x + ZS_SG_RING >= P ? ring[x & (ZS_SG_RING - 1u)] : dst[x];
  }
#endif
  // a value of the last ZS_SG_RING (x + ZS_SG_RING >= P), from the ring
  __device__ __forceinline__ uint32_t near(uint32_t x) const { return ring[x & (ZS_SG_RING - 1u)]; }
  // the eight values at x .. x + 7 (< P): all stored, all in the ring, or across the two.  (Element
  // by element, each value's ring-or-HBM branch made the compiler wait for every load on its own: eight
  // round trips to HBM for a far copy's round instead of one.)
  __device__ __forceinline__ void get8(uint32_t x, uint32_t (&v)[8]) {
#if !(ZS_SEG_EXP & 1)
    if (x + 7u + ZS_SG_RING < P) {
      const zs_g_u16* const d = dst + x;  // (one address, immediate offsets)
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) v[j] = d[j];
      return;
    }
    if (x + ZS_SG_RING >= P) {
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) v[j] = ring[(x + j) & (ZS_SG_RING - 1u)];
      return;
    }
#endif
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) v[j] = get(x + j);
  }
  __device__ __forceinline__ void finish() {
    flush();
    if (F < P) *reinterpret_cast<zs_g_u4*>(dst + F) = *reinterpret_cast<const zs_l_u4*>(ring + (F & (ZS_SG_RING - 1u)));
  }
  // A long run of n >= ZS_SG_BULK values given by their 8-value units: one by one up to an
  // 8-aligned position, then whole 16-byte units straight to HBM from registers (no LDS
  // round trip per value: a lane's 44,000-value run of distance-1 copies took 4.4 ms through
  // the ring), the ring refilled with the last ZS_SG_RING values, the rest one by one.
  // unit(x): the packed values of positions x .. x + 7; one(x): the value at x.
  template <typename U, typename O>
  __device__ __forceinline__ void run(uint32_t n, U unit, O one) {
    const uint32_t end = P + n;
    while (P & 7u) {
      room(1);
      put(one(P));
    }
    flush();  // F = P
    const uint32_t e8 = end & ~7u;
    for (; P < e8; P += 8u) *reinterpret_cast<zs_g_u4*>(dst + P) = zs_v4(unit(P));
    F = P;
#pragma unroll
    for (uint32_t k = 0; k < ZS_SG_RING; k += 8u)
      *reinterpret_cast<zs_l_u4*>(ring + ((P - ZS_SG_RING + k) & (ZS_SG_RING - 1u))) = zs_v4(unit(P - ZS_SG_RING + k));
    while (P < end) {
      room(1);
      put(one(P));
    }
  }
};
#ifndef ZS_SG_BULK
#define ZS_SG_BULK 64u  // (>= ZS_SG_RING + 15: the ring's values after the aligned units all belong to the run)
#endif
static_assert(ZS_SG_BULK >= ZS_SG_RING + 15u, "bulk runs too short for the ring refill");
// value i (runtime, < 8) of eight u16 values packed two per word: bit selects, not an
// indexed array (a select chain on i the compiler turns into a scratch-memory table)
static __device__ __forceinline__ uint32_t zs_sg_pick8(const uint32_t (&w)[4], uint32_t i) {
  const uint32_t a = (i & 2u) ? w[1] : w[0], b = (i & 2u) ? w[3] : w[2];
  const uint32_t c = (i & 4u) ? b : a;
  return (i & 1u) ? c >> 16 : c & 0xffffu;
}

// n values from piece position x0 (negative: markers for the history before
// the piece); false: a marker further back than a u16 says
static __device__ __forceinline__ bool zs_sg_copy(zs_sg_out& W, int32_t x0, uint32_t n) {
  if (x0 < 0) {
    // the part before the piece: markers 255 + k, k falling by one per value (the
    // first, the furthest back, must fit a u16), eight per round
    const uint32_t back = (uint32_t)(-x0);
    if (back > ZS_SPLIT_MARK_MAX) return false;
    const uint32_t m = min(n, back);
    if (m >= ZS_SG_BULK) {  // the marker at position x: a0 - x
      const uint32_t a0 = 255u + back + W.P;
      W.run(
          m,
          [a0](uint32_t x) {
            const uint32_t a = a0 - x;
            return make_uint4(a | (a - 1u) << 16, (a - 2u) | (a - 3u) << 16, (a - 4u) | (a - 5u) << 16,
                              (a - 6u) | (a - 7u) << 16);
          },
          [a0](uint32_t x) { return a0 - x; });
    } else
    for (uint32_t i = 0; i < m; i += 8) {
      W.room(8);
#pragma unroll
      for (uint32_t j = 0; j < 8; j++)
        if (i + j < m) W.put(255u + back - (i + j));
    }
    if (m == n) return true;
    n -= m;
    x0 = 0;
  }
  const int32_t d = (int32_t)W.P - x0;
  if (x0 >= 0 && d >= 8) {
    for (uint32_t i = 0; i < n; i += 8) {
      W.room(8);
      uint32_t v[8];
      W.get8((uint32_t)x0 + i, v);
      const uint32_t k = min(8u, n - i);
#pragma unroll
      for (uint32_t j = 0; j < 8; j++)
        if (j < k) W.put(v[j]);
    }
    return true;
  }
  if (x0 >= 0) {  // period d < 8: the first dd = d * ceil(8 / d) values one by one, then a
                  // copy from dd back (the pattern repeats at dd >= 8 too), eight per round
    const uint32_t dd = (uint32_t)d * ((8u + (uint32_t)d - 1u) / (uint32_t)d);
    const uint32_t first = min(n, dd);
    uint32_t v[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) v[j] = (int32_t)j < d ? W.near((uint32_t)x0 + j) : 0u;  // (d < 8 back)
    if ((d & (d - 1)) == 0 && n >= ZS_SG_BULK) {
      // d = 1, 2, 4: every 8-aligned unit holds the same values (runs: the deflate64 fixtures'
      // 257-byte distance-1 copies)
      const uint32_t P0 = W.P, dm = (uint32_t)d - 1u, rb = (0u - P0) & dm;
      const uint32_t pv[4] = {v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16};
      uint32_t u[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) u[k] = zs_sg_pick8(pv, (rb + k) & dm);
      const uint4 w = make_uint4(u[0] | u[1] << 16, u[2] | u[3] << 16, u[4] | u[5] << 16, u[6] | u[7] << 16);
      W.run(
          n, [w](uint32_t) { return w; },
          [v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3], P0, dm](uint32_t x) {  // (by value: v stays in registers)
            const uint32_t i = (x - P0) & dm;  // d = 1, 2, 4: i < 4
            return i == 0 ? v0 : i == 1 ? v1 : i == 2 ? v2 : v3;
          });
      return true;
    }
    uint32_t j = 0;
    W.room(16);
    const uint32_t pv[4] = {v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16};
    for (uint32_t i = 0; i < first; i++) {
      W.put(zs_sg_pick8(pv, j));
      j = j + 1 == (uint32_t)d ? 0u : j + 1;
    }
    const uint32_t rest = n - first;
    const uint32_t xs = W.P - dd;
    for (uint32_t i = 0; i < rest; i += 8) {
      W.room(8);
      uint32_t u[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) u[k] = W.near(xs + i + k);  // (at most 2 dd <= 28 back)
      const uint32_t k8 = min(8u, rest - i);
#pragma unroll
      for (uint32_t k = 0; k < 8; k++)
        if (k < k8) W.put(u[k]);
    }
    return true;
  }
  return true;  // (x0 >= 0 here: one of the two paths above)
}

#if ZS_SEG_EXP & 1
#define ZS_SEG_DBG_N 65536u
__device__ unsigned long long zs_seg_dbg[ZS_SEG_DBG_N][4];  // per span slot: start, end (max), symbols (max lane), far reads (max lane)
extern "C" int zs_seg_dbg_fetch(void* out, unsigned long long bytes) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_seg_dbg), bytes < sizeof(zs_seg_dbg) ? bytes : sizeof(zs_seg_dbg));
}
#endif
template <bool D64, bool REFW>
__global__ __launch_bounds__(64) void zs_k_seg_decode(const uint8_t* __restrict__ in,
                                                      const uint64_t* __restrict__ in_off,
                                                      const uint32_t* __restrict__ in_len,
                                                      const uint32_t* __restrict__ list,
                                                      const uint32_t* __restrict__ nspan,
                                                      const uint32_t* __restrict__ spans,
                                                      const zs_seg_blk* __restrict__ blk,
                                                      const zs_seg_lane* __restrict__ lanes,
                                                      const zcode* __restrict__ tcache, zs_seg_mem* __restrict__ mem,
                                                      const uint64_t* __restrict__ sbase,
                                                      uint16_t* __restrict__ scratch) {
  __shared__ zcode codes[ZS_SEG_TAB_DEC];
  __shared__ __attribute__((aligned(16))) uint16_t ring[ZS_SEG_LANES][ZS_SG_RING];
  const uint32_t lane = threadIdx.x;
  const uint32_t ns = *nspan;
  for (uint32_t k = blockIdx.x; k < ns; k += gridDim.x) {
  const uint32_t b = zs_u(spans[k]);
  const zs_seg_blk& Bk = blk[b];
  const uint32_t m = zs_u(Bk.m);
  if (m == ZS_SEG_NONE || !(Bk.flags & ZS_SEG_B_OK) || mem[m].bad) continue;
  if (Bk.flags & ZS_SEG_B_STORED) {  // the input's bytes as values, 8 per lane and round
    const zs_seg_lane& p = lanes[(size_t)b * ZS_SEG_LANES];
    const uint8_t* sp = in + in_off[list[m]] + (p.start >> 3);
    uint4* dst = reinterpret_cast<uint4*>(scratch + sbase[m] + p.off);  // (16-byte aligned, padded)
    for (uint32_t i = 8u * lane; i < p.cnt; i += 8u * ZS_SEG_LANES) {
      uint32_t v[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) v[j] = i + j < p.cnt ? sp[i + j] : 0u;
      dst[i >> 3] = make_uint4(v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16);
    }
    continue;
  }
  const uint32_t ntab = zs_u(Bk.pad[0]), tab = zs_u(Bk.tab);
  __syncthreads();  // (the previous span's tables are no longer read)
  for (uint32_t i = lane; i < min(ntab, ZS_SEG_TAB_DEC); i += 64) codes[i] = tcache[(size_t)tab * ZS_SEG_TAB + i];
  __syncthreads();
  const zs_seg_lane& p = lanes[(size_t)b * ZS_SEG_LANES + lane];
#if ZS_SEG_EXP & 1
  const unsigned long long dbg_t0 = wall_clock64();
  if (lane == 0 && b < ZS_SEG_DBG_N) {
    zs_seg_dbg[b][0] = dbg_t0;
    zs_seg_dbg[b][1] = 0;
    zs_seg_dbg[b][2] = 0;
    zs_seg_dbg[b][3] = 0;
  }
  __syncthreads();
  uint32_t dbg_sym = 0;
#endif
  if (lane >= zs_u(Bk.nl) || p.start == ZS_SEG_NONE || !(p.act & 1u)) continue;
  const uint32_t s = list[m];
  const uint32_t lmask = (1u << Bk.lbits) - 1u, dmask = (1u << Bk.dbits) - 1u, emask = D64 ? 31u : 15u;
  const zcode* lt = codes;
  const uint32_t dofs = zs_u(Bk.dofs);
  const zs_sg_dtab dt = {(const zs_l_zc*)(codes + dofs), (const zs_g_zc*)(tcache + (size_t)tab * ZS_SEG_TAB + dofs),
                         ZS_SEG_TAB_DEC - dofs};
  zs_sg_reader G;
  zs_sg_init(G, in + in_off[s], in_len[s]);
  zs_sg_seek(G, p.start);
  zs_sg_out W;
  W.dst = (zs_g_u16*)(scratch + sbase[m] + p.off);
  W.ring = (zs_l_u16*)ring[lane];
  W.P = 0;
  W.F = 0;
  W.ovf = false;
  const uint32_t O = p.O, dend = p.dend;
  zs_refcalls_t<uint32_t> C;
  C.B = p.B;
  C.wn = p.wn;
  C.wh = p.wh;
  C.cend = p.cend;
  C.fast = (p.act >> 1) & 1u;
  C.sfar = 8u * C.cend - 96u;
  C.ofar = C.B + 65536u - 516u;
  bool bad = false;
  uint32_t sb = p.start;
  while (sb < dend) {
    if (W.P - W.F >= ZS_SG_RING / 2u) W.flush();
    const zs_sg_sym y = zs_sg_decode(G, lt, lmask, dt, dmask, emask);
    const uint32_t o = O + W.P;
#if ZS_SEG_EXP & 1
    dbg_sym++;
#endif
    if (y.kind == ZS_SG_LIT) {
      if (REFW) C.symbol(sb, o, 1u, y.l1, 0u, 0u, 0u, false);
      W.room(1);
      W.put(y.val);
    } else if (y.kind == ZS_SG_COPY) {
      if (y.val > o) {  // "invalid distance too far back": the exact path reports it
        bad = true;
        break;
      }
      uint32_t tail = 0;
      if (REFW && C.symbol(sb, o, y.len, y.l1, y.e1, y.l2, y.e2, false)) tail = C.wrap(o, y.len, y.val);
      if (!zs_sg_copy(W, (int32_t)W.P - (int32_t)y.val, y.len - tail)) {
        bad = true;
        break;
      }
      // the window-wrap copy: the call's first output bytes (from C.B on)
      if (tail && !zs_sg_copy(W, (int32_t)C.B - (int32_t)O, tail)) {
        bad = true;
        break;
      }
    } else if (y.kind == ZS_SG_EOB) {
      if (REFW) C.symbol(sb, o, 0u, y.l1, 0u, 0u, 0u, true);
      bad = zs_sg_bitpos(G) != dend;  // only the block's last piece ends with its end of block
      break;
    } else {
      bad = true;
      break;
    }
    sb = zs_sg_bitpos(G);
  }
  bad |= sb > dend || W.P != p.dcnt || W.ovf;
  if (!bad) W.finish();
  if (bad) atomicOr(&mem[m].bad, 1u);
#if ZS_SEG_EXP & 1
  if (b < ZS_SEG_DBG_N) {
    atomicMax(&zs_seg_dbg[b][1], wall_clock64());
    atomicMax(&zs_seg_dbg[b][2], (unsigned long long)dbg_sym);
    atomicMax(&zs_seg_dbg[b][3], (unsigned long long)W.far);
  }
#endif
  }
}

// ---------------------------------------------------------------- resolve
// One workgroup per member: the pieces in order (the plan's table: output
// position, values, scratch offset); a piece's markers name bytes before its
// start, all final by then -- in the LDS ring of the last 64 KiB, or (rarely: a
// marker carried far into a long piece) in the output already stored.  A round
// covers up to 4,096 values of one piece; the next round's values are loaded
// before this one's markers are looked up.  Bytes leave as whole words, 16 KiB
// at a time.
// T threads per member, an LDS ring of the last RING final bytes (a marker
// further back reads the output already stored): <256, 32 KiB> -- four members per
// CU -- for batches that fill the chip (4,096 x 256 KiB: resolve 2.27 -> ~1.8 ms),
// <512, 64 KiB> for a few members (the 512-member shard: 0.50 vs 0.59 ms)
#define ZS_SG_RES_T T
#define ZS_SG_RES_RING RING
#define ZS_SG_RES_E 8u                                  // values per thread per round
#define ZS_SG_RES_R (ZS_SG_RES_T * ZS_SG_RES_E)        // values per round
#define ZS_SG_RES_PT 256u                               // piece-table entries staged in LDS
template <uint32_t T, uint32_t RING>
__global__ __launch_bounds__(T) void zs_k_seg_resolve(const uint32_t* __restrict__ list,
                                                        const zs_seg_mem* __restrict__ mem,
                                                        const uint32_t* __restrict__ pbase,
                                                        const uint4* __restrict__ ptab,
                                                        const uint64_t* __restrict__ sbase,
                                                        const uint16_t* __restrict__ scratch, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        zs_lane_res* __restrict__ res, uint32_t* __restrict__ lens_out,
                                                        uint32_t* __restrict__ n_ok, uint32_t* __restrict__ n_left,
                                                        uint32_t* __restrict__ left) {
  extern __shared__ __attribute__((aligned(16))) uint32_t zs_rring[];  // ZS_SG_RES_RING bytes
  __shared__ uint4 tab[ZS_SG_RES_PT];
  uint8_t* ring = reinterpret_cast<uint8_t*>(zs_rring);
  const uint32_t m = blockIdx.x, t = threadIdx.x;
  const uint32_t s = list[m];
  const zs_seg_mem M = mem[m];
  if (M.bad) {
    if (t == 0) {
      zs_lane_res r = {1u, 0u, 0u, 0u};
      res[s] = r;
      lens_out[s] = 0;
      left[atomicAdd(n_left, 1u)] = s;  // (the wave kernel's list)
    }
    return;
  }
  uint32_t* dst = reinterpret_cast<uint32_t*>(out + out_off[s]);
  const uint16_t* scr = scratch + sbase[m];
  const uint4* pt = ptab + pbase[m];
  const uint32_t np = M.npieces;
  uint32_t wdone = 0;  // words stored
  bool far = false;
  uint32_t tb = 0;     // the staged table's first piece
  for (uint32_t i = t; i < ZS_SG_RES_PT && i < np; i += ZS_SG_RES_T) tab[i] = pt[i];
  __syncthreads();
  // the current round (piece k from value i0) and its values
  uint32_t k = 0, i0 = 0;
  uint32_t cur[ZS_SG_RES_E], nxt[ZS_SG_RES_E];
  auto load = [&](const uint4 e, uint32_t j0, uint32_t (&v)[ZS_SG_RES_E]) {
#pragma unroll
    for (uint32_t q = 0; q < ZS_SG_RES_E; q++) {
      const uint32_t i = j0 + q * ZS_SG_RES_T + t;
      v[q] = i < e.y ? scr[e.z + i] : 0u;
    }
  };
  if (np) load(tab[0], 0, cur);
  while (k < np) {
    const uint4 e = tab[k - tb];
    uint32_t k2 = k, j2 = i0 + ZS_SG_RES_R;
    if (j2 >= e.y) {
      k2 = k + 1;
      j2 = 0;
    }
    const bool restage = k2 < np && k2 - tb >= ZS_SG_RES_PT;
#if !(ZS_SEG_EXP & 64)
    // this round's values first, then the next round's loads: they fly while the markers are looked up.
    // (Issued first, the compiler waited for all of them before the first marker: vmcnt(0) on a value loaded
    // a round earlier and copied across the loop.)
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
#endif
    if (k2 < np && !restage) load(tab[k2 - tb], j2, nxt);
    const uint32_t O = e.x;
    // this round's markers.  (Read for all eight values together, a wave's stored words before any pick,
    // the markers cost more except on 4,096 x 256 KiB: 12.90 -> 12.75 ms there, but C5-i 8.17 -> 8.32 ms and
    // the 512-member shard 0.44 -> 0.58 ms; idle lanes' work and registers.)
#pragma unroll
    for (uint32_t q = 0; q < ZS_SG_RES_E; q++) {
      const uint32_t i = i0 + q * ZS_SG_RES_T + t;
      const uint32_t x = cur[q];
      if (i < e.y && x >= 256u) {
        const uint32_t tg = O - (x - 255u);
        if (O + i - tg < ZS_SG_RES_RING - ZS_SG_RES_R) {
          cur[q] = ring[tg & (ZS_SG_RES_RING - 1u)];
        } else if ((tg >> 2) < wdone) {
          const uint32_t w = __hip_atomic_load(dst + (tg >> 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          cur[q] = (w >> (8u * (tg & 3u))) & 0xffu;
        } else {
          far = true;  // a byte of a word not stored yet, out of the ring: the other paths decode the member
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < ZS_SG_RES_E; q++) {
      const uint32_t i = i0 + q * ZS_SG_RES_T + t;
      if (i < e.y) ring[(O + i) & (ZS_SG_RES_RING - 1u)] = (uint8_t)cur[q];
    }
    __syncthreads();
    // the complete words, 16 KiB at a time (and at the end)
    const uint32_t wend = k2 >= np ? (O + e.y) >> 2 : (k2 == k ? (O + j2) >> 2 : (O + e.y) >> 2);
    if (wend - wdone >= 4096u || k2 >= np) {
      for (uint32_t w = wdone + t; w < wend; w += ZS_SG_RES_T) dst[w] = zs_rring[w & (ZS_SG_RES_RING / 4u - 1u)];
      wdone = wend;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // (far markers read them back)
      __syncthreads();
    }
    if (restage) {  // the next table entries (a member of more than ZS_SG_RES_PT pieces)
      tb = k2;
      for (uint32_t i = t; i < ZS_SG_RES_PT && tb + i < np; i += ZS_SG_RES_T) tab[i] = pt[tb + i];
      __syncthreads();
      load(tab[0], j2, nxt);
    }
    k = k2;
    i0 = j2;
#pragma unroll
    for (uint32_t q = 0; q < ZS_SG_RES_E; q++) cur[q] = nxt[q];
  }
  if (M.total & 3u) {  // the last bytes one by one: nothing is stored past the member's end
    uint8_t* db = out + out_off[s];
    if (t < (M.total & 3u)) db[4u * wdone + t] = ring[(4u * wdone + t) & (ZS_SG_RES_RING - 1u)];
  }
  far = __syncthreads_or(far);
  if (t == 0) {
    if (!far) atomicAdd(n_ok, 1u);  // (statistics: zs_last_inflate_seg_count)
    else left[atomicAdd(n_left, 1u)] = s;
    zs_lane_res r = {far ? 1u : 0u, far ? 0u : M.total, M.consumed, M.want};
    res[s] = r;
    lens_out[s] = far ? 0u : M.total;
  }
}

#define ZS_SEG_WALK_INST(D, W, ST)                                                                                 \
  template __global__ void zs_k_seg_walk<D, W, ST>(const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*,  \
                                               uint32_t, const uint32_t*, uint32_t, int, const uint64_t*,          \
                                               const uint32_t*, zs_seg_blk*, zs_seg_lane*, zcode*, zs_seg_ent*,    \
                                               zs_seg_mem*, uint32_t*, uint32_t*, uint32_t, int);
ZS_SEG_WALK_INST(false, 1024u, false)
ZS_SEG_WALK_INST(false, 1024u, true)
ZS_SEG_WALK_INST(true, 1024u, false)
ZS_SEG_WALK_INST(false, 2048u, true)
ZS_SEG_WALK_INST(true, 2048u, false)
#define ZS_SEG_DEC_INST(D, W)                                                                                       \
  template __global__ void zs_k_seg_decode<D, W>(const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*, \
                                                 const uint32_t*, const uint32_t*, const zs_seg_blk*,              \
                                                 const zs_seg_lane*,                                               \
                                                 const zcode*, zs_seg_mem*, const uint64_t*, uint16_t*);
ZS_SEG_DEC_INST(false, false)
ZS_SEG_DEC_INST(false, true)
ZS_SEG_DEC_INST(true, false)

template __global__ void zs_k_seg_resolve<256u, 32768u>(const uint32_t*, const zs_seg_mem*, const uint32_t*,
                                                        const uint4*, const uint64_t*, const uint16_t*, uint8_t*,
                                                        const uint64_t*, zs_lane_res*, uint32_t*, uint32_t*,
                                                        uint32_t*, uint32_t*);
template __global__ void zs_k_seg_resolve<512u, 65536u>(const uint32_t*, const zs_seg_mem*, const uint32_t*,
                                                        const uint4*, const uint64_t*, const uint16_t*, uint8_t*,
                                                        const uint64_t*, zs_lane_res*, uint32_t*, uint32_t*,
                                                        uint32_t*, uint32_t*);
