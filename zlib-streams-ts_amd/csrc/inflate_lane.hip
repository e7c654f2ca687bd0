// inflate_lane.hip -- the lane-per-member inflate path of zs_inflate_batch*
// (see the comment below); zs_k_inflate in inflate.hip is the exact path.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_inflate.h"
#include "zs_inftab.h"

// One LANE per member.  The exact kernel above spends a whole wave on one
// stream because it re-enacts the stream layer's call boundaries; a member
// whose decoding those boundaries cannot change decodes straight through in one
// lane instead: a deflate64 member (the reference decodes it with the slow state
// machine only, whose window copies are exact), or a deflate / zlib / gzip member
// that one inflate() call of the reference decodes whole (see ZS_INF_REF_WRAP
// below).  zlib's own tables (inflate_table above, so invalid codes are
// recognised exactly as the reference does), a 64-bit bit buffer, output written
// to HBM and match history read back from it.  A member takes the exact path
// instead (zs_k_inflate over the bailed members) on ANY condition that is not a
// clean end of stream -- a data error, truncated input, a dictionary request,
// gzip header fields, a checksum or length mismatch, or output capacity -- so
// statuses, phases and messages always come from the exact state machine.
struct zs_lane_tabs {
  zcode codes[ENOUGH_LENS + ENOUGH_DISTS_9];
  uint16_t lens[320];
  uint16_t work[288];
};

struct zs_lane_reader {
  const uint32_t* w4;  // the aligned words holding the member's bytes
  uint32_t sh, last;   // the member's offset in its first word; index of the word holding its last byte
  uint32_t n, pos;  // bytes moved into hold so far
  uint64_t hold;
  uint32_t bits;
  uint32_t pf;      // input bytes [pos, pos + 4), loaded one refill ahead (zero past the end)
};

// input bytes [at, at + 4), zero past the end: two aligned word loads with
// clamped indices and a funnel shift -- no branch, so the load stays in flight
// until the refill that uses it (a branch per byte made the compiler wait on
// each byte in turn)
static __device__ __forceinline__ uint32_t zs_lr_load4(const zs_lane_reader& R, uint32_t at) {
  const uint32_t q = (at + R.sh) >> 2;
  const uint32_t lo = R.w4[min(q, R.last)], hi = R.w4[min(q + 1u, R.last)];
  const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, R.sh);
  const uint32_t valid = at < R.n ? R.n - at : 0u;
  return valid >= 4u ? v : v & ((1u << (8u * valid)) - 1u);
}
// bits < 32 -> bits >= 32: the prefetched word enters hold and the next one is
// requested, so its latency overlaps the decoding of the bits just added
static __device__ __forceinline__ void zs_lr_fill(zs_lane_reader& R) {
  R.hold |= (uint64_t)R.pf << R.bits;
  R.bits += 32;
  R.pos += 4;
  R.pf = zs_lr_load4(R, R.pos);
}
// bits consumed so far
static __device__ __forceinline__ uint64_t zs_lr_bitpos(const zs_lane_reader& R) {
  return (uint64_t)R.pos * 8u - R.bits;
}
// consumed bits beyond the input: a truncated stream (the exact path reports it)
static __device__ __forceinline__ bool zs_lr_over(const zs_lane_reader& R) {
  return zs_lr_bitpos(R) > (uint64_t)R.n * 8u;
}
static __device__ __forceinline__ uint32_t zs_lr_take(zs_lane_reader& R, uint32_t k) {  // k <= 32
  if (R.bits < k) zs_lr_fill(R);
  const uint32_t v = (uint32_t)R.hold & (k == 32 ? 0xffffffffu : ((1u << k) - 1));
  R.hold >>= k;
  R.bits -= k;
  return v;
}
static __device__ __forceinline__ void zs_lr_align(zs_lane_reader& R) {
  const uint32_t d = R.bits & 7u;
  R.hold >>= d;
  R.bits -= d;
}

// decode one Huffman symbol with a zlib table (root `rbits`); returns the final entry
static __device__ __forceinline__ zcode zs_lane_decode(zs_lane_reader& R, const zcode* t, uint32_t rbits) {
  if (R.bits < 32) zs_lr_fill(R);
  zcode here = t[(uint32_t)R.hold & ((1u << rbits) - 1)];
  if (C_OP(here) && (C_OP(here) & 0xf0) == 0) {  // second-level table
    const uint32_t rb = C_BITS(here);
    const zcode last = here;
    here = t[C_VAL(last) + (((uint32_t)R.hold & ((1u << (rb + C_OP(last))) - 1)) >> rb)];
    R.hold >>= rb;
    R.bits -= rb;
  }
  R.hold >>= C_BITS(here);
  R.bits -= C_BITS(here);
  return here;
}

// LDS root tables of one lane: 8-bit lit/len and 6-bit distance roots, u16
// entries (code length << 12 | symbol), 0 = code longer than the root (the lane
// then decodes with its zlib table in HBM).  640 B per lane: four 64-lane
// workgroups fill a CU's 160 KB.
#define ZS_LROOT 8u
#define ZS_DROOT 6u
struct zs_lane_lds {
  uint16_t lit[1u << ZS_LROOT];
  uint16_t dist[1u << ZS_DROOT];
};

static __device__ void zs_lane_root(uint16_t* tab, uint32_t rbits, const uint16_t* lens, uint32_t n) {
  uint32_t count[16], next[16];
  for (uint32_t l = 0; l < 16; l++) count[l] = 0;
  for (uint32_t i = 0; i < n; i++) count[lens[i]]++;
  count[0] = 0;
  uint32_t code = 0;
  for (uint32_t l = 1; l < 16; l++) {  // canonical first codes (RFC 1951 3.2.2)
    code = (code + count[l - 1]) << 1;
    next[l] = code;
  }
  for (uint32_t k = 0; k < (1u << rbits); k++) tab[k] = 0;
  for (uint32_t sym = 0; sym < n; sym++) {
    const uint32_t l = lens[sym];
    if (l == 0) continue;
    const uint32_t c = next[l]++;
    if (l > rbits) continue;
    const uint32_t r = __builtin_bitreverse32(c) >> (32 - l);  // the stream sends codes MSB first
    for (uint32_t k = r; k < (1u << rbits); k += 1u << l) tab[k] = (uint16_t)((l << 12) | sym);
  }
}

// a root-table symbol as the zlib table entry the decoder consumes (zs_lbase /
// zs_dbase's ops: 16 + extra bits, deflate64 128 + extra bits)
static __device__ __forceinline__ zcode zs_lit_entry(uint32_t sym, bool d64) {
  if (sym < 256) return zpack(0, 0, sym);
  if (sym == 256) return zpack(32 + 64, 0, 0);
  const uint32_t c = sym - 257;  // length codes: base / extra bits (inflate/constants.ts:8-23)
  const uint32_t f = d64 ? 128u : 16u;
  if (c < 8) return zpack(f, 0, c + 3);
  if (c == 28) return d64 ? zpack(128 + 16, 0, 3) : zpack(16, 0, 258);  // deflate64: 3 + 16 extra bits
  const uint32_t x = (c >> 2) - 1;
  return zpack(f + x, 0, ((4u | (c & 3u)) << x) + 3u);
}
static __device__ __forceinline__ zcode zs_dist_entry(uint32_t d, bool d64) {
  const uint32_t f = d64 ? 128u : 16u;
  if (d < 4) return zpack(f, 0, d + 1);
  const uint32_t x = (d >> 1) - 1;  // codes 30/31 (deflate64 only): 32769 / 49153 + 14 extra bits
  return zpack(f + x, 0, ((2u | (d & 1u)) << x) + 1u);
}

// Output of one lane, write-combined in registers: the bytes of the current
// 16-byte aligned unit collect in u0..u2 (its completed words, oldest first)
// and cw (the word being filled), and a completed unit leaves as ONE 16-byte
// store instead of sixteen byte stores (one lane's bytes are on one line; 64
// lanes' byte stores were 64 separate transactions each).  P counts bytes from
// the unit-aligned base below the member's first byte (out_off is 4-aligned, so
// the first unit is entered at word w0 = (dst & 15) / 4 and its earlier words
// -- another member's -- are never stored).
struct zs_lane_out {
  uint32_t* base;  // 16-byte aligned, <= dst
  uint32_t P, w0;
  uint32_t u0, u1, u2, cw;
  __device__ __forceinline__ void init(uint8_t* dst) {
    const uintptr_t a = (uintptr_t)dst;
    base = reinterpret_cast<uint32_t*>(a & ~(uintptr_t)15);
    P = (uint32_t)(a & 15u);
    w0 = P >> 2;
    u0 = u1 = u2 = cw = 0;
  }
  // the completed unit at P - 16 (P a multiple of 16): one 16-byte store, or
  // dword stores from w0 on for the member's first unit
  __device__ __forceinline__ void store_unit(uint32_t w3) {
    uint32_t* q = base + ((P - 16u) >> 2);
    if (P - 16u >= 16u || w0 == 0) {
      *reinterpret_cast<uint4*>(q) = make_uint4(u0, u1, u2, w3);
    } else {
      if (w0 <= 1) q[1] = u1;
      if (w0 <= 2) q[2] = u2;
      q[3] = w3;
    }
  }
  // a completed word (P a multiple of 4 after it)
  __device__ __forceinline__ void word(uint32_t w) {
    P += 4;
    if ((P & 15u) == 0) {
      store_unit(w);
    } else {
      u0 = u1;
      u1 = u2;
      u2 = w;
    }
  }
  // n (1..4) bytes, the low bytes of v (bytes above n zero)
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    const uint32_t a = P & 3u;
    cw |= v << (8u * a);
    if (a + n >= 4u) {
      const uint32_t w = cw;
      cw = a ? v >> (32u - 8u * a) : 0u;  // the bytes past the word
      P -= a;
      word(w);
      P += a + n - 4u;
    } else {
      P += n;
    }
  }
  __device__ __forceinline__ void byte(uint32_t b) { put(b & 0xffu, 1u); }
  // the current unit's bytes so far go to memory (dword stores; the last
  // word's bytes past P are inside the member's capacity and are rewritten
  // later): after this, every byte below P is in memory
  __device__ __forceinline__ void spill() {
    const uint32_t ub = P & ~15u, wi = (P >> 2) & 3u;  // completed words of this unit
    uint32_t* q = base + (ub >> 2);
    const uint32_t first = ub == 0 ? w0 : 0u;
    // word i of the unit (i < wi) is u[3 - wi + i]
    if (wi >= 3 && first <= 0) q[0] = u0;
    if (wi >= 2 && first <= wi - 2) q[wi - 2] = u1;
    if (wi >= 1 && first <= wi - 1) q[wi - 1] = u2;
    if ((P & 3u) && first <= wi) q[wi] = cw;
  }
  // after bytes were stored straight to memory up to P: the current unit's
  // words back into the registers
  __device__ __forceinline__ void reload() {
    const uint32_t ub = P & ~15u, wi = (P >> 2) & 3u;
    const uint32_t* q = base + (ub >> 2);
    // only words up to the one holding P are read (the unit may end past the buffer)
    const uint32_t x0 = q[0], x1 = wi >= 1 ? q[1] : 0u, x2 = wi >= 2 ? q[2] : 0u, x3 = wi >= 3 ? q[3] : 0u;
    // the shift register holds word i (i < wi) at u[3 - wi + i]
    u2 = wi == 3 ? x2 : wi == 2 ? x1 : wi == 1 ? x0 : 0u;
    u1 = wi == 3 ? x1 : wi == 2 ? x0 : 0u;
    u0 = wi == 3 ? x0 : 0u;
    const uint32_t a = P & 3u;
    const uint32_t xw = wi == 0 ? x0 : wi == 1 ? x1 : wi == 2 ? x2 : x3;
    cw = a ? xw & ((1u << (8u * a)) - 1u) : 0u;
  }
};

__global__ __launch_bounds__(64) void zs_k_inflate_lane(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint32_t* __restrict__ out_cap, int wbits, uint32_t n_members,
                                                        zs_lane_tabs* __restrict__ tabs, zs_lane_res* __restrict__ res,
                                                        uint32_t* __restrict__ lens_out, int flags,
                                                        uint32_t wave_min) {
  extern __shared__ zs_lane_lds LL[];  // blockDim.x entries
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_members) return;
  if (wave_min && in_len[s] > wave_min) return;  // a large member: zs_k_inflate_wave decodes it (inflate_wave.hip)
  zs_lane_tabs& T = tabs[s];
  zs_lane_lds& F = LL[threadIdx.x];
  zs_lane_reader R;
  {
    const uint8_t* src = in + in_off[s];
    R.n = in_len[s];
    R.sh = (uint32_t)((uintptr_t)src & 3u);
    // an empty member reads (and masks off) a word of in_len[] instead: its own address may be past the buffer
    R.w4 = R.n ? reinterpret_cast<const uint32_t*>(src - R.sh) : in_len;
    R.last = R.n ? (R.sh + R.n - 1u) >> 2 : 0u;
  }
  R.pos = 0;
  R.hold = 0;
  R.bits = 0;
  R.pf = zs_lr_load4(R, 0);
  uint8_t* dst = out + out_off[s];
  zs_lane_out W;
  W.init(dst);
  // This path decodes a member in one go, without the stream layer's call
  // boundaries.  A member whose input fits one 32 KiB sub-chunk and whose
  // output fits one 64 KiB output buffer is decoded by ONE inflate() call of
  // the reference (streams.ts:6-7,78-93) that never copies from the window, so
  // the window-wrap behaviour (ZS_INF_REF_WRAP) cannot arise; any other member
  // takes the exact path, which emulates the calls.
  // deflate64 members never reach inflate_fast in the reference (inflate.ts:841),
  // so they carry no call-boundary behaviour and decode here at any size.
  const bool d64 = wbits == -16;
  const bool ref_wrap = (flags & ZS_INF_REF_WRAP) != 0 && !d64;
  const uint32_t cap = ref_wrap ? min(out_cap[s], 65536u) : out_cap[s];
  const uint32_t lmask = d64 ? 31u : 15u;  // length extra-bit mask (inflate.ts:891)
  uint32_t total = 0;
  zs_lane_res r = {1u, 0u, 0u, 0u};
  const int wrap = wbits < 0 ? 0 : (wbits >> 4) + 5;  // inflate.ts:152-160
  bool bail = ref_wrap && R.n > 32768u;  // several sub-chunks: exact path
  // ---- wrapper header (inflate.ts:377-580): plain zlib / gzip headers only
  if (!bail && wrap) {
    const uint32_t b0 = zs_lr_take(R, 8), b1 = zs_lr_take(R, 8);
    if ((wrap & 2) && b0 == 0x1f && b1 == 0x8b) {
      const uint32_t cm = zs_lr_take(R, 8), flg = zs_lr_take(R, 8);
      zs_lr_take(R, 32);  // MTIME
      zs_lr_take(R, 16);  // XFL, OS
      if (cm != 8 || flg != 0) bail = true;  // FEXTRA / FNAME / FCOMMENT / FHCRC / reserved: exact path
    } else if (wrap & 1) {
      if (((b0 << 8) | b1) % 31 || (b0 & 15) != 8 || (b0 >> 4) + 8 > 15 || (b1 & 0x20)) bail = true;
    } else {
      bail = true;  // "incorrect header check"
    }
  }
  // ---- blocks
  bool last = false;
  while (!bail && !last) {
    last = zs_lr_take(R, 1) != 0;
    const uint32_t type = zs_lr_take(R, 2);
    const zcode* lt;
    const zcode* dt;
    uint32_t lbits, dbits;
    if (type == 0) {  // stored (inflate.ts:615-660)
      zs_lr_align(R);
      const uint32_t len = zs_lr_take(R, 16), nlen = zs_lr_take(R, 16);
      if (len != (nlen ^ 0xffffu) || zs_lr_over(R) || total + len > cap) { bail = true; break; }
      for (uint32_t i = 0; i < len; i++) W.byte(zs_lr_take(R, 8));
      total += len;
      if (zs_lr_over(R)) { bail = true; break; }
      continue;
    }
    if (type == 1) {  // fixed tables (inflate.ts:218-280)
      uint32_t sym, used;
      for (sym = 0; sym < 144; sym++) T.lens[sym] = 8;
      for (; sym < 256; sym++) T.lens[sym] = 9;
      for (; sym < 280; sym++) T.lens[sym] = 7;
      for (; sym < 288; sym++) T.lens[sym] = 8;
      lbits = 9;
      zs_inflate_table(LENS, T.lens, 288, T.codes, &lbits, T.work, d64, &used);
      for (sym = 0; sym < 32; sym++) T.lens[sym] = 5;
      dbits = 5;
      zs_inflate_table(DISTS, T.lens, 32, T.codes + used, &dbits, T.work, d64, &sym);
      lt = T.codes;
      dt = T.codes + used;
      for (sym = 0; sym < 288; sym++) T.lens[sym] = sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8;
      zs_lane_root(F.lit, ZS_LROOT, T.lens, 286);  // 286/287 stay out of the root: invalid codes decode via T
      for (sym = 0; sym < 30; sym++) T.lens[sym] = 5;
      zs_lane_root(F.dist, ZS_DROOT, T.lens, d64 ? 32 : 30);  // deflate: 30/31 likewise
    } else if (type == 2) {  // dynamic (inflate.ts:662-836)
      const uint32_t nlen = zs_lr_take(R, 5) + 257, ndist = zs_lr_take(R, 5) + 1, ncode = zs_lr_take(R, 4) + 4;
      if (nlen > 286 || (!d64 && ndist > 30)) { bail = true; break; }
      uint32_t i;
      for (i = 0; i < ncode; i++) T.lens[ZS_BL_ORDER[i]] = (uint16_t)zs_lr_take(R, 3);
      for (; i < 19; i++) T.lens[ZS_BL_ORDER[i]] = 0;
      uint32_t cbits = 7, used;
      if (zs_inflate_table(CODES, T.lens, 19, T.codes, &cbits, T.work, d64, &used)) { bail = true; break; }
      i = 0;
      while (i < nlen + ndist) {
        const zcode here = zs_lane_decode(R, T.codes, cbits);
        const uint32_t v = C_VAL(here);
        if (v < 16) { T.lens[i++] = (uint16_t)v; continue; }
        uint32_t rep, val = 0;
        if (v == 16) {
          if (i == 0) { bail = true; break; }
          val = T.lens[i - 1];
          rep = 3 + zs_lr_take(R, 2);
        } else if (v == 17) {
          rep = 3 + zs_lr_take(R, 3);
        } else {
          rep = 11 + zs_lr_take(R, 7);
        }
        if (i + rep > nlen + ndist) { bail = true; break; }
        while (rep--) T.lens[i++] = (uint16_t)val;
      }
      if (bail || zs_lr_over(R) || T.lens[256] == 0) { bail = true; break; }
      lbits = 9;
      uint32_t lused, dused;
      if (zs_inflate_table(LENS, T.lens, nlen, T.codes, &lbits, T.work, d64, &lused)) { bail = true; break; }
      dbits = 6;
      if (zs_inflate_table(DISTS, T.lens + nlen, ndist, T.codes + lused, &dbits, T.work, d64, &dused)) {
        bail = true;
        break;
      }
      lt = T.codes;
      dt = T.codes + lused;
      zs_lane_root(F.lit, ZS_LROOT, T.lens, nlen);
      zs_lane_root(F.dist, ZS_DROOT, T.lens + nlen, ndist);
    } else {
      bail = true;  // "invalid block type"
      break;
    }
    // symbols (inffast.ts:5-228 semantics, without the call boundaries)
    for (;;) {
      if (R.bits < 32) zs_lr_fill(R);
      zcode here;
      const uint32_t fe = F.lit[(uint32_t)R.hold & ((1u << ZS_LROOT) - 1)];
      if (fe >> 12) {
        R.hold >>= fe >> 12;
        R.bits -= fe >> 12;
        here = zs_lit_entry(fe & 0x1ffu, d64);
      } else {
        here = zs_lane_decode(R, lt, lbits);
      }
      uint32_t op = C_OP(here);
      if (op == 0) {
        if (total >= cap) { bail = true; break; }
        W.byte(C_VAL(here));
        total++;
        continue;
      }
      if (op & 32) break;                   // end of block
      if (op & 64) { bail = true; break; }  // "invalid literal/length code"
      uint32_t len = C_VAL(here) + zs_lr_take(R, op & lmask);
      if (R.bits < 32) zs_lr_fill(R);
      const uint32_t de = F.dist[(uint32_t)R.hold & ((1u << ZS_DROOT) - 1)];
      if (de >> 12) {
        R.hold >>= de >> 12;
        R.bits -= de >> 12;
        here = zs_dist_entry(de & 0x1fu, d64);
      } else {
        here = zs_lane_decode(R, dt, dbits);
      }
      op = C_OP(here);
      if (op & 64) { bail = true; break; }  // "invalid distance code"
      const uint32_t dist = C_VAL(here) + zs_lr_take(R, op & 15u);
      if (dist > total || total + len > cap) { bail = true; break; }  // too far back / capacity
      const uint8_t* from = dst + total - dist;
      uint8_t* to = dst + total;
      const uint32_t fsh = (uint32_t)((uintptr_t)from & 3u);
      const uint32_t* fw = reinterpret_cast<const uint32_t*>(from - fsh);
      if (dist >= 16u + (W.P & 15u)) {
        // every source byte of every 16-byte round lies below the unit being
        // combined, so is in memory already: 16 bytes per round trip, into the
        // write combiner a word at a time
        for (uint32_t i = 0; i < len; i += 16) {
          uint32_t x[5];
#pragma unroll
          for (int k = 0; k < 5; k++) x[k] = fw[(i >> 2) + (uint32_t)k];
          const uint32_t rem = len - i;
#pragma unroll
          for (uint32_t k = 0; k < 4; k++) {
            const uint32_t wd = __builtin_amdgcn_alignbyte(x[k + 1], x[k], fsh);
            if (rem >= 4u * k + 4u) {
              W.put(wd, 4u);
            } else if (rem > 4u * k) {
              const uint32_t nb = rem - 4u * k;
              W.put(wd & ((1u << (8u * nb)) - 1u), nb);
            }
          }
        }
        total += len;
        continue;
      }
      // a source within the unit being combined: its bytes go to memory, the
      // copy stores bytes straight to memory, and the combiner picks the unit up
      W.spill();
      // A copy waits for its source bytes once per chunk (loads after the
      // stores of the chunk before), so the chunk is as wide as the distance
      // allows.  Source words are aligned loads funnel-shifted into place; a
      // word that is read always holds at least one byte of the output region
      // (so never leaves its pages), and only bytes below `to` are used.
      if (dist >= 16) {  // 16 bytes per round trip
        for (uint32_t i = 0; i < len; i += 16) {
          uint32_t x[5];
#pragma unroll
          for (int k = 0; k < 5; k++) x[k] = fw[(i >> 2) + (uint32_t)k];
#pragma unroll
          for (uint32_t j = 0; j < 16; j++) {
            const uint32_t wd = __builtin_amdgcn_alignbyte(x[(j >> 2) + 1], x[j >> 2], fsh);
            if (i + j < len) to[i + j] = (uint8_t)(wd >> (8 * (j & 3)));
          }
        }
      } else if (dist >= 8) {  // 8 independent loads, then 8 stores: one memory round trip per 8 bytes
        for (uint32_t i = 0; i < len; i += 8) {
          uint8_t b[8];
#pragma unroll
          for (int k = 0; k < 8; k++) b[k] = i + k < len ? from[i + k] : 0;
#pragma unroll
          for (int k = 0; k < 8; k++)
            if (i + k < len) to[i + k] = b[k];
        }
      } else {
        // overlapping copy, period dist < 8: the dist bytes before `to` are
        // read once (three words, clamped to the last written one) and the
        // run is stored from registers -- not a round trip per byte
        const uint32_t last = (uint32_t)((to - 1) - (from - fsh)) >> 2;
        const uint32_t x0 = fw[0], x1 = fw[min(1u, last)], x2 = fw[min(2u, last)];
        const uint32_t p0 = __builtin_amdgcn_alignbyte(x1, x0, fsh), p1 = __builtin_amdgcn_alignbyte(x2, x1, fsh);
        uint32_t j = 0;
        for (uint32_t i = 0; i < len; i++) {
          to[i] = (uint8_t)((j < 4 ? p0 >> (8 * j) : p1 >> (8 * (j - 4))) & 0xffu);
          j = j + 1 == dist ? 0u : j + 1;
        }
      }
      total += len;
      W.P += len;
      W.reload();
    }
    if (zs_lr_over(R)) bail = true;
  }
  if (!bail) W.spill();  // the last unit's bytes
  // ---- trailer (inflate.ts:1006-1036)
  if (!bail && wrap) {
    zs_lr_align(R);
    const uint32_t a = zs_lr_take(R, 32);
    if (wrap & 2 && !(wrap & 1)) {  // gzip: crc32 LE, then ISIZE LE
      r.want = a;
      const uint32_t isize = zs_lr_take(R, 32);
      if (isize != total) bail = true;
    } else {
      r.want = __builtin_bswap32(a);  // zlib: adler32 big-endian
    }
    if (zs_lr_over(R)) bail = true;
  }
  if (!bail) {
    r.bail = 0;
    r.out_len = total;
    r.consumed = (uint32_t)((zs_lr_bitpos(R) + 7u) >> 3);
  }
  res[s] = r;
  lens_out[s] = r.out_len;  // for the checksum pass over the decoded bytes
}

size_t zs_inflate_lane_scratch_bytes() { return sizeof(zs_lane_tabs); }
size_t zs_inflate_lane_lds_bytes() { return sizeof(zs_lane_lds); }

