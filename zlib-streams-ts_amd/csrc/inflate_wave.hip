// inflate_wave.hip -- the wave-per-member inflate path for LARGE members.
//
// The lane path (inflate_lane.hip) gives each member one lane, so a member's
// decode rate is that of one lane whose every match copy is a round trip
// through HBM (its history is the output it just stored): a few MB/s.  That is
// the right trade for a batch of many 64 KiB members, but one large member in a
// batch (C5-ii's 2 MB deflate64 fixture) then sets the whole
// batch's time.  A member whose input exceeds a threshold (option
// inflate_wave_min) decodes here instead, concurrently with the lane kernel:
//  * one wave per member; the Huffman decode is wave-uniform (table entries and
//    input words moved to SGPRs with readfirstlane, so the symbol loop is scalar
//    control flow around one LDS lookup per code);
//  * the last 64 KiB of output live in an LDS ring (the deflate64 window), so a
//    match copy reads its source from LDS -- 64 bytes per lane-parallel step,
//    a period < 64 copy stored from one read per lane -- and every byte is also
//    stored to HBM, never read back;
//  * zlib's own tables (inflate_table, zs_inftab.h) in LDS, built by all lanes
//    on identical values.
// Outcome contract = the lane path's (zs_lane_res): any condition that is not a
// clean end of stream sets bail and the exact kernel (zs_k_inflate) redecodes
// the member, so statuses, phases and messages come from the exact state
// machine (inflate.ts:332-1185).  Symbol semantics: inffast.ts:5-228 without
// call boundaries -- valid for deflate64 at any size (the reference never runs
// inflate_fast on it, inflate.ts:841) and for the other formats when the
// reference's window-wrap copy is not being reproduced (the host routes
// members here only then).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_inflate.h"
#include "zs_inftab.h"

#define ZS_WRING (1u << 16)  // history ring: the deflate64 window (deflate's 32 KiB fits)
#define ZS_WMASK (ZS_WRING - 1u)

struct zs_wave_lds {
  uint8_t ring[ZS_WRING];
  uint32_t inw[1024];  // ZS_WIN_IN staged input words
  zcode codes[ENOUGH_LENS + ENOUGH_DISTS_9];
  uint16_t lens[320];
  uint16_t work[288];
};

static __device__ __forceinline__ uint32_t zs_u(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// wave-uniform bit reader: the zs_lane_reader scheme (clamped aligned words,
// one refill ahead) with every value in SGPRs.  The input words are staged in
// LDS, 4 KiB at a time by the whole wave: a refill is then an LDS read, which
// the table lookups' waits cover, where a direct load would wait behind the
// output stores (vmcnt) or -- as a scalar load -- make every table lookup's
// lgkmcnt wait for it.
#define ZS_WIN_IN 1024u  // staged input words
struct zs_wave_reader {
  const uint32_t* w4;  // the aligned words holding the member's bytes
  uint32_t* inw;       // LDS: words [qb, qb + ZS_WIN_IN) of w4 (clamped to `last`)
  uint32_t qb;
  uint32_t sh, last, n, pos;
  uint64_t hold;
  uint32_t bits;
  uint32_t pf;
};

static __device__ __forceinline__ void zs_wr_stage(zs_wave_reader& R, uint32_t q) {
  R.qb = q;
#pragma unroll 4
  for (uint32_t i = threadIdx.x; i < ZS_WIN_IN; i += 64) R.inw[i] = R.w4[min(q + i, R.last)];
}
static __device__ __forceinline__ uint32_t zs_wr_load4(zs_wave_reader& R, uint32_t at) {
  const uint32_t q = (at + R.sh) >> 2;
  if (q + 1u >= R.qb + ZS_WIN_IN) zs_wr_stage(R, q);
  const uint32_t lo = zs_u(R.inw[q - R.qb]), hi = zs_u(R.inw[q + 1u - R.qb]);
  // (at + sh) & 3 is sh except after a stored block's seek
  const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * ((at + R.sh) & 3u)));
  const uint32_t valid = at < R.n ? R.n - at : 0u;
  return valid >= 4u ? v : v & ((1u << (8u * valid)) - 1u);
}
static __device__ __forceinline__ void zs_wr_fill(zs_wave_reader& R) {
  R.hold |= (uint64_t)R.pf << R.bits;
  R.bits += 32;
  R.pos += 4;
  R.pf = zs_wr_load4(R, R.pos);
}
static __device__ __forceinline__ uint64_t zs_wr_bitpos(const zs_wave_reader& R) { return (uint64_t)R.pos * 8u - R.bits; }
static __device__ __forceinline__ bool zs_wr_over(const zs_wave_reader& R) { return zs_wr_bitpos(R) > (uint64_t)R.n * 8u; }
static __device__ __forceinline__ uint32_t zs_wr_take(zs_wave_reader& R, uint32_t k) {  // k <= 32
  if (R.bits < k) zs_wr_fill(R);
  const uint32_t v = (uint32_t)R.hold & (k == 32 ? 0xffffffffu : ((1u << k) - 1));
  R.hold >>= k;
  R.bits -= k;
  return v;
}
static __device__ __forceinline__ void zs_wr_align(zs_wave_reader& R) {
  const uint32_t d = R.bits & 7u;
  R.hold >>= d;
  R.bits -= d;
}
// restart the reader at byte `at` (after a stored block copied straight from the input)
static __device__ __forceinline__ void zs_wr_seek(zs_wave_reader& R, uint32_t at) {
  R.pos = at;
  R.hold = 0;
  R.bits = 0;
  R.pf = zs_wr_load4(R, at);
}
static __device__ __forceinline__ zcode zs_wr_decode(zs_wave_reader& R, const zcode* t, uint32_t rbits) {
  if (R.bits < 32) zs_wr_fill(R);
  zcode here = zs_u(t[(uint32_t)R.hold & ((1u << rbits) - 1)]);
  if (C_OP(here) && (C_OP(here) & 0xf0) == 0) {  // second-level table
    const uint32_t rb = C_BITS(here);
    const zcode last = here;
    here = zs_u(t[C_VAL(last) + (((uint32_t)R.hold & ((1u << (rb + C_OP(last))) - 1)) >> rb)]);
    R.hold >>= rb;
    R.bits -= rb;
  }
  R.hold >>= C_BITS(here);
  R.bits -= C_BITS(here);
  return here;
}

__global__ __launch_bounds__(64) void zs_k_inflate_wave(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint32_t* __restrict__ out_cap, int wbits,
                                                        const uint32_t* __restrict__ list, uint32_t n_list,
                                                        zs_lane_res* __restrict__ res, uint32_t* __restrict__ lens_out) {
  extern __shared__ uint8_t zs_wsm[];
  zs_wave_lds& W = *reinterpret_cast<zs_wave_lds*>(zs_wsm);
  if (blockIdx.x >= n_list) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t s = zs_u(list[blockIdx.x]);
  const uint8_t* src = in + in_off[s];
  zs_wave_reader R;
  R.n = zs_u(in_len[s]);
  R.sh = (uint32_t)((uintptr_t)src & 3u);
  R.w4 = R.n ? reinterpret_cast<const uint32_t*>(src - R.sh) : in_len;  // an empty member reads (and masks) in_len[]
  R.last = R.n ? (R.sh + R.n - 1u) >> 2 : 0u;
  R.inw = W.inw;
  zs_wr_stage(R, 0);
  R.pos = 0;
  R.hold = 0;
  R.bits = 0;
  R.pf = zs_wr_load4(R, 0);
  uint8_t* dst = out + out_off[s];
  const uint32_t cap = zs_u(out_cap[s]);
  const bool d64 = wbits == -16;
  const uint32_t lmask = d64 ? 31u : 15u;  // length extra-bit mask (inflate.ts:891)
  const int wrap = wbits < 0 ? 0 : (wbits >> 4) + 5;  // inflate.ts:152-160
  uint32_t total = 0;
  zs_lane_res r = {1u, 0u, 0u, 0u};
  bool bail = false;
  // ---- wrapper header (inflate.ts:377-580): plain zlib / gzip headers only, as the lane path
  if (wrap) {
    const uint32_t b0 = zs_wr_take(R, 8), b1 = zs_wr_take(R, 8);
    if ((wrap & 2) && b0 == 0x1f && b1 == 0x8b) {
      const uint32_t cm = zs_wr_take(R, 8), flg = zs_wr_take(R, 8);
      zs_wr_take(R, 32);  // MTIME
      zs_wr_take(R, 16);  // XFL, OS
      if (cm != 8 || flg != 0) bail = true;
    } else if (wrap & 1) {
      if (((b0 << 8) | b1) % 31 || (b0 & 15) != 8 || (b0 >> 4) + 8 > 15 || (b1 & 0x20)) bail = true;
    } else {
      bail = true;
    }
  }
  bool last = false;
  while (!bail && !last) {
    last = zs_wr_take(R, 1) != 0;
    const uint32_t type = zs_wr_take(R, 2);
    uint32_t lbits, dbits, lused;
    if (type == 0) {  // stored (inflate.ts:615-660): bytes straight from the input, 64 per step
      zs_wr_align(R);
      const uint32_t len = zs_wr_take(R, 16), nlen = zs_wr_take(R, 16);
      const uint32_t at = (uint32_t)(zs_wr_bitpos(R) >> 3);
      if (len != (nlen ^ 0xffffu) || zs_wr_over(R) || at + len > R.n || total + len > cap) { bail = true; break; }
      for (uint32_t i = 0; i < len; i += 64) {
        const uint32_t k = i + lane;
        if (k < len) {
          const uint8_t b = src[at + k];
          W.ring[(total + k) & ZS_WMASK] = b;
          dst[total + k] = b;
        }
      }
      total += len;
      zs_wr_seek(R, at + len);
      continue;
    }
    if (type == 1) {  // fixed tables (inflate.ts:218-280)
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
    } else if (type == 2) {  // dynamic (inflate.ts:662-836)
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
      bail = true;  // "invalid block type"
      break;
    }
    lbits = zs_u(lbits);
    dbits = zs_u(dbits);
    const zcode* lt = W.codes;
    const zcode* dt = W.codes + zs_u(lused);
    // symbols (inffast.ts:5-228 semantics, without the call boundaries)
    for (;;) {
      zcode here = zs_wr_decode(R, lt, lbits);
      uint32_t op = C_OP(here);
      if (op == 0) {
        if (total >= cap) { bail = true; break; }
        if (lane == 0) {
          const uint8_t b = (uint8_t)C_VAL(here);
          W.ring[total & ZS_WMASK] = b;
          dst[total] = b;
        }
        total++;
        continue;
      }
      if (op & 32) break;                   // end of block
      if (op & 64) { bail = true; break; }  // "invalid literal/length code"
      const uint32_t len = C_VAL(here) + zs_wr_take(R, op & lmask);
      here = zs_wr_decode(R, dt, dbits);
      op = C_OP(here);
      if (op & 64) { bail = true; break; }  // "invalid distance code"
      const uint32_t dist = C_VAL(here) + zs_wr_take(R, op & 15u);
      if (dist > total || total + len > cap) { bail = true; break; }  // too far back / capacity
      if (dist >= 64 || dist >= len) {
        // a step's sources lie at least 64 bytes back, i.e. before the step
        for (uint32_t i = 0; i < len; i += 64) {
          const uint32_t k = i + lane;
          if (k < len) {
            const uint8_t b = W.ring[(total - dist + k) & ZS_WMASK];
            W.ring[(total + k) & ZS_WMASK] = b;
            dst[total + k] = b;
          }
        }
      } else {
        // period dist < 64: lane k < step (a multiple of dist) always stores
        // the byte dist - k % dist before the copy
        const uint32_t per = 64u / dist, step = per * dist;
        const uint32_t m = lane - (lane / dist) * dist;
        const uint8_t b = W.ring[(total - dist + m) & ZS_WMASK];
        for (uint32_t i = 0; i < len; i += step) {
          const uint32_t k = i + lane;
          if (lane < step && k < len) {
            W.ring[(total + k) & ZS_WMASK] = b;
            dst[total + k] = b;
          }
        }
      }
      total += len;
    }
    if (zs_wr_over(R)) bail = true;
  }
  // ---- trailer (inflate.ts:1006-1036); the check value is verified after the checksum pass
  if (!bail && wrap) {
    zs_wr_align(R);
    const uint32_t a = zs_wr_take(R, 32);
    if (wrap & 2 && !(wrap & 1)) {
      r.want = a;
      const uint32_t isize = zs_wr_take(R, 32);
      if (isize != total) bail = true;
    } else {
      r.want = __builtin_bswap32(a);
    }
    if (zs_wr_over(R)) bail = true;
  }
  if (!bail) {
    r.bail = 0;
    r.out_len = total;
    r.consumed = (uint32_t)((zs_wr_bitpos(R) + 7u) >> 3);
  }
  if (lane == 0) {
    res[s] = r;
    lens_out[s] = r.out_len;
  }
}

size_t zs_inflate_wave_lds_bytes() { return sizeof(zs_wave_lds); }
