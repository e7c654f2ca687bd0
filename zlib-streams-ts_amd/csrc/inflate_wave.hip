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
#include "zs_wave.h"

// history ring: the window (32 KiB; deflate64 64 KiB), at the start of the
// dynamic LDS; then the staged input and zlib's tables.  Deflate: 40,792 B, four
// workgroups per CU; deflate64: 73,560 B, two.
struct zs_wave_tabs {
  uint32_t inw[ZS_WIN_IN];
  zcode codes[ENOUGH_LENS + ENOUGH_DISTS_9];
  uint16_t lens[320];
  uint16_t work[288];
};
static __host__ __device__ inline uint32_t zs_wave_ring_bytes(bool d64) { return d64 ? 65536u : 32768u; }

// REFW: a deflate / zlib / gzip member with the reference's window-wrap copy
// reproduced (flags & ZS_INF_REF_WRAP); the other instance (deflate64, or
// inflate_ref_wrap = 0) carries no call bookkeeping.
// one member s, by the whole wave
template <bool REFW>
static __device__ __forceinline__ void zs_wave_member(uint8_t* zs_wsm, const uint8_t* __restrict__ in,
                                                      const uint64_t* __restrict__ in_off,
                                                      const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                      const uint64_t* __restrict__ out_off,
                                                      const uint32_t* __restrict__ out_cap, int wbits,
                                                      zs_lane_res* __restrict__ res, uint32_t* __restrict__ lens_out,
                                                      const uint32_t s) {
  const bool d64 = wbits == -16;
  uint8_t* ring = zs_wsm;
  const uint32_t rmask = zs_wave_ring_bytes(d64) - 1u;
  zs_wave_tabs& W = *reinterpret_cast<zs_wave_tabs*>(zs_wsm + zs_wave_ring_bytes(d64));
  const uint32_t lane = threadIdx.x;
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
  uint32_t* dstw = reinterpret_cast<uint32_t*>(dst);  // out_off is 4-aligned
  const uint32_t* ringw = reinterpret_cast<const uint32_t*>(ring);
  const uint32_t cap = zs_u(out_cap[s]);
  const uint32_t lmask = d64 ? 31u : 15u;  // length extra-bit mask (inflate.ts:891)
  const int wrap = wbits < 0 ? 0 : (wbits >> 4) + 5;  // inflate.ts:152-160
  // the reference's call boundaries matter for deflate / zlib / gzip (deflate64 never runs inflate_fast)
  constexpr bool refw = REFW;
  zs_refcalls C;
  C.init();
  uint32_t total = 0, flushed = 0;
  zs_lane_res r = {1u, 0u, 0u, 0u};
  bool bail = false;
  // output leaves the ring 256 bytes (one dword per lane) at a time
  auto flush = [&]() {
    while (total - flushed >= 256u) {
      dstw[(flushed >> 2) + lane] = ringw[((flushed & rmask) >> 2) + lane];
      flushed += 256u;
    }
  };
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
      if (refw) C.stored(at, total, len);
      for (uint32_t i = 0; i < len; i += 64) {
        const uint32_t k = i + lane;
        if (k < len) ring[(total + lane) & rmask] = src[at + k];
        total += min(64u, len - i);
        flush();
      }
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
    // symbols (inffast.ts:5-228 semantics; the reference's call boundaries tracked by C)
    for (;;) {
      const uint64_t b0 = zs_wr_bitpos(R);
      zcode here = zs_wr_decode(R, lt, lbits);
      uint32_t op = C_OP(here);
      if (op == 0) {
        if (total >= cap) { bail = true; break; }
        if (refw) C.symbol(b0, total, 1u, (uint32_t)(zs_wr_bitpos(R) - b0), 0u, 0u, 0u, false);
        if (lane == 0) ring[total & rmask] = (uint8_t)C_VAL(here);
        total++;
        flush();
        continue;
      }
      if (op & 32) {  // end of block
        if (refw) C.symbol(b0, total, 0u, (uint32_t)(zs_wr_bitpos(R) - b0), 0u, 0u, 0u, true);
        break;
      }
      if (op & 64) { bail = true; break; }  // "invalid literal/length code"
      const uint64_t b1 = zs_wr_bitpos(R);
      const uint32_t len = C_VAL(here) + zs_wr_take(R, op & lmask);
      const uint64_t b2 = zs_wr_bitpos(R);
      here = zs_wr_decode(R, dt, dbits);
      op = C_OP(here);
      if (op & 64) { bail = true; break; }  // "invalid distance code"
      const uint64_t b3 = zs_wr_bitpos(R);
      const uint32_t dist = C_VAL(here) + zs_wr_take(R, op & 15u);
      if (dist > total || total + len > cap) { bail = true; break; }  // too far back / capacity
      uint32_t tail = 0;  // bytes the reference takes from its call's first output bytes
      if (refw && C.symbol(b0, total, len, (uint32_t)(b1 - b0), (uint32_t)(b2 - b1), (uint32_t)(b3 - b2),
                           (uint32_t)(zs_wr_bitpos(R) - b3), false))
        tail = C.wrap(total, len, dist);
      // A deflate64 copy can be longer than the ring (length code 285: up to
      // 65,538 bytes): it goes in pieces of at most half the ring, the complete
      // words stored after each, so no piece overwrites bytes not yet in HBM
      // (the sources stay right: the ring holds the latest 64 KiB, dist <= 64 KiB).
      for (uint32_t left = len - tail; left;) {
        const uint32_t pn = min(left, 32768u);
        if (dist >= 64 || dist >= pn) {
          // a step's sources lie at least 64 bytes back, i.e. before the step
          for (uint32_t i = 0; i < pn; i += 64) {
            const uint32_t k = i + lane;
            if (k < pn) ring[(total + k) & rmask] = ring[(total - dist + k) & rmask];
          }
        } else {
          // period dist < 64: lane k < step (a multiple of dist) always stores
          // the byte dist - k % dist before the copy
          const uint32_t per = 64u / dist, step = per * dist;
          const uint32_t m = lane - (lane / dist) * dist;
          const uint8_t b = ring[(total - dist + m) & rmask];
          for (uint32_t i = 0; i < pn; i += step) {
            const uint32_t k = i + lane;
            if (lane < step && k < pn) ring[(total + k) & rmask] = b;
          }
        }
        total += pn;
        left -= pn;
        flush();
      }
      if (tail) {
        // the window-wrap copy: output[0..tail) of the current call, one byte
        // at a time (it may overlap the bytes it writes); bytes older than the
        // ring are in HBM already (flushed <= 256 bytes behind)
        if (lane == 0) {
          for (uint32_t i = 0; i < tail; i++) {
            const uint32_t x = C.B + i, t = total + i;
            ring[t & rmask] = x + rmask + 1u >= t + 1u ? ring[x & rmask] : dst[x];
          }
        }
        total += tail;
        flush();
      }
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
    // the last bytes: whole words (the last one's bytes past total are inside the capacity)
    const uint32_t wend = (total + 3u) >> 2;
    for (uint32_t w = (flushed >> 2) + lane; w < wend; w += 64) dstw[w] = ringw[(w & (rmask >> 2))];
    r.bail = 0;
    r.out_len = total;
    r.consumed = (uint32_t)((zs_wr_bitpos(R) + 7u) >> 3);
  }
  if (lane == 0) {
    res[s] = r;
    lens_out[s] = r.out_len;
  }
}

size_t zs_inflate_wave_lds_bytes(bool d64) { return zs_wave_ring_bytes(d64) + sizeof(zs_wave_tabs); }

// list[0 .. n_list): the members.  skip_done: list is the segmented decode's
// leftovers (inflate_seg.hip), n_dev their count: a grid of fixed size walks it,
// so the usual case -- none -- costs no dispatch of one workgroup per member.
template <bool REFW>
__global__ __launch_bounds__(64) void zs_k_inflate_wave(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint32_t* __restrict__ out_cap, int wbits,
                                                        const uint32_t* __restrict__ list, uint32_t n_list,
                                                        zs_lane_res* __restrict__ res, uint32_t* __restrict__ lens_out,
                                                        const uint32_t* __restrict__ n_dev) {
  extern __shared__ __attribute__((aligned(16))) uint8_t zs_wsm[];
  const uint32_t nl = n_dev ? min(n_list, zs_u(*n_dev)) : n_list;
  for (uint32_t k = blockIdx.x; k < nl; k += gridDim.x) {
    __syncthreads();  // (the LDS of the member before is free)
    zs_wave_member<REFW>(zs_wsm, in, in_off, in_len, out, out_off, out_cap, wbits, res, lens_out, zs_u(list[k]));
  }
}

template __global__ void zs_k_inflate_wave<false>(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                                  const uint64_t*, const uint32_t*, int, const uint32_t*, uint32_t,
                                                  zs_lane_res*, uint32_t*, const uint32_t*);
template __global__ void zs_k_inflate_wave<true>(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                                 const uint64_t*, const uint32_t*, int, const uint32_t*, uint32_t,
                                                 zs_lane_res*, uint32_t*, const uint32_t*);
