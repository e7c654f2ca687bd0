// deflate_fast.hip -- the greedy parser of levels 1..3 (deflate_fast,
// deflate.ts:1281-1350) on gfx950.
//
// Unlike levels 4..9, deflate_fast does not insert the positions inside a
// match longer than max_lazy (deflate.ts:1310-1322), so its hash chains depend
// on the parse and cannot be precomputed per position.  One
// workgroup (one wave) per stream therefore replays the reference serially,
// with the exact window-relative head[] / prev[] tables of the reference
// (u16, 32 K entries each, slid by 32 K on the same schedule as fill_window,
// deflate.ts:180-190) resident in LDS.  All 64 lanes run the state machine in
// lock-step and cooperate on the byte work: a candidate is compared 64 bytes
// per step (ballot).  The bytes come from LDS and registers, not from memory:
// a 32 KiB ring in LDS holds the input before the current 256-byte chunk
// (everything a candidate at distance <= MAX_DIST can start at), and two
// registers per lane hold the current and next chunk (the scan bytes, the hash
// bytes, the literals), the next-but-one chunk's load in flight as the parse
// enters a chunk.  head + prev + ring fill the CU's 160 KiB of LDS.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"

struct zs_fast_lds {
  uint16_t head[32768];
  uint16_t prev[32768];
  uint32_t ring[8192];  // input byte x (x < 256 c) at byte (x & 32767)
};

__global__ __launch_bounds__(64) void zs_k_fast(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                const uint32_t* __restrict__ in_len,
                                                const uint64_t* __restrict__ pos_base,
                                                const uint32_t* __restrict__ blk_base, uint32_t* __restrict__ syms,
                                                zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,
                                                int chain, int lazy, int nice_cfg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t zs_fast_smem[];
  zs_fast_lds& L = *reinterpret_cast<zs_fast_lds*>(zs_fast_smem);
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  uint32_t* sy = syms + pos_base[s] + s;
  zs_block* blk = blocks + blk_base[s];
  for (uint32_t i = lane; i < 32768; i += 64) { L.head[i] = 0; L.prev[i] = 0; }  // CLEAR_HASH (deflate.ts:120-123)
  __syncthreads();

  // chunk window: r0 = input bytes [256 c + 4 lane, +4), r1 = the next chunk's
  uint32_t c = 0;
  uint32_t r0 = zs_load_word(src, n, 4 * lane), r1 = zs_load_word(src, n, 256 + 4 * lane);
  uint8_t* const ringb = reinterpret_cast<uint8_t*>(L.ring);
  auto advance_to = [&](uint32_t q) {  // make the window's first chunk the one holding q
    while (q >= 256u * (c + 1)) {
      L.ring[((256u * c) & 32767u) / 4 + lane] = r0;  // chunk c leaves the registers for the ring
      r0 = r1;
      r1 = zs_load_word(src, n, 256u * (c + 2) + 4 * lane);
      c++;
    }
  };
  // byte q (wave-uniform, q in [256 c, 256 c + 512)) of the window
  auto win_byte = [&](uint32_t q) -> uint32_t {
    const uint32_t o = q - 256u * c;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)(o < 256u ? r0 : r1), (int)((o >> 2) & 63u));
    return (w >> (8 * (o & 3))) & 0xffu;
  };
  // byte y of the input for this lane (y in [256 c - 32768, 256 c + 512)): the
  // ring below the window, the window's registers (cross-lane) above.  Every
  // lane must execute it (ds_bpermute reads the registers of other lanes).
  auto lane_byte = [&](uint32_t y) -> uint32_t {
    const uint32_t o = y - 256u * c;  // wraps for y below the window
    const int from = (int)(((o >> 2) & 63u) * 4u);
    const uint32_t w0 = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)r0);
    const uint32_t w1 = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)r1);
    const uint32_t rb = ringb[y & 32767u];
    const uint32_t wb = ((o & 256u) ? w1 : w0) >> (8 * (o & 3));
    return y < 256u * c ? rb : wb & 0xffu;
  };
  // SURVEY A1 (caller guarantees q + 2 < n, q < 256 c + 510); rolled one byte
  // at a time over consecutive positions as UPDATE_HASH does (deflate.ts:109-111)
  uint32_t hq = 0xfffffff0u, hv = 0;  // hq + 1 never equals a position
  auto hash_at = [&](uint32_t q) -> uint32_t {
    hv = q == hq + 1 ? ((hv << 5) ^ win_byte(q + 2)) & ZS_HASH_MASK
                     : ((win_byte(q) << 10) ^ (win_byte(q + 1) << 5) ^ win_byte(q + 2)) & ZS_HASH_MASK;
    hq = q;
    return hv;
  };

  uint32_t base = 0;  // absolute position of window index 0
  uint32_t nsym = 0, in_blk = 0, nflush = 0, blk_start = 0;
  uint32_t ml = 0, ms_rel = 0;  // match_length / match_start (window-relative)
  uint32_t p = 0;
  auto insert = [&](uint32_t q) -> uint32_t {  // INSERT_STRING (deflate.ts:113-118), window-relative
    const uint32_t h = hash_at(q);
    const uint32_t rel = q - base;
    const uint32_t hh = L.head[h];
    // lane 0 writes; the wave's later LDS reads are ordered behind these writes
    if (lane == 0) { L.prev[rel & 0x7fffu] = (uint16_t)hh; L.head[h] = (uint16_t)rel; }
    return hh;
  };
  // Symbols are held one per lane (lane nsym % 64) and stored 64 at a time: a
  // store per symbol would make every following load wait for it (on gfx9
  // stores share vmcnt with loads).
  uint32_t sbuf = 0;
  auto drain = [&]() {
    const uint32_t k = nsym & 63u;
    if (lane < k) sy[nsym - k + lane] = sbuf;
  };
  auto emit = [&](uint32_t v) {
    sbuf = lane == (nsym & 63u) ? v : sbuf;
    nsym++;
    in_blk++;
    if ((nsym & 63u) == 0) sy[nsym - 64 + lane] = sbuf;
  };
  auto close_block = [&](uint32_t end, uint32_t last) {
    if (lane == 0) {
      zs_block b;
      b.sym_start = nsym - in_blk;
      b.sym_count = in_blk;
      b.in_start = blk_start;
      b.in_end = end;
      b.type = 0; b.hdr_bits = 0; b.data_bits = 0; b.pad = 0; b.bit_off = 0; b.bit_end = 0;
      b.last = last | (blk_start < base ? 2u : 0u);
      blk[nflush] = b;
    }
    nflush++;
    in_blk = 0;
    blk_start = end;
  };

  while (p < n) {
    advance_to(p);
    // fill_window slide (deflate.ts:180-190): same schedule as deflate_slow
    if (p - base >= ZS_SLIDE_AT && min(n, base + 65536u) - p < ZS_MIN_LOOKAHEAD) {
      for (uint32_t i = lane; i < 32768; i += 64) {
        const uint32_t a = L.head[i], b = L.prev[i];
        L.head[i] = (uint16_t)(a >= 32768u ? a - 32768u : 0u);
        L.prev[i] = (uint16_t)(b >= 32768u ? b - 32768u : 0u);
      }
      __syncthreads();
      base += 32768u;
      ms_rel -= 32768u;
    }
    const uint32_t look = n - p;
    uint32_t hash_head = 0;
    if (look >= ZS_MIN_MATCH) hash_head = insert(p);
    const uint32_t srel = p - base;
    if (hash_head != 0 && srel - hash_head <= ZS_MAX_DIST) {
      // longest_match with prev_length = MIN_MATCH - 1 (deflate_fast never sets it), deflate.ts:1053-1115
      uint32_t chain_length = (uint32_t)chain;
      const uint32_t maxc = look < ZS_MAX_MATCH ? look : ZS_MAX_MATCH;
      const uint32_t nice = look < (uint32_t)nice_cfg ? look : (uint32_t)nice_cfg;
      const uint32_t limit = srel > ZS_MAX_DIST ? srel - ZS_MAX_DIST : 0;
      uint32_t best = ZS_MIN_MATCH - 1, cur = hash_head;
      // lane_byte reads other lanes' registers: every lane runs it, then masks
      const uint32_t sbv = lane_byte(p + lane);
      const uint32_t sb = p + lane < n ? sbv : 0x100u;  // scan bytes 0..63
      do {
        const uint32_t mpos = base + cur;
        uint32_t k = 0;
        // compare 64 bytes per step (the first 64 from LDS / registers, any further ones from memory)
        const uint32_t mbv = lane_byte(mpos + lane);
        uint32_t mb = mpos + lane < n ? mbv : 0x1ffu;
        uint64_t neq = __ballot(mb != sb || lane >= maxc);
        while (neq == 0 && k + 64 < maxc) {
          k += 64;
          const uint32_t sbk = p + k + lane < n ? src[p + k + lane] : 0x100u;
          mb = mpos + k + lane < n ? src[mpos + k + lane] : 0x1ffu;
          neq = __ballot(mb != sbk || k + lane >= maxc);
        }
        k += neq ? (uint32_t)__builtin_ctzll(neq) : 64u;
        const uint32_t len = k < maxc ? k : maxc;
        if (len > best) {
          ms_rel = cur;
          best = len;
          if (len >= nice) break;
        }
        cur = L.prev[cur & 0x7fffu];
      } while (cur > limit && --chain_length != 0);
      ml = best <= look ? best : look;
    }
    if (ml >= ZS_MIN_MATCH) {
      emit(0x80000000u | ((ml - ZS_MIN_MATCH) << 16) | (srel - ms_rel));
      const uint32_t after = p + ml;
      if (ml <= (uint32_t)lazy && n - after >= ZS_MIN_MATCH) {
        for (uint32_t q = p + 1; q < after; q++) insert(q);  // insert inside short matches
      }
      p = after;
      ml = 0;
    } else {
      emit(win_byte(p));
      p++;
    }
    if (in_blk == ZS_SYM_END) close_block(p, 0);
  }
  close_block(n, 1);
  drain();
  if (lane == 0) {
    streams[s].nsym = nsym;
    streams[s].nblk = nflush;
  }
}
