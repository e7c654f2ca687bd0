// deflate_fast.hip -- the greedy parser of levels 1..3 (deflate_fast,
// deflate.ts:1281-1350) on gfx950.
//
// Two kernels.  zs_k_fast_serial (below) is the first design: one wave replays
// the reference step by step.  zs_k_fast (at the end of the file, the default)
// replays it a group of 64 positions at a time from speculative per-lane chain
// walks; option fast_group = 0 selects the serial one.
//
// zs_k_fast_serial:
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
#include <type_traits>
#include "zs_common.h"
#include "zs_kernels.h"

struct zs_fast_lds {
  uint16_t head[32768];
  uint16_t prev[32768];
  uint32_t ring[8192];  // input byte x (x < 256 c) at byte (x & 32767)
};

__global__ __launch_bounds__(64) void zs_k_fast_serial(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
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

// ---------------------------------------------------------------- zs_k_fast
// The group-speculative replay (CPU model: tools/emu/emu_fast_group.c,
// tests/test_emu_fast.py).  One wave per stream keeps the reference's exact
// window-relative head[] / prev[] (u16, LDS, slid on the reference schedule)
// and works on groups of 64 consecutive positions [g0, g0 + 64), lane i
// holding position g0 + i:
//   1. every lane inserts its position speculatively -- the superset of what
//      deflate_fast inserts, which skips the inside of matches longer than
//      max_lazy (deflate.ts:1310-1322) -- through one lane-ordered
//      ds_mskor_rtn_b32 on its head[] half-word (gfx950 applies same-address
//      LDS atomics of one instruction in lane order; zs_selftest checks it):
//      each lane gets its superset chain's first link; the first lane of each
//      hash then puts the original head back;
//   2. every lane walks its superset chain (budget, MAX_DIST limit and nice
//      as longest_match, deflate.ts:1053-1115; lengths compared 4 bytes at a
//      time up to nice) and records which in-group positions it visited;
//   3. the serial parse replays the group from the lane results with scalar
//      control flow: a step's result is exact iff every in-group position its
//      walk met was truly inserted (the true chain is the superset chain minus
//      the skipped positions); the ~3 % of steps whose walk met a skipped one
//      re-walk the true chain (in-group links from ballots over the truly
//      inserted lanes), and a result at nice is extended to its exact length;
//   4. the truly inserted positions enter head[] / prev[] in lane order (one
//      more exchange).
// Steps start below g0 + 64 - max_lazy (the inside of a short match, <= max_lazy
// positions, stays inside the group) and below the position at which fill_window's next
// slide is due (deflate.ts:180-190), so a group never straddles a slide.
// The input sits in a 32 KiB LDS ring holding [E - 32768, E) with
// g0 + 160 <= E <= g0 + 262: every candidate (distance <= MAX_DIST) and every
// scan byte up to g0 + 122 + 32; 256-byte chunks are prefetched in registers
// one chunk ahead and appended 64 bytes at a time.
#define ZS_FG_LONG 0xffffu  // a lane result longer than nice + 32: extended by the serial replay

struct zs_fastg_lds {
  uint32_t head[16384];   // u16 head[h] at half (h & 1) of word h >> 1
  uint16_t prev[32768];
  uint32_t ring[8192];    // input byte x at byte (x & 32767)
};

typedef __attribute__((address_space(3))) uint32_t zs_fg_lds_u32;
static __device__ __forceinline__ uint32_t zs_fg_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const zs_fg_lds_u32*)p;
}
static __device__ __forceinline__ uint32_t zs_fg_mskor(uint32_t addr, uint32_t mask, uint32_t val) {
  uint32_t old;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(old)
               : "v"(addr), "v"(mask), "v"(val)
               : "memory");
  return old;
}

// NW: words compared per walk candidate: nice / 4 (2 / 4 / 8 at levels 1 / 2 / 3).
// ORD = false (option lane_order = 0, or a device that fails the self-test): the
// links the lane-ordered exchanges hand out come from zs_wave_match instead --
// the highest lower lane of the same hash, else head[h] -- and the last lane of
// each hash stores head[h] with a plain half-word store.
template <int NW, bool ORD>
__global__ __launch_bounds__(64) void zs_k_fast(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                const uint32_t* __restrict__ in_len,
                                                const uint64_t* __restrict__ pos_base,
                                                const uint32_t* __restrict__ blk_base, uint32_t* __restrict__ syms,
                                                zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,
                                                int chain, int lazy, int nice_cfg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t zs_fastg_smem[];
  zs_fastg_lds& L = *reinterpret_cast<zs_fastg_lds*>(zs_fastg_smem);
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  uint32_t* sy = syms + pos_base[s] + s;
  zs_block* blk = blocks + blk_base[s];
  for (uint32_t i = lane; i < 16384; i += 64) { L.head[i] = 0; reinterpret_cast<uint32_t*>(L.prev)[i] = 0; }
  const uint8_t* ringb = reinterpret_cast<const uint8_t*>(L.ring);
  auto rword = [&](uint32_t x) -> uint32_t {  // input bytes [x, x + 4) from the ring
    const uint32_t w = x >> 2;
    return __builtin_amdgcn_alignbyte(L.ring[(w + 1) & 8191u], L.ring[w & 8191u], x & 3u);
  };

  // ring fill: E = end of the ring's bytes; pf = bytes [P, P + 256) (4 per lane), nx = [P + 256, P + 512) in flight
  uint32_t E = 0, P = 0;
  uint32_t pf = zs_load_word(src, n, 4 * lane), nx = zs_load_word(src, n, 256 + 4 * lane);
  auto fill_to = [&](uint32_t want) {
    while (E < want) {
      if ((lane >> 4) == ((E - P) >> 6)) L.ring[((P >> 2) + lane) & 8191u] = pf;
      E += 64;
      if (E == P + 256) {
        P += 256;
        pf = nx;
        nx = zs_load_word(src, n, P + 256 + 4 * lane);
      }
    }
  };

  uint32_t base = 0, p = 0;
  uint32_t nsym = 0, in_blk = 0, nflush = 0, blk_start = 0;
#ifdef ZS_FG_PROF
  unsigned long long fg_acc[5] = {0, 0, 0, 0, 0}, fg_last = __builtin_readcyclecounter();
  uint32_t fg_rw = 0, fg_lg = 0;
#define FG_T(k)                                              \
  do {                                                       \
    const unsigned long long t_ = __builtin_readcyclecounter(); \
    fg_acc[k] += t_ - fg_last;                               \
    fg_last = t_;                                            \
  } while (0)
#define FG_C(v) (v)++
#else
#define FG_T(k) do {} while (0)
#define FG_C(v) do {} while (0)
#endif
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
  // exact match length at scan position a (wave-uniform) against candidate c < a, capped at maxc:
  // 64 bytes per ballot, the first 64 from the ring, further ones from memory
  auto exact_len = [&](uint32_t a, uint32_t c, uint32_t maxc) -> uint32_t {
    uint32_t k = 0;
    uint64_t neq = __ballot(ringb[(a + lane) & 32767u] != ringb[(c + lane) & 32767u] || lane >= maxc);
    while (neq == 0 && k + 64 < maxc) {
      k += 64;
      const uint32_t sb = a + k + lane < n ? src[a + k + lane] : 0x100u;
      const uint32_t mb = c + k + lane < n ? src[c + k + lane] : 0x1ffu;
      neq = __ballot(mb != sb || k + lane >= maxc);
    }
    k += neq ? (uint32_t)__builtin_ctzll(neq) : 64u;
    return k < maxc ? k : maxc;
  };

  while (p < n) {
    // fill_window slide (deflate.ts:180-190), same schedule as deflate_slow
    const uint32_t m = min(n, base + 65536u);
    if (p - base >= ZS_SLIDE_AT && m - p < ZS_MIN_LOOKAHEAD) {
      for (uint32_t i = lane; i < 16384; i += 64) {
        const uint32_t a = L.head[i];
        const uint32_t b = reinterpret_cast<uint32_t*>(L.prev)[i];
        const uint32_t a0 = a & 0xffffu, a1 = a >> 16, b0 = b & 0xffffu, b1 = b >> 16;
        L.head[i] = (a0 >= 32768u ? a0 - 32768u : 0u) | ((a1 >= 32768u ? a1 - 32768u : 0u) << 16);
        reinterpret_cast<uint32_t*>(L.prev)[i] = (b0 >= 32768u ? b0 - 32768u : 0u) |
                                                 ((b1 >= 32768u ? b1 - 32768u : 0u) << 16);
      }
      base += 32768u;
      continue;  // re-evaluate the group bounds against the new base
    }
    FG_T(0);
    const uint32_t g0 = p, rg0 = g0 - base;
    uint32_t tslide = base + ZS_SLIDE_AT;
    if (m >= ZS_MIN_LOOKAHEAD - 1 && m - (ZS_MIN_LOOKAHEAD - 1) > tslide) tslide = m - (ZS_MIN_LOOKAHEAD - 1);
    const uint32_t g1 = min(min(g0 + 64u - (uint32_t)lazy, tslide), n);
    fill_to(g0 + 160u);

    // ---- 1. speculative insertion of every lane's position
    const uint32_t q = g0 + lane;
    const bool ok = q + 2 < n;  // INSERT_STRING needs lookahead >= MIN_MATCH (deflate.ts:1296)
    const uint32_t hw = rword(q);
    const uint32_t h = (((hw & 0xffu) << 10) ^ (((hw >> 8) & 0xffu) << 5) ^ ((hw >> 16) & 0xffu)) & ZS_HASH_MASK;
    const uint32_t ha = zs_fg_addr(&L.head[h >> 1]), sh = 16u * (h & 1u);
    const uint32_t hm = ok ? 0xffffu << sh : 0u;
    uint32_t sp;
    if (ORD) {
      sp = (zs_fg_mskor(ha, hm, ok ? (rg0 + lane) << sh : 0u) >> sh) & 0xffffu;
      const bool spin = sp != 0u && sp >= rg0;  // the link is an earlier lane of the group
      // the first lane of each hash restores the original head, which every lane then reads
      (void)zs_fg_mskor(ha, ok && !spin ? hm : 0u, ok && !spin ? sp << sh : 0u);
    } else {
      const int pl = zs_lane_below(zs_wave_match(h, ok), lane);
      sp = !ok ? 0u : pl >= 0 ? rg0 + (uint32_t)pl : (L.head[h >> 1] >> sh) & 0xffffu;
    }
    const uint32_t orig = ok ? (L.head[h >> 1] >> sh) & 0xffffu : 0u;

    FG_T(1);
    // ---- 2. superset-chain walks, lengths up to nice: nw = nice / 4 words per candidate, all
    //         loaded before the first compare (2 / 4 / 8 at levels 1 / 2 / 3)
    const uint32_t look = n - q;  // wraps for lanes past the end; they are inactive
    const uint32_t srel = q - base;
    const uint32_t maxc = min(look, (uint32_t)ZS_MAX_MATCH), nice = min(look, (uint32_t)nice_cfg);
    const uint32_t capn = min(nice, maxc);
    const uint32_t limit = srel > ZS_MAX_DIST ? srel - ZS_MAX_DIST : 0u;
    bool act = ok && q < g1 && sp != 0u && srel - sp <= ZS_MAX_DIST;
    uint32_t best = ZS_MIN_MATCH - 1, bms = 0, cur = sp;
    uint64_t vis = 0;
    uint32_t sw[NW];
    {
      uint32_t A[NW + 1];
#pragma unroll
      for (int j = 0; j <= NW; j++) A[j] = L.ring[((q >> 2) + j) & 8191u];
#pragma unroll
      for (int j = 0; j < NW; j++) sw[j] = __builtin_amdgcn_alignbyte(A[j + 1], A[j], q & 3u);
    }
    // first differing byte of the W words at scan S and candidate c, 4 W if none (all loads issued first)
    auto diff_at = [&](uint32_t c, const uint32_t* S, auto Wc) -> uint32_t {
      constexpr int W = decltype(Wc)::value;
      uint32_t A[W + 1];
#pragma unroll
      for (int j = 0; j <= W; j++) A[j] = L.ring[((c >> 2) + j) & 8191u];
      uint32_t len = 4u * W;
#pragma unroll
      for (int j = W - 1; j >= 0; j--) {
        const uint32_t x = __builtin_amdgcn_alignbyte(A[j + 1], A[j], c & 3u) ^ S[j];
        len = x ? 4u * j + ((uint32_t)__builtin_ctz(x) >> 3) : len;
      }
      return len;
    };
    using NWc = std::integral_constant<int, NW>;
    for (int t = 0; t < chain; t++) {
      if (__ballot(act) == 0) break;
      // straight-line: the link, the candidate's words and the in-group link issue together
      const bool cin = cur != 0u && cur >= rg0;
      const uint32_t pl = L.prev[cur & 0x7fffu];
      const uint32_t lsp = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((cur - rg0) & 63u) * 4u), (int)sp);
      const uint32_t len = min(diff_at(base + cur, sw, NWc{}), capn);
      vis |= act && cin ? 1ull << ((cur - rg0) & 63u) : 0ull;
      const bool better = act && len > best;
      best = better ? len : best;
      bms = better ? cur : bms;
      act = act && !(better && len >= nice);
      cur = cin ? lsp : pl;
      act = act && cur > limit;
    }
    // a result at nice: its exact length from 32 more bytes per lane; ZS_FG_LONG if they all match too
    if (best >= nice && best >= ZS_MIN_MATCH && nice < maxc) {
      const uint32_t o = 4u * NW;
      uint32_t S2[8], A2[9];
#pragma unroll
      for (int j = 0; j < 9; j++) A2[j] = L.ring[(((q + o) >> 2) + j) & 8191u];
#pragma unroll
      for (int j = 0; j < 8; j++) S2[j] = __builtin_amdgcn_alignbyte(A2[j + 1], A2[j], (q + o) & 3u);
      const uint32_t e = o + diff_at(base + bms + o, S2, std::integral_constant<int, 8>{});
      best = e >= maxc ? maxc : (e < o + 32u ? e : ZS_FG_LONG);
    }

    FG_T(2);
    // ---- 3. replay of the group.  Each lane's step is precomputed: its symbol, the lane after
    //         it, and what it inserts (its own position, the inside of a short match).  Pointer
    //         doubling gives every lane's chain of next-lane links to the group's end; then, in parallel, the path's
    //         insertions give each step's truly inserted set (a step only sees positions below
    //         it, all decided by earlier steps), and the first step whose walk met a position the
    //         path skipped -- or whose match needs more than nice + 32 bytes compared -- is found
    //         by one ballot.  The steps before it are exact and stored in one go (rank = earlier
    //         steps); it runs the slow path, and the chase resumes after it.
    const bool isM = best >= ZS_MIN_MATCH;
    const uint32_t sym = isM ? 0x80000000u | ((best - ZS_MIN_MATCH) << 16) | (srel - bms) : (hw & 0xffu);
    const uint32_t shortc = isM && best != ZS_FG_LONG && best <= (uint32_t)lazy && n - (q + best) >= ZS_MIN_MATCH
                                ? best - 1u : 0u;
    const uint32_t pk = min(lane + (isM ? best : 1u), 511u) | (ok ? 512u : 0u) | (shortc << 10) |
                        (best == ZS_FG_LONG ? 0x4000u : 0u);
    const uint32_t vlo = (uint32_t)vis, vhi = (uint32_t)(vis >> 32);
    const uint64_t okm = __ballot(ok);
    uint64_t tm = 0;  // truly inserted lanes
    const uint32_t j1 = g1 - g0;
    const uint32_t nextv = pk & 511u, shc = (pk >> 10) & 15u;
    auto put = [&](uint32_t v) {  // one symbol of a slow step
      if (lane == 0) sy[nsym] = v;
      nsym++;
      in_blk++;
    };
    auto flush = [&](uint64_t path) {  // store the path's symbols in order; close a block on its 16383rd
      const uint32_t cnt = (uint32_t)__builtin_popcountll(path);
      if (cnt == 0) return;
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(path >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)path, 0u));
      if ((path >> lane) & 1ull) sy[nsym + rk] = sym;
      if (in_blk + cnt >= ZS_SYM_END) {
        const uint32_t k = ZS_SYM_END - in_blk;  // symbols up to and including the cut
        uint64_t m = path;
        for (uint32_t t = 1; t < k; t++) m &= m - 1;
        const uint32_t c = (uint32_t)__builtin_ctzll(m);
        nsym += k;
        in_blk += k;
        close_block(g0 + (uint32_t)__builtin_amdgcn_readlane((int)nextv, (int)c), 0);
        nsym += cnt - k;
        in_blk += cnt - k;
      } else {
        nsym += cnt;
        in_blk += cnt;
      }
    };
    // every lane's path to the group's end (the lanes its step chain visits), by pointer doubling:
    // S(l) = {l, nx(l), nx(nx(l)), ...} with nx absorbing at the end; six ds_bpermute levels instead of a
    // chain of dependent readlanes, and a restart after a slow step is one more lookup
    uint32_t slo, shi;
    {
      uint64_t S = 1ull << lane;
      uint32_t J = nextv < j1 ? nextv : lane;
#pragma unroll
      for (int k = 0; k < 6; k++) {
        const int a = (int)(J * 4u);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)S);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(S >> 32));
        J = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)J);
        S |= ((uint64_t)hi << 32) | lo;
      }
      slo = (uint32_t)S;
      shi = (uint32_t)(S >> 32);
    }
    uint32_t j = p - g0;
    while (j < j1) {
      // the steps from lane j to the group's end, if every lane result on the way holds
      const uint64_t path = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)shi, (int)j) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)slo, (int)j);
      const uint32_t jj = (uint32_t)__builtin_amdgcn_readlane((int)nextv, (int)(63u - (uint32_t)__builtin_clzll(path)));
      // in parallel: what the path inserts (its own positions, the inside of its short matches),
      // then the first step whose walk met a position the path skips (or that needs the slow extension)
      const bool onp = (path >> lane) & 1ull;
      const uint64_t le = path & (lane == 63u ? ~0ull : (2ull << lane) - 1ull);
      const uint32_t owner = le ? 63u - (uint32_t)__builtin_clzll(le) : 0u;
      const uint32_t osc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(owner * 4u), (int)shc);
      const bool inside = !onp && le != 0 && lane - owner <= osc;
      const uint64_t tmn = tm | __ballot((onp && ok) || inside);
      const uint64_t bad = __ballot(onp && ((best == ZS_FG_LONG) || (vis & ~tmn) != 0));
      if (bad == 0) {
        flush(path);
        tm = tmn;
        j = jj;
        break;
      }
      const uint32_t f = (uint32_t)__builtin_ctzll(bad);
      const uint64_t below = (1ull << f) - 1ull;
      flush(path & below);
      tm = tmn & below;
      // slow step at lane f
      const uint32_t i = f;
      p = g0 + i;
      const uint32_t lk = n - p, sr = p - base;
      tm |= okm & (1ull << i);
      const uint64_t vi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)vhi, (int)i) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)vlo, (int)i);
      uint32_t ml = 0, ms = 0;
      const uint32_t mx = min(lk, (uint32_t)ZS_MAX_MATCH), nc = min(lk, (uint32_t)nice_cfg);
      if ((vi & ~tm) == 0) {
        FG_C(fg_lg);
        ms = (uint32_t)__builtin_amdgcn_readlane((int)bms, (int)i);
        ml = exact_len(p, base + ms, mx);
      } else {
        // re-walk the true chain: in-group links through the truly inserted lanes of the same hash
        FG_C(fg_rw);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)h, (int)i);
        auto true_link = [&](uint32_t l, uint32_t hl) -> uint32_t {
          const uint64_t c = __ballot(h == hl) & tm & ((1ull << l) - 1ull);
          return c ? rg0 + 63u - (uint32_t)__builtin_clzll(c) : (uint32_t)__builtin_amdgcn_readlane((int)orig, (int)l);
        };
        const uint32_t hh = true_link(i, hi);
        if (hh != 0u && sr - hh <= ZS_MAX_DIST) {
          const uint32_t lim = sr > ZS_MAX_DIST ? sr - ZS_MAX_DIST : 0u;
          uint32_t cl = (uint32_t)chain, b2 = ZS_MIN_MATCH - 1, c = hh;
          do {
            const uint32_t len = exact_len(p, base + c, mx);
            if (len > b2) {
              ms = c;
              b2 = len;
              if (len >= nc) break;
            }
            if (c != 0u && c >= rg0) {
              const uint32_t l = c - rg0;
              c = true_link(l, (uint32_t)__builtin_amdgcn_readlane((int)h, (int)l));
            } else {
              c = L.prev[c & 0x7fffu];
            }
          } while (c > lim && --cl != 0);
          ml = b2 >= ZS_MIN_MATCH ? b2 : 0u;
        }
      }
      if (ml >= ZS_MIN_MATCH) {
        put(0x80000000u | ((ml - ZS_MIN_MATCH) << 16) | (sr - ms));
        const uint32_t after = p + ml;
        if (ml <= (uint32_t)lazy && n - after >= ZS_MIN_MATCH)  // insert inside short matches
          tm |= ((1ull << (after - g0)) - 1ull) & ~((2ull << i) - 1ull);
        j = after - g0;
      } else {
        put((uint32_t)__builtin_amdgcn_readlane((int)hw, (int)i) & 0xffu);
        j = i + 1;
      }
      if (in_blk == ZS_SYM_END) close_block(g0 + j, 0);
    }
    p = g0 + j;

    FG_T(3);
    // ---- 4. the truly inserted positions enter head[] / prev[] in lane order
    const bool ins = (tm >> lane) & 1ull;
    uint32_t tp;
    if (ORD) {
      tp = (zs_fg_mskor(ha, ins ? hm : 0u, ins ? (rg0 + lane) << sh : 0u) >> sh) & 0xffffu;
    } else {
      const uint64_t im = zs_wave_match(h, ins);
      const int pl = zs_lane_below(im, lane);
      tp = pl >= 0 ? rg0 + (uint32_t)pl : (L.head[h >> 1] >> sh) & 0xffffu;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      if (ins && (im >> lane) == 1ull) reinterpret_cast<uint16_t*>(L.head)[h] = (uint16_t)(rg0 + lane);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
    if (ins) L.prev[(rg0 + lane) & 0x7fffu] = (uint16_t)tp;
    FG_T(4);
  }
#ifdef ZS_FG_PROF
  if (lane == 0 && s < 4)
    printf("fgprof s=%d n=%u t1=%llu t2=%llu t3=%llu t4=%llu t0=%llu rw=%u lg=%u\n", s, n, fg_acc[1], fg_acc[2], fg_acc[3],
           fg_acc[4], fg_acc[0], fg_rw, fg_lg);
#endif
  close_block(n, 1);
  if (lane == 0) {
    streams[s].nsym = nsym;
    streams[s].nblk = nflush;
  }
}

template __global__ void zs_k_fast<2, true>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, const uint32_t*,
                                      uint32_t*, zs_block*, zs_stream*, int, int, int);
template __global__ void zs_k_fast<4, true>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, const uint32_t*,
                                      uint32_t*, zs_block*, zs_stream*, int, int, int);
template __global__ void zs_k_fast<8, true>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, const uint32_t*,
                                      uint32_t*, zs_block*, zs_stream*, int, int, int);
template __global__ void zs_k_fast<2, false>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, const uint32_t*,
                                      uint32_t*, zs_block*, zs_stream*, int, int, int);
template __global__ void zs_k_fast<4, false>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, const uint32_t*,
                                      uint32_t*, zs_block*, zs_stream*, int, int, int);
template __global__ void zs_k_fast<8, false>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, const uint32_t*,
                                      uint32_t*, zs_block*, zs_stream*, int, int, int);
