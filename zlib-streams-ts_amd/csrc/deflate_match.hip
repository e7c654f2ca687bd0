// deflate_match.hip -- LZ77 match finding for deflate levels 4..9 on gfx950.
//
// The reference finds matches serially: deflate_slow (deflate.ts:1352-1448)
// inserts every position into a 15-bit hash chain (INSERT_STRING,
// deflate.ts:113-118) and calls longest_match (deflate.ts:1053-1115) at the
// positions its lazy parse visits.  At levels 4..9 every position <= n-3 is
// inserted exactly once and in order (verified call-by-call in
// F11), so the chains -- and the result of longest_match at a position for a
// given chain budget -- are a pure function of the input bytes.  This file
// computes them for EVERY position in parallel:
//
//   zs_k_prev  : prevd[p] = distance to the previous position with the same
//                hash (0 = none / farther than 32767), i.e. the reference's
//                prev[] chain in absolute coordinates.  One wave per stream,
//                one lane-ordered LDS exchange per position.
//
//   zs_k_match : per position, the (length, distance) longest_match returns
//                for the full chain budget and for the budget >> 2 used when
//                prev_length >= good_match (deflate.ts:1075-1077).  One
//                workgroup per 8 KiB tile; the tile's 32 KiB look-back window
//                and its chain links are staged in LDS, each lane walks the
//                chain of one position with 4-byte compares.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"

// ---------------------------------------------------------------- zs_k_prev
// One wave per stream walks the positions in order, 64 at a time.  Lane l of
// a 64-position group swaps its position into head[h] with ONE ds_wrxchg_rtn:
// gfx950 applies same-address LDS atomics of one wave instruction in increasing
// lane order (probed: tools/probes/lds_atomic_order.hip, re-checked at run time
// by zs_selftest), so the value each lane gets back is exactly the previous
// position with the same hash -- the reference's prev[] link.  head[] holds
// q + 1 (absolute, 32-bit), so no slide (deflate.ts:125-141) is needed.
// ORD = false (option lane_order = 0, or a device that fails the self-test):
// each lane's link is the highest lower lane of the group with the same hash
// (zs_wave_match) or head[h], and the group's last lane of each hash stores it.
#define ZS_PREV_STAGE 4096u
template <bool ORD>
__global__ __launch_bounds__(64) void zs_k_prev(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                const uint32_t* __restrict__ in_len,
                                                const uint64_t* __restrict__ pos_base, uint16_t* __restrict__ prevd,
                                                uint32_t min_len) {
  __shared__ uint32_t head[32768];
  __shared__ uint32_t stg[ZS_PREV_STAGE / 4 + 2];  // input bytes [c0, c0 + 4096 + 8)
  const int s = blockIdx.x;
  const uint32_t n = in_len[s];
  if (n <= min_len) return;  // a stream zs_k_bucket + zs_k_sweep handle (min_len 65537; 0 = every stream)
  const uint8_t* src = in + in_off[s];
  uint16_t* out = prevd + pos_base[s];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < 32768; i += 64) head[i] = 0;
  const bool aligned = ((uintptr_t)src & 3u) == 0;
  for (uint32_t c0 = 0; c0 < n; c0 += ZS_PREV_STAGE) {
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = lane; i < ZS_PREV_STAGE / 4 + 2; i += 64) {
      const uint32_t at = c0 + 4 * i;
      uint32_t v = 0;
      if (aligned && at + 4 <= n) {
        v = *(const uint32_t*)(src + at);
      } else {
        for (uint32_t k = 0; k < 4; k++)
          if (at + k < n) v |= (uint32_t)src[at + k] << (8 * k);
      }
      stg[i] = v;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const uint32_t c1 = min(n, c0 + ZS_PREV_STAGE);
    for (uint32_t g0 = c0; g0 < c1; g0 += 256) {
      uint32_t h[4], e[4];
      bool valid[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t p = g0 + 64 * j + lane;
        const uint32_t o = p - c0;
        const uint32_t w = __builtin_amdgcn_alignbyte(stg[(o >> 2) + 1], stg[o >> 2], o & 3u);
        valid[j] = p + 2 < n && p < c1;  // positions <= n-3 are inserted (deflate.ts:1367-1370)
        h[j] = (((w & 0xffu) << 10) ^ (((w >> 8) & 0xffu) << 5) ^ ((w >> 16) & 0xffu)) & ZS_HASH_MASK;
      }
      // in order: group j's exchanges land after group j-1's (LDS executes a wave's ops in order)
      if (ORD) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t p = g0 + 64 * j + lane;
          e[j] = valid[j] ? atomicExch(&head[h[j]], p + 1) : 0u;
        }
      } else {
        for (int j = 0; j < 4; j++) {
          const uint32_t p = g0 + 64 * j + lane;
          const uint64_t mm = zs_wave_match(h[j], valid[j]);
          const int pl = zs_lane_below(mm, lane);
          e[j] = !valid[j] ? 0u : pl >= 0 ? g0 + 64 * j + (uint32_t)pl + 1u : head[h[j]];
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
          if (valid[j] && (mm >> lane) == 1ull) head[h[j]] = p + 1;  // the last lane of its hash
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
        }
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t p = g0 + 64 * j + lane;
        if (p < c1) {
          const uint32_t d = e[j] ? p - (e[j] - 1) : 0u;
          out[p] = (uint16_t)(valid[j] && d != 0u && d <= 32767u ? d : 0xffffu);
        }
      }
    }
  }
}

template __global__ void zs_k_prev<true>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, uint16_t*,
                                         uint32_t);
template __global__ void zs_k_prev<false>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, uint16_t*,
                                          uint32_t);

// --------------------------------------------------------------- zs_k_match
#define ZS_TILE 8192u
#define ZS_LOOKBACK 32768u
#define ZS_WIN_BYTES (ZS_LOOKBACK + ZS_TILE + 272u)  // + MAX_MATCH + slack for 4-byte reads
#define ZS_WIN_WORDS (ZS_WIN_BYTES / 4)
#define ZS_M_PV ((ZS_WIN_WORDS + 2 + 3) & ~3u)                 // word offsets in zs_k_match's LDS
#define ZS_M_ORDER (ZS_M_PV + (ZS_LOOKBACK + ZS_TILE) / 2)
#define ZS_M_BINS (ZS_M_ORDER + ZS_TILE / 2)
#define ZS_M_WORDS (ZS_M_BINS + 256 + 4)
static_assert(4 * ZS_M_PV < 65536, "link base must fit a DS offset");

static __device__ __forceinline__ uint32_t win_word(const uint32_t* wb, uint32_t off) {
  const uint32_t i = off >> 2;
  return __builtin_amdgcn_alignbyte(wb[i + 1], wb[i], off & 3u);
}

__global__ __launch_bounds__(1024) void zs_k_match(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len,
                                                   const uint64_t* __restrict__ pos_base,
                                                   const uint16_t* __restrict__ prevd, uint2* __restrict__ mres,
                                                   int chain, int nice_cfg, uint32_t min_len) {
  // One LDS array, carved by hand so the window sits at address 0 and the
  // links at a constant below 64 KiB: the walk's LDS reads then need no base
  // add (the link base rides in the instruction's offset field).
  //   wb    window bytes [w0, w1), zero padded
  //   pv    chain links of [w0, t1); before they are staged the same LDS holds
  //         a 32768-bucket u16 histogram of the window's hashes (ordering key)
  //   order tile positions, longest expected chains first
  __shared__ __attribute__((aligned(16))) uint32_t lds[ZS_M_WORDS];
  uint32_t* const wb = lds;
  uint32_t* const pvw = lds + ZS_M_PV;
  uint16_t* const pv = (uint16_t*)pvw;
  uint16_t* const order = (uint16_t*)(lds + ZS_M_ORDER);
  uint32_t* const bins = lds + ZS_M_BINS;
  uint32_t& next = lds[ZS_M_BINS + 256];  // work queue over order[]: the next unclaimed group of 64
  const int s = blockIdx.y;
  const uint32_t n = in_len[s];
  const uint32_t t0 = blockIdx.x * ZS_TILE;
  if (t0 >= n || n <= min_len) return;  // n <= min_len: zs_k_sweep's stream
  const uint32_t t1 = min(n, t0 + ZS_TILE);
  const uint32_t w0 = t0 > ZS_LOOKBACK ? t0 - ZS_LOOKBACK : 0;  // multiple of 4
  const uint32_t w1 = min(n, t1 + ZS_MAX_MATCH + 4);
  const uint8_t* src = in + in_off[s];
  const uint16_t* pd = prevd + pos_base[s];
  // Staging.  All global loads are issued up front, 16 B per load: the links
  // of [w0, t1) (pos_base and w0 are multiples of 8, so 16-B aligned) go to
  // registers and are written to LDS only after the ordering phase below, which
  // uses the same LDS; the window bytes [w0, w1) go to LDS now.  (Bytes past w1
  // are never used by a result: every compare is clamped to maxc <= n - p.)
  const uint32_t npv = t1 - w0;  // links to stage, <= ZS_LOOKBACK + ZS_TILE
  uint4 lk[(ZS_LOOKBACK + ZS_TILE) / 8 / 1024];
  {
    const uint4* src16 = (const uint4*)(pd + w0);
#pragma unroll
    for (uint32_t j = 0; j < (ZS_LOOKBACK + ZS_TILE) / 8 / 1024; j++) {
      const uint32_t i = threadIdx.x + 1024 * j;  // entries [8i, 8i + 8)
      if (8 * i + 8 <= npv) lk[j] = src16[i];
      else {
        uint32_t v[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
        for (uint32_t k = 0; k < 8; k++)
          if (8 * i + k < npv) {
            const uint32_t sh = 16 * (k & 1);
            v[k >> 1] = (v[k >> 1] & ~(0xffffu << sh)) | ((uint32_t)pd[w0 + 8 * i + k] << sh);
          }
        lk[j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  }
  const uint32_t nwords = (w1 - w0 + 3) / 4 + 2;  // window words incl. 8 B of zero slack
  if ((((uintptr_t)(src + w0)) & 15u) == 0) {
    constexpr uint32_t J = (ZS_WIN_WORDS + 2 + 4095) / 4096;
    uint4 wv[J];
#pragma unroll
    for (uint32_t j = 0; j < J; j++) {
      const uint32_t i = threadIdx.x + 1024 * j;  // bytes [w0 + 16i, w0 + 16i + 16)
      const uint32_t b = w0 + 16 * i;
      if (b + 16 <= n) wv[j] = ((const uint4*)(src + w0))[i];
      else {
        uint32_t v[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 16; k++)
          if (b + k < n) v[k >> 2] |= (uint32_t)src[b + k] << (8 * (k & 3));
        wv[j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < J; j++) {
      const uint32_t i = threadIdx.x + 1024 * j;
      if (4 * i < nwords) *(uint4*)(wb + 4 * i) = wv[j];
    }
  } else {
    for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) {
      uint32_t v = 0;
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t b = w0 + 4 * i + k;
        if (b < w1) v |= (uint32_t)src[b] << (8 * k);
      }
      wb[i] = v;
    }
  }
  // Deal positions to lanes by decreasing expected chain length (a counting
  // sort): the 64 chains a wave walks in lock-step then have similar lengths,
  // instead of every wave waiting for its longest chain.  A chain holds the
  // earlier positions with the same hash, so the key is how often the
  // position's hash occurs in the window [w0, t1) -- a u16 histogram built in
  // the LDS the links are staged into afterwards.  The key only orders the
  // work, never changes a result.
  for (uint32_t i = threadIdx.x; i < 32768 / 8; i += blockDim.x) *(uint4*)(pvw + 4 * i) = make_uint4(0, 0, 0, 0);
  if (threadIdx.x < 256) bins[threadIdx.x] = 0;
  if (threadIdx.x == 0) next = 0;
  __syncthreads();
  const uint32_t hend = min(t1, n > 2 ? n - 2 : 0u);  // positions <= n-3 are inserted (deflate.ts:1367-1370)
  // four consecutive positions per thread from two window words
  for (uint32_t i = threadIdx.x; 4 * i < hend - w0; i += blockDim.x) {
    const uint32_t lo = wb[i], hi = wb[i + 1];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, k);
      const uint32_t h = (((w & 0xffu) << 10) ^ (((w >> 8) & 0xffu) << 5) ^ ((w >> 16) & 0xffu)) & ZS_HASH_MASK;
      if (4 * i + k < hend - w0) atomicAdd(&pvw[h >> 1], 1u << (16 * (h & 1u)));
    }
  }
  __syncthreads();
  const uint32_t cap = (uint32_t)chain < 255u ? (uint32_t)chain : 255u;
  uint32_t key[ZS_TILE / 1024];
#pragma unroll
  for (uint32_t i = 0; i < ZS_TILE / 1024; i++) {
    const uint32_t p = t0 + threadIdx.x + 1024 * i;
    uint32_t c = 0;
    if (p < hend) {
      const uint32_t w = win_word(wb, p - w0);
      const uint32_t h = (((w & 0xffu) << 10) ^ (((w >> 8) & 0xffu) << 5) ^ ((w >> 16) & 0xffu)) & ZS_HASH_MASK;
      c = (pvw[h >> 1] >> (16 * (h & 1u))) & 0xffffu;
    }
    key[i] = p < t1 ? 255u - min(c, cap) : 0u;
    if (p < t1) atomicAdd(&bins[key[i]], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the 256 bins, one wave
    uint32_t v[4], t = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) { v[j] = bins[threadIdx.x * 4 + j]; t += v[j]; }
    uint32_t x = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (threadIdx.x >= (uint32_t)d) x += y;
    }
    uint32_t run = x - t;
#pragma unroll
    for (int j = 0; j < 4; j++) { bins[threadIdx.x * 4 + j] = run; run += v[j]; }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < ZS_TILE / 1024; i++) {
    const uint32_t o = threadIdx.x + 1024 * i;
    if (t0 + o < t1) order[atomicAdd(&bins[key[i]], 1u)] = (uint16_t)o;
  }
  // the links (a missing one is 0xffff: the walk's signed `cur - d <= limit`
  // test then also ends the chain, and a head distance > MAX_DIST is invalid)
#pragma unroll
  for (uint32_t j = 0; j < (ZS_LOOKBACK + ZS_TILE) / 8 / 1024; j++) {
    const uint32_t i = threadIdx.x + 1024 * j;
    if (8 * i < npv) *(uint4*)(pvw + 4 * i) = lk[j];
  }
  __syncthreads();

  const uint32_t budget = (uint32_t)chain, budget_small = (uint32_t)chain >> 2;
  uint2* out = mres + pos_base[s];
  // Waves claim groups of 64 sorted positions from a queue, longest chains
  // first: a wave that drew short chains takes more groups, so the 16 waves end
  // together (a static deal leaves the CU idle while the wave holding the
  // longest chains of every round finishes).
  const uint32_t lane = threadIdx.x & 63u;
  for (;;) {
    uint32_t g = 0;
    if (lane == 0) g = atomicAdd(&next, 64u);
    g = __builtin_amdgcn_readfirstlane(g);
    if (g >= t1 - t0) break;
    const uint32_t oi = g + lane;
    if (oi >= t1 - t0) break;
    const uint32_t p = t0 + order[oi];
    uint2 r = make_uint2(0, 0);
    const uint32_t d0 = p + 2 < n ? pv[p - w0] : 0xffffu;
    const uint32_t q0 = p - d0;
    // head candidate: non-NIL, distance <= MAX_DIST (deflate.ts:1376)
    if (q0 != 0 && d0 <= ZS_MAX_DIST) {
      const uint32_t look = n - p;
      const uint32_t maxc = look < ZS_MAX_MATCH ? look : ZS_MAX_MATCH;       // deflate.ts:1068
      const uint32_t nice = look < (uint32_t)nice_cfg ? look : (uint32_t)nice_cfg;  // deflate.ts:1078-1080
      // the walk runs in window coordinates (cr = cur - w0)
      const int limit = (p > ZS_MAX_DIST ? (int)(p - ZS_MAX_DIST) : 0) - (int)w0;  // deflate.ts:1060
      const uint32_t sp = p - w0;
      const uint32_t s0 = win_word(wb, sp), s1 = win_word(wb, sp + 4);
      // best = (len << 16) | cr: its maximum is the first candidate among the
      // longest, as the walk visits cr in decreasing order -- "first strictly
      // longer wins" (deflate.ts:1100-1105); starts at MIN_MATCH - 1 = 2
      uint32_t best = (2u << 16) | 0xffffu;
      uint32_t cr = q0 - w0;
      // The 8-byte compare gives k = min(matched bytes, 8).  Below kx = min(nice,
      // 8) the candidate is final (k < nice <= maxc, no clamp); at k >= kx it
      // goes to the rare path that extends the compare, clamps to maxc and tests
      // nice (nice >= 8 unless the stream ends within 8 bytes).
      const uint32_t kx = nice < 8u ? nice : 8u;
      // Every candidate a lane evaluates is one chain step, and a lane leaves at
      // a nice match or the chain's end: the reference's chain counter is the
      // step count.  The walk runs in two phases so that the chain >> 2 result
      // (deflate.ts:1075-1077) is a snapshot between them, not a per-step test.
      auto walk = [&](uint32_t rem) {
        // the step budget is counted down in a VGPR (the asm hides that it is
        // uniform): its test then joins the per-lane exit mask in one v_cmp
        asm volatile("v_mov_b32 %0, %1" : "=v"(rem) : "s"(rem));
        for (;;) {
          const uint32_t cp = cr;
          // the chain link and the first 8 bytes (three aligned LDS words) are read together
          uint32_t d = pv[cp];
          const uint32_t wi = cp >> 2;
          const uint32_t a0 = wb[wi], a1 = wb[wi + 1], a2 = wb[wi + 2];
          const uint32_t x0 = __builtin_amdgcn_alignbyte(a1, a0, cp) ^ s0;  // alignbyte uses cp & 3
          const uint32_t x1 = __builtin_amdgcn_alignbyte(a2, a1, cp) ^ s1;
          // first differing bit, 64 if none (ffbl(0) = ~0, and the clamped add keeps it there)
          uint32_t f0, f1;
          asm("v_ffbl_b32 %0, %1" : "=v"(f0) : "v"(x0));
          asm("v_ffbl_b32 %0, %1\n\tv_add_u32_e64 %0, %0, 32 clamp" : "=&v"(f1) : "v"(x1));
          uint32_t k = min(min(f0, f1), 64u) >> 3;
          if (__builtin_expect(k >= kx, 0)) {
            if (k == 8u) {  // longer than 8 bytes: finish the compare
              while (k < maxc) {
                const uint32_t y = win_word(wb, cp + k) ^ win_word(wb, sp + k);
                if (y) { k += (uint32_t)(__builtin_ctz(y) >> 3); break; }
                k += 4;
              }
            }
            k = k < maxc ? k : maxc;
            if (k >= nice) d = 0xffffu;  // nice match (deflate.ts:1103): end the chain like a missing link
          }
          best = max(best, (k << 16) | cr);
          const int nxt = (int)cr - (int)d;
          cr = (uint32_t)nxt;
          // ends: no link / cur <= limit (deflate.ts:1109), or the budget
          if ((nxt <= limit) | (--rem == 0)) return;
        }
      };
      // A lane leaving the first phase early has ended its chain; the others all
      // stand at step chain >> 2, so the second phase starts at a uniform step and
      // whether a lane goes on is recomputed from cr -- no loop live-out state
      // beyond it.
      walk(budget_small);
      const uint32_t best_s = best;  // lanes still walking: after chain >> 2 candidates; others: final
      asm volatile("" : "+v"(cr));  // recompute the chain-end test below instead of keeping a mask live
      if (budget_small < budget && (int)cr > limit) walk(budget - budget_small);
      const uint32_t flag = d0 == ZS_MAX_DIST ? 0x8000u : 0u;  // SURVEY A3 slide-NIL corner, resolved in parse
      const uint32_t bl = best >> 16, bsl = best_s >> 16;
      r.x = (bl << 16) | (bl > 2 ? sp - (best & 0xffffu) : 0u) | flag;
      r.y = (bsl << 16) | (bsl > 2 ? sp - (best_s & 0xffffu) : 0u);
    }
    out[p] = r;
  }
}
