// deflate_sweep.hip -- LZ77 match finding for deflate levels 4..9 on gfx950,
// streams of at most 65,537 bytes (the batch workloads' 64 KiB streams).
//
// What it computes is what zs_k_match (deflate_match.hip) computes: for EVERY
// position p, the (length, distance) the reference's longest_match
// (deflate.ts:1053-1115) returns at p for the full chain budget and for the
// budget >> 2 used when prev_length >= good_match (deflate.ts:1075-1077).  At
// levels 4..9 every position <= n-3 is inserted into its hash chain exactly
// once and in order, so p's chain is "every earlier inserted
// position with the same 15-bit hash, most recent first", cut at
// limit = p - MAX_DIST (deflate.ts:1060,1109) and by the budget.
//
// How is different.  Instead of following prev[] links (a dependent LDS
// round trip per chain step), the positions are counting-sorted by (hash,
// position) into a "member" array (zs_k_bucket).  Member k's chain is then
// simply members k-1, k-2, ... of its bucket, and the t-th predecessor is the
// t-th chain step.  zs_k_sweep gives each lane one member and sweeps t = 1,
// 2, ... for all 64 lanes at once: lane i reads the record of member
// k0 + i - t from a per-wave LDS ring (consecutive lanes, consecutive 16-byte
// records: conflict-free, and no load depends on the previous step), compares
// the 11-byte signatures with xor + ffbl, and keeps the first maximum.
//
// Exactness (checked off the GPU by tools/emu/emu_bucket_sweep.c against a
// direct longest_match, and on the GPU by tests/test_gpu_deflate.py):
//   * liveness: record key = hash << 16 | pos; the head (t = 1) needs
//     key >= hash << 16 | max(limit, 1) (non-NIL, distance <= MAX_DIST,
//     deflate.ts:1376), the chain (t >= 2) key > hash << 16 | limit
//     (deflate.ts:1109); a member of another bucket fails both.  Liveness is
//     monotone in t, so a lane leaves at its first dead step.
//   * first strictly longer match wins (deflate.ts:1100-1105): the best is the
//     maximum of (len << 16) | (0xffff - t).  Lengths are clamped to maxc =
//     min(258, lookahead) (deflate.ts:1068): short candidates match at most
//     10 bytes, and a lane with maxc <= 12 re-walks its chain exactly.
//   * a candidate whose 11 signature bytes all match (maxc > 12) is "long":
//     its exact length needs the window.  Up to four are recorded in chain
//     order and extended after the sweep, with the nice cut-off (nice >= 16 at
//     levels 4..9, so no short candidate reaches it unless the stream ends
//     first, where maxc clamps it); when one exists within the budget the
//     result is among them (every short one is <= 10).
//     A fifth long candidate ends the lane's sweep, and the lane re-walks its
//     chain from the first long one (repetitive data: the first is usually a
//     nice match).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"

#define ZS_SWEEP_MAX 65537u  // position + 1 <= 65535 for every inserted position: u16 members and offsets
#define ZS_SW_WIN_WORDS ((ZS_SWEEP_MAX + 20u + 3u) / 4u + 2u)
#define ZS_SW_SIG 11u  // signature bytes compared per chain step (see sw_lcp)
#define ZS_SW_RING 128u  // records per wave (two blocks of 64 members), stored twice (mirror)

typedef __attribute__((address_space(3))) uint32_t zs_sw_lds_u32;
static __device__ __forceinline__ uint32_t sw_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const zs_sw_lds_u32*)p;
}

static __device__ __forceinline__ uint32_t sw_hash(uint32_t w) {  // SURVEY A1, bytes 0..2 of w
  return (((w & 0xffu) << 10) ^ (((w >> 8) & 0xffu) << 5) ^ ((w >> 16) & 0xffu)) & ZS_HASH_MASK;
}

// -------------------------------------------------------------- zs_k_bucket
// One workgroup (4 waves) per stream: a counting sort of the inserted
// positions p <= n-3 by their hash, stable in position, into members[] (u16,
// the stream's range of the per-position workspace).  Pass 1 counts (32768 u16
// buckets, two per LDS word; all four waves), an exclusive scan turns the
// counts into offsets, and pass 2 -- one wave -- walks the positions in order,
// 64 per instruction, claiming slots with ONE ds_add_rtn_u32 per lane: gfx950
// applies same-address LDS atomics of one wave instruction in increasing lane
// order (zs_selftest checks it, including the 16-bit half form used here), so
// equal hashes get slots in position order.  Pass 1 hashes input words held
// in registers, pass 2 a 4 KiB LDS stage of the input.  Results of the
// positions that are not inserted (the last two) are zeroed.
#define ZS_BK_THREADS 256u
#define ZS_BK_INFLIGHT 8  // pass 2: wave instructions (x 64 positions) per wait
#define ZS_BK_CHUNK 2048u  // pass 2: positions per chunk (input bytes staged in LDS, slots queued)

__global__ __launch_bounds__(ZS_BK_THREADS) void zs_k_bucket(const uint8_t* __restrict__ in,
                                                            const uint64_t* __restrict__ in_off,
                                                            const uint32_t* __restrict__ in_len,
                                                            const uint64_t* __restrict__ pos_base,
                                                            uint16_t* __restrict__ members, uint2* __restrict__ mres) {
  __shared__ uint32_t cnt[16384];
  __shared__ uint32_t part[ZS_BK_THREADS];
  __shared__ uint32_t stg[ZS_BK_CHUNK / 4 + 2];
  __shared__ uint16_t q[2][ZS_BK_CHUNK];
  const int s = blockIdx.x;
  const uint32_t n = in_len[s];
  if (n > ZS_SWEEP_MAX) return;  // zs_k_prev / zs_k_match's stream
  const uint32_t tid = threadIdx.x;
  const uint8_t* src = in + in_off[s];
  uint16_t* mem = members + pos_base[s];
  uint2* out = mres + pos_base[s];
  const uint32_t m = n > 2 ? n - 2 : 0u;  // inserted positions (deflate.ts:1367-1370)
  for (uint32_t p = m + tid; p < n; p += ZS_BK_THREADS) out[p] = make_uint2(0, 0);
  if (m == 0) return;
  for (uint32_t i = tid; i < 16384 / 4; i += ZS_BK_THREADS) reinterpret_cast<uint4*>(cnt)[i] = make_uint4(0, 0, 0, 0);
  const bool aligned = ((uintptr_t)src & 3u) == 0;
  __syncthreads();
  // pass 1: bucket sizes (unordered adds, all waves).  Thread t hashes the 16
  // positions [p0 + 16 t, +16) from 5 input words; the next 4 KiB block's words
  // are loaded before this block's adds (a load round trip per block, not per
  // four positions).
  {
    uint32_t w[5], nw[5];
    auto load5 = [&](uint32_t p0, uint32_t* x) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < 5; k++) x[k] = zs_load_word(src, n, p0 + 16 * tid + 4 * k);
    };
    load5(0, nw);
    for (uint32_t p0 = 0; p0 < m; p0 += 16 * ZS_BK_THREADS) {
#pragma unroll
      for (int k = 0; k < 5; k++) w[k] = nw[k];
      if (p0 + 16 * ZS_BK_THREADS < m) load5(p0 + 16 * ZS_BK_THREADS, nw);
#pragma unroll
      for (uint32_t j = 0; j < 16; j++) {
        const uint32_t p = p0 + 16 * tid + j;
        const uint32_t h = sw_hash(__builtin_amdgcn_alignbyte(w[(j >> 2) + 1], w[j >> 2], j & 3u));
        if (p < m) atomicAdd(&cnt[h >> 1], 1u << (16u * (h & 1u)));
      }
    }
  }
  __syncthreads();
  // exclusive scan: thread i owns words [64i, 64i + 64) (buckets 128i ...)
  {
    uint32_t sum = 0;
    for (uint32_t j = 0; j < 64; j++) {
      const uint32_t w = cnt[64 * tid + ((j + tid) & 63u)];  // rotated: threads hit different banks
      sum += (w & 0xffffu) + (w >> 16);
    }
    part[tid] = sum;
    __syncthreads();
    if (tid < 64) {  // scan of the 256 partial sums, one wave
      uint32_t v[4], t = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) { v[j] = part[4 * tid + j]; t += v[j]; }
      uint32_t x = t;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (tid >= (uint32_t)d) x += y;
      }
      uint32_t run = x - t;
#pragma unroll
      for (int j = 0; j < 4; j++) { part[4 * tid + j] = run; run += v[j]; }
    }
    __syncthreads();
    uint32_t run = part[tid];
    for (uint32_t j = 0; j < 64; j++) {
      const uint32_t i = 64 * tid + ((j + tid) & 63u);
      (void)i;
      const uint32_t w = cnt[64 * tid + j];
      const uint32_t lo = w & 0xffffu;
      cnt[64 * tid + j] = run | ((run + lo) << 16);
      run += lo + (w >> 16);
    }
  }
  __syncthreads();
  // pass 2: wave 0 claims the slots in position order, ZS_BK_CHUNK positions
  // at a time, into an LDS queue (slot of chunk position o at q[c & 1][o]);
  // waves 1..3 scatter the previous chunk's positions to their slots while it
  // claims the next one (stores from one wave alone take longer than the
  // claims: 64 scattered 2-byte stores per instruction).  The input goes
  // through LDS a chunk at a time (stg), the next chunk's loads in flight in
  // registers while this chunk's positions are claimed, ZS_BK_INFLIGHT
  // instructions per wait.
  const uint32_t wave = tid >> 6, lane = tid & 63u;
  constexpr uint32_t CW = ZS_BK_CHUNK / 4 / 64;  // words per lane per chunk
  uint32_t nxt[CW + 1];
  auto fetch = [&](uint32_t c0) {
#pragma unroll
    for (uint32_t i = 0; i <= CW; i++) {
      const uint32_t w = 64 * i + lane;  // word index within the chunk (+ 2 words of overlap)
      const uint32_t at = c0 + 4 * w;
      uint32_t v = 0;
      if (w < ZS_BK_CHUNK / 4 + 2) {
        if (aligned && at + 4 <= n) v = *(const uint32_t*)(src + at);
        else
          for (uint32_t k = 0; k < 4; k++)
            if (at + k < n) v |= (uint32_t)src[at + k] << (8 * k);
      }
      nxt[i] = v;
    }
  };
  if (wave == 0) fetch(0);
  const uint32_t nch = (m + ZS_BK_CHUNK - 1) / ZS_BK_CHUNK;
  for (uint32_t c = 0; c <= nch; c++) {
    const uint32_t c0 = c * ZS_BK_CHUNK;
    if (wave == 0 && c < nch) {
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t i = 0; i <= CW; i++)
        if (64 * i + lane < ZS_BK_CHUNK / 4 + 2) stg[64 * i + lane] = nxt[i];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      if (c0 + ZS_BK_CHUNK < m) fetch(c0 + ZS_BK_CHUNK);
      const uint32_t c1 = min(m, c0 + ZS_BK_CHUNK);
      uint16_t* const qc = q[c & 1u];
      for (uint32_t g0 = c0; g0 < c1; g0 += 64 * ZS_BK_INFLIGHT) {
        uint32_t a[ZS_BK_INFLIGHT], v[ZS_BK_INFLIGHT], sh[ZS_BK_INFLIGHT], e[ZS_BK_INFLIGHT];
#pragma unroll
        for (int j = 0; j < ZS_BK_INFLIGHT; j++) {
          const uint32_t p = g0 + 64 * j + lane;
          const uint32_t o = p - c0;
          const uint32_t h = sw_hash(__builtin_amdgcn_alignbyte(stg[(o >> 2) + 1], stg[o >> 2], o & 3u));
          sh[j] = 16u * (h & 1u);
          a[j] = sw_lds_addr(&cnt[h >> 1]);
          v[j] = p < c1 ? 1u << sh[j] : 0u;  // a lane past the chunk adds nothing
        }
        // in order: instruction j's adds land after instruction j-1's (LDS executes a wave's ops in order)
        asm volatile(
            "ds_add_rtn_u32 %0, %8, %16\n\t"
            "ds_add_rtn_u32 %1, %9, %17\n\t"
            "ds_add_rtn_u32 %2, %10, %18\n\t"
            "ds_add_rtn_u32 %3, %11, %19\n\t"
            "ds_add_rtn_u32 %4, %12, %20\n\t"
            "ds_add_rtn_u32 %5, %13, %21\n\t"
            "ds_add_rtn_u32 %6, %14, %22\n\t"
            "ds_add_rtn_u32 %7, %15, %23\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(e[0]), "=&v"(e[1]), "=&v"(e[2]), "=&v"(e[3]), "=&v"(e[4]), "=&v"(e[5]), "=&v"(e[6]), "=&v"(e[7])
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(v[0]),
              "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7])
            : "memory");
#pragma unroll
        for (int j = 0; j < ZS_BK_INFLIGHT; j++) {
          const uint32_t p = g0 + 64 * j + lane;
          if (p < c1) qc[p - c0] = (uint16_t)(e[j] >> sh[j]);
        }
      }
    } else if (wave != 0 && c > 0) {
      const uint32_t b0 = c0 - ZS_BK_CHUNK, cnt1 = min(m, c0) - b0;
      const uint16_t* const qp = q[(c - 1) & 1u];
      for (uint32_t o = tid - 64u; o < cnt1; o += ZS_BK_THREADS - 64u) mem[qp[o]] = (uint16_t)(b0 + o);
    }
    __syncthreads();
  }
}

// --------------------------------------------------------------- zs_k_sweep
static __device__ __forceinline__ uint32_t sw_word(const uint32_t* win, uint32_t off) {
  const uint32_t i = off >> 2;
  return __builtin_amdgcn_alignbyte(win[i + 1], win[i], off & 3u);
}

// exact length of a candidate whose first ZS_SW_SIG bytes match, clamped to maxc
static __device__ __forceinline__ uint32_t sw_extend(const uint32_t* win, uint32_t p, uint32_t q, uint32_t maxc) {
  uint32_t k = ZS_SW_SIG;
  while (k < maxc) {
    const uint32_t y = sw_word(win, q + k) ^ sw_word(win, p + k);
    if (y) { k += (uint32_t)(__builtin_ctz(y) >> 3); break; }
    k += 4;
  }
  return k < maxc ? k : maxc;
}

// Signatures are 11 bytes: a record's third word keeps bytes 8..10 (byte 11
// zeroed, sw_rec2) and the lane's own third word carries a sentinel bit 24
// (sw_own2), so the xor of the third words always has bit 24 set.  The
// matched-byte count then saturates at 11 by itself -- no per-step cap -- and
// lanes whose lookahead is at most 12 bytes (maxc <= 12, the last positions
// of a stream) take an exact re-walk after the sweep instead.
static __device__ __forceinline__ uint32_t sw_rec2(uint32_t w2) { return w2 & 0x00ffffffu; }
static __device__ __forceinline__ uint32_t sw_own2(uint32_t w2) { return (w2 & 0x00ffffffu) | 0x01000000u; }
// matched bytes (0..11) of a candidate's record words (a) against the lane's own (b)
static __device__ __forceinline__ uint32_t sw_lcp(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t b0, uint32_t b1,
                                                  uint32_t b2) {
  uint32_t f0, f1, f2;
  asm("v_ffbl_b32 %0, %1" : "=v"(f0) : "v"(a0 ^ b0));
  asm("v_ffbl_b32 %0, %1\n\tv_add_u32_e64 %0, %0, 32 clamp" : "=&v"(f1) : "v"(a1 ^ b1));
  asm("v_ffbl_b32 %0, %1\n\tv_add_u32_e32 %0, 64, %0" : "=&v"(f2) : "v"(a2 ^ b2));
  // ffbl(0) = ~0 and the clamped add keep "no difference" at ~0; f2 <= 88 (the sentinel)
  return min(min(f0, f1), f2) >> 3;
}

struct SwRec {
  uint32_t w0, w1, w2, key;  // bytes [q, q + 12) and hash << 16 | q
};

__global__ __launch_bounds__(1024) void zs_k_sweep(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len,
                                                   const uint64_t* __restrict__ pos_base,
                                                   const uint16_t* __restrict__ members, uint2* __restrict__ mres,
                                                   int chain, int nice_cfg) {
  __shared__ __attribute__((aligned(16))) SwRec ring[16][2 * ZS_SW_RING];
  __shared__ __attribute__((aligned(16))) uint32_t win[ZS_SW_WIN_WORDS];
  __shared__ uint32_t next;
  const int s = blockIdx.x;
  const uint32_t n = in_len[s];
  if (n > ZS_SWEEP_MAX || n < 3) return;
  const uint32_t m = n - 2;
  const uint8_t* src = in + in_off[s];
  const uint16_t* mem = members + pos_base[s];
  uint2* out = mres + pos_base[s];
  // the whole stream in LDS, zero padded (reads run up to 16 bytes past n)
  if ((((uintptr_t)src) & 15u) == 0) {
    for (uint32_t i = threadIdx.x; 4 * i < ZS_SW_WIN_WORDS; i += 1024) {
      const uint32_t b = 16 * i;
      uint4 v;
      if (b + 16 <= n) v = ((const uint4*)src)[i];
      else {
        uint32_t t[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 16; k++)
          if (b + k < n) t[k >> 2] |= (uint32_t)src[b + k] << (8 * (k & 3));
        v = make_uint4(t[0], t[1], t[2], t[3]);
      }
      if (4 * i + 3 < ZS_SW_WIN_WORDS) *(uint4*)(win + 4 * i) = v;
      else for (uint32_t k = 0; 4 * i + k < ZS_SW_WIN_WORDS; k++) win[4 * i + k] = (&v.x)[k];
    }
  } else {
    for (uint32_t i = threadIdx.x; i < ZS_SW_WIN_WORDS; i += 1024) {
      uint32_t v = 0;
      for (uint32_t k = 0; k < 4; k++)
        if (4 * i + k < n) v |= (uint32_t)src[4 * i + k] << (8 * k);
      win[i] = v;
    }
  }
  if (threadIdx.x == 0) next = 0;
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  SwRec* const R = ring[threadIdx.x >> 6];
  const uint32_t budget = (uint32_t)chain, budget_s = (uint32_t)chain >> 2;
  const uint32_t nchunks = (m + 63) / 64;
  // Member j's record lives in ring slot j mod 128 and again 128 slots later,
  // so that a block's 64 steps read slots base .. base + 63 without wrapping.
  auto put_rec = [&](int j, SwRec r) {
    const uint32_t i = (uint32_t)j & (ZS_SW_RING - 1);
    R[i] = r;
    R[i + ZS_SW_RING] = r;
  };
  auto load_rec = [&](int j) {  // key 0 = no member: fails every liveness test
    SwRec r = {0, 0, 0, 0};
    if (j >= 0 && (uint32_t)j < m) {
      const uint32_t q = mem[j];
      r.w0 = sw_word(win, q);
      r.w1 = sw_word(win, q + 4);
      r.w2 = sw_rec2(sw_word(win, q + 8));
      r.key = (sw_hash(r.w0) << 16) | q;
    }
    put_rec(j, r);
  };
  for (;;) {
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&next, 1u);
    c = __builtin_amdgcn_readfirstlane(c);
    if (c >= nchunks) break;
    const int k0 = (int)(64 * c);
    const int k = k0 + (int)lane;
    const bool own = (uint32_t)k < m;
    const uint32_t p = own ? mem[k] : 0u;
    const uint32_t s0 = sw_word(win, p), s1 = sw_word(win, p + 4), s2r = sw_word(win, p + 8);
    const uint32_t s2 = sw_own2(s2r);
    const uint32_t h = sw_hash(s0);
    const uint32_t look = n - p;
    const uint32_t maxc = look < ZS_MAX_MATCH ? look : ZS_MAX_MATCH;                 // deflate.ts:1068
    const uint32_t nice = look < (uint32_t)nice_cfg ? look : (uint32_t)nice_cfg;      // deflate.ts:1078-1080
    const bool tail = maxc <= 12u;  // exact re-walk after the sweep
    const uint32_t long_thr = tail ? 12u : ZS_SW_SIG;  // a tail lane records no long candidates
    const uint32_t limit = p > ZS_MAX_DIST ? p - ZS_MAX_DIST : 0u;                   // deflate.ts:1060
    const uint32_t khead = (h << 16) | (limit > 1u ? limit : 1u);
    const uint32_t klim = (h << 16) | limit;
    // ring: this chunk's block and the one before it
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    put_rec(k, own ? SwRec{s0, s1, sw_rec2(s2r), (h << 16) | p} : SwRec{0, 0, 0, 0});
    load_rec(k - 64);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();

    uint32_t best = 2u << 16, best_s = 2u << 16;
    uint32_t nl = 0, l0 = 0, l1 = 0, l2 = 0, l3 = 0;  // long candidates: t << 16 | pos, in chain order
    bool ovf = false;
    // The live lanes as a wave-uniform lane mask (SGPRs): a chain step is a
    // compare into a mask, scalar ands and one masked select per lane.
    uint64_t alive_m = 0;
    uint32_t head = 0;  // bit 0: head candidate valid; 0x8000: at exactly MAX_DIST
    auto note_long = [&](uint32_t t, uint32_t key) {
      if (nl == 4) {  // a fifth: the lane stops (cleared from alive_m by the caller) and re-walks its chain afterwards
        ovf = true;
      } else {
        const uint32_t e = (t << 16) | (key & 0xffffu);
        l0 = nl == 0 ? e : l0;
        l1 = nl == 1 ? e : l1;
        l2 = nl == 2 ? e : l2;
        l3 = nl == 3 ? e : l3;
        nl++;
      }
    };
    // t = 1: the head candidate (deflate.ts:1376)
    {
      const SwRec r = R[(uint32_t)(k - 1) & (ZS_SW_RING - 1)];
      bool a1 = false;
      if (own && r.key >= khead) {
        a1 = true;
        head = 1u | ((p - (r.key & 0xffffu)) == ZS_MAX_DIST ? 0x8000u : 0u);
        const uint32_t kk = sw_lcp(r.w0, r.w1, r.w2, s0, s1, s2);
        if (kk >= long_thr) note_long(1, r.key);
        best = max(best, (kk << 16) | (0xffffu - 1u));
      }
      alive_m = __builtin_amdgcn_ballot_w64(a1);
    }
    // One chain step for every lane: a dead lane's result simply stops
    // changing (no per-step exit, no exec-mask bookkeeping).
    // A step returns its score, 0 for a dead lane (below every best).  The
    // caller takes the maximum of a group's scores (v_max3), folds it into
    // best with one v_max, and finds the group's long candidates from it: a
    // live long candidate scores at least long_thr << 16, a dead one 0.
    const uint32_t long16 = long_thr << 16;
    auto step = [&](const uint4 r, uint32_t t) -> uint32_t {
      alive_m &= __builtin_amdgcn_ballot_w64(r.w > klim);  // the chain ends at the first dead step (deflate.ts:1109)
      const uint32_t kk = sw_lcp(r.x, r.y, r.z, s0, s1, s2);
      uint32_t sc, sl;
      // one v_lshl_or (the compiler would otherwise fold the >> 3 into a shift, an and and an or)
      asm("v_lshl_or_b32 %0, %1, 16, %2" : "=v"(sl) : "v"(kk), "s"(0xffffu - t));
      asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(sc) : "v"(sl), "s"(alive_m));
      return sc;
    };
    // Long candidates are rare (~1 % of groups): a group with one is re-run
    // step by step to record them in chain order.
    auto relong = [&](const SwRec* Rg, uint32_t t0, uint32_t cnt, uint64_t al_m) {
      bool al = ((al_m >> lane) & 1u) != 0;
      for (uint32_t u = 0; u < cnt; u++) {
        const SwRec r = Rg[-(int)u];
        al = al && r.key > klim;
        if (al && sw_lcp(r.w0, r.w1, r.w2, s0, s1, s2) >= long_thr) {
          note_long(t0 + u, r.key);
          if (ovf) al = false;
        }
      }
      alive_m &= ~__builtin_amdgcn_ballot_w64(ovf);
    };
    // Steps 2..4 (block 0, before the first full group).
    {
      const SwRec* const Rg = R + (((uint32_t)(k - 64) & (ZS_SW_RING - 1)) + 64u - 2u);
      const uint64_t alive0 = alive_m;
      uint32_t gm = 0;
      for (uint32_t u = 0; u < 3; u++) gm = max(gm, step(*(const uint4*)(Rg - (int)u), 2u + u));
      best = max(best, gm);
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(gm >= long16) != 0, 0)) relong(Rg, 2u, 3u, alive0);
    }
    // Steps [ta, tb] of block b in groups of four (ta = 1 mod 4, tb = 0 mod 4,
    // wave-uniform).  Step t reads slot base_b + 64b + 64 - t: one address per
    // group, immediate offsets inside, all four records loaded up front.
    auto run = [&](uint32_t b, uint32_t ta, uint32_t tb) {
      const uint32_t base_b = (uint32_t)(k - 64 * (int)b - 64) & (ZS_SW_RING - 1);
      const SwRec* const Rb = R + base_b + 64u * b + 64u;
      for (uint32_t t0 = ta; t0 <= tb; t0 += 4) {
        const SwRec* const Rg = Rb - t0;  // step t0 + u reads Rg[-u]
        const uint4 r0 = *(const uint4*)(Rg), r1 = *(const uint4*)(Rg - 1), r2 = *(const uint4*)(Rg - 2),
                    r3 = *(const uint4*)(Rg - 3);
        const uint64_t alive0 = alive_m;
        const uint32_t c0 = step(r0, t0), c1 = step(r1, t0 + 1);
        const uint32_t c2 = step(r2, t0 + 2), c3 = step(r3, t0 + 3);
        const uint32_t gm = max(max(c0, c1), max(c2, c3));
        best = max(best, gm);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(gm >= long16) != 0, 0)) relong(Rg, t0, 4u, alive0);
        if (!alive_m) break;
      }
    };
    bool snapped = false;
    for (uint32_t b = 0;; b++) {
      // block b = steps (64b, 64b + 64]: members k0 - 64b - 64 ... k0 - 64b + 62, i.e. the blocks b and b + 1 back
      if (b >= 1) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        load_rec(k - 64 * (int)(b + 1));
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
      const uint32_t ta = b == 0 ? 5u : 64u * b + 1u;
      const uint32_t tb = min(64u * b + 64u, budget);
      if (!snapped && budget_s <= tb) {  // the chain >> 2 result (deflate.ts:1075-1077); budgets are multiples of 4
        if (budget_s >= ta) run(b, ta, budget_s);
        best_s = best;
        snapped = true;
        if (budget_s + 1u <= tb) run(b, max(ta, budget_s + 1u), tb);
      } else {
        run(b, ta, tb);
      }
      if (tb >= budget || !alive_m) break;
    }
    if (!snapped) best_s = best;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if (own) {
      uint32_t rx = 0, ry = 0;
      if (head) {
        if (tail) {  // maxc <= 12: min(lcp, maxc) exactly, first maximum in chain order (deflate.ts:1082-1105)
          uint32_t b = 2u << 16, bs = 2u << 16;
          for (uint32_t t = 1; t <= budget && (int)t <= k; t++) {
            const uint32_t q = mem[k - (int)t];
            const uint32_t key = (sw_hash(sw_word(win, q)) << 16) | q;
            if (t == 1u ? key < khead : key <= klim) break;
            uint32_t len = 12;
            for (uint32_t o = 0; o < 12u; o += 4) {
              const uint32_t y = sw_word(win, q + o) ^ sw_word(win, p + o);
              if (y) { len = o + (uint32_t)(__builtin_ctz(y) >> 3); break; }
            }
            const uint32_t sc = ((len < maxc ? len : maxc) << 16) | (0xffffu - t);
            b = max(b, sc);
            if (t <= budget_s) bs = max(bs, sc);
          }
          best = b;
          best_s = bs;
        }
        const uint32_t bl = best >> 16, bsl = best_s >> 16;
        uint32_t bd = bl > 2u ? p - mem[k - (int)(0xffffu - (best & 0xffffu))] : 0u;
        uint32_t bsd = bsl > 2u ? p - mem[k - (int)(0xffffu - (best_s & 0xffffu))] : 0u;
        uint32_t L = bl, Ls = bsl;
        if (nl) {
          uint32_t lb = 0, ld = 0, lbs = 0, lds = 0;
          auto take = [&](uint32_t t, uint32_t q) -> bool {
            const uint32_t len = sw_extend(win, p, q, maxc);
            if (len > lb) { lb = len; ld = p - q; }
            if (t <= budget_s && len > lbs) { lbs = len; lds = p - q; }
            return len >= nice;  // nice match: the walk ends (deflate.ts:1103)
          };
          if (ovf) {  // re-walk the chain from the first long candidate
            for (uint32_t t = l0 >> 16; t <= budget && (int)t <= k; t++) {
              const uint32_t q = mem[k - (int)t];
              const uint32_t w0 = sw_word(win, q), w1 = sw_word(win, q + 4), w2 = sw_rec2(sw_word(win, q + 8));
              const uint32_t key = (sw_hash(w0) << 16) | q;
              if (t == 1u ? key < khead : key <= klim) break;
              if (sw_lcp(w0, w1, w2, s0, s1, s2) < long_thr) continue;
              if (take(t, q)) break;
            }
          } else {
            if (!take(l0 >> 16, l0 & 0xffffu) && nl > 1 && !take(l1 >> 16, l1 & 0xffffu) && nl > 2 &&
                !take(l2 >> 16, l2 & 0xffffu) && nl > 3)
              take(l3 >> 16, l3 & 0xffffu);
          }
          L = lb;
          bd = ld;
          if (lbs) { Ls = lbs; bsd = lds; }
        }
        rx = (L << 16) | (L > 2u ? bd : 0u) | (head & 0x8000u);
        ry = (Ls << 16) | (Ls > 2u ? bsd : 0u);
      }
      out[p] = make_uint2(rx, ry);
    }
  }
}
