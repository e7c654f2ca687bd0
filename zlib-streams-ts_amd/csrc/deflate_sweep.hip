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
// k0 + i - t from a per-wave LDS ring (dense arrays: consecutive lanes read
// consecutive elements, conflict-free, and no load depends on the previous
// step), compares signatures with xor + ffbl, and keeps the first longest
// through a group maximum (sw_body below).
//
// Signatures: the 11 bytes after the hashed position's first byte, with a
// sentinel bit (SwSig<false>); for streams of 7-bit bytes (ASCII text) 8
// bytes [X, b3..b9] where X recovers the 9 bits of b0..b2 the 15-bit hash
// loses (SwSig<true>: bucket-mates with equal X and hash have equal b0..b2).
//
// Exactness (checked off the GPU by tools/emu/emu_bucket_sweep.c against a
// direct longest_match, and on the GPU by tests/test_gpu_deflate.py):
//   * liveness: record key = hash << 16 | pos; the head (t = 1) needs
//     key >= hash << 16 | max(limit, 1) (non-NIL, distance <= MAX_DIST,
//     deflate.ts:1376), the chain (t >= 2) key > hash << 16 | limit
//     (deflate.ts:1109); a member of another bucket fails both.  Liveness is
//     monotone in t.
//   * first strictly longer match wins (deflate.ts:1100-1105): the maximum of
//     a group's scores (matched bits, low bits = 7 - its place in the group)
//     is its first longest candidate; a group's winner replaces the best only
//     when longer.  Lengths are clamped to maxc = min(258, lookahead)
//     (deflate.ts:1068); the last positions of a stream re-walk exactly.
//   * a candidate whose whole signature matches is "long": the lanes holding
//     one extend it on the spot from the stream window (nice cut-off,
//     deflate.ts:1100-1105); long candidates beat every short one.
//   * both budgets in one sweep: the chain >> 2 result is a snapshot of the
//     state after step chain >> 2 (groups are cut there).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"
#include <type_traits>

// the window in LDS: ZS_SEG_WPOS inserted positions, a longest match past the
// last of them (258 bytes) and the 16-byte overreach of the word compares
#define ZS_SW_WIN_WORDS ((ZS_SEG_WPOS + 258u + 20u + 3u) / 4u + 2u)
#define ZS_SW_RING 128u  // records per wave (two blocks of 64 members), stored twice (mirror)
#ifndef ZS_SW_EXP
#define ZS_SW_EXP 0  // experiments (timing A/B only; 0 in the product)
#endif
#define ZS_SW_MW 320u    // per-wave LDS window of member positions (chain + 64 <= ZS_SW_MW: levels 4..7)

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
#define ZS_BK_WPT (16384u / ZS_BK_THREADS)  // scan: count words per thread
#define ZS_BK_PPL (ZS_BK_THREADS / 64u)     // scan: partial sums per lane of the wave-level scan
#ifndef ZS_BK_PROF
#define ZS_BK_PROF 0  // timing experiments: wall-clock per pass summed over workgroups (0 in the product)
#endif
#if ZS_BK_PROF
__device__ unsigned long long zs_bk_stat[4];  // pass 1, scan, pass 2, workgroups
extern "C" int zs_bucket_stats(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_bk_stat), sizeof(zs_bk_stat));
}
#define BK_MARK(i) do { if (threadIdx.x == 0) { const unsigned long long t_ = wall_clock64(); atomicAdd(&zs_bk_stat[i], t_ - bk_t); bk_t = t_; } } while (0)
#else
#define BK_MARK(i) do { } while (0)
#endif
#define ZS_BK_INFLIGHT 8  // pass 2: wave instructions (x 64 positions) per wait
#define ZS_BK_CHUNK 2048u  // pass 2: positions per chunk (input bytes staged in LDS, slots queued)

template <bool ORD>  // false: claims ranked by zs_wave_match instead of the LDS atomics' lane order
__global__ __launch_bounds__(ZS_BK_THREADS) void zs_k_bucket(const uint8_t* __restrict__ in,
                                                            const uint64_t* __restrict__ in_off,
                                                            const uint32_t* __restrict__ in_len,
                                                            const uint64_t* __restrict__ pos_base,
                                                            const zs_sweep_seg* __restrict__ segs,
                                                            uint16_t* __restrict__ members, uint2* __restrict__ mres) {
  __shared__ uint32_t cnt[16384];
  __shared__ uint32_t part[ZS_BK_THREADS];
  __shared__ uint32_t stg[ZS_BK_CHUNK / 4 + 2];
  __shared__ uint16_t q[2][ZS_BK_CHUNK];
  const zs_sweep_seg G = segs[blockIdx.x];
  const int s = (int)G.s;
  const uint32_t nrel = in_len[s] - G.base;  // bytes from the window's start to the stream's end
  const uint32_t tid = threadIdx.x;
  const uint8_t* src = in + in_off[s] + G.base;
  uint16_t* mem = members + G.mb;
  uint2* out = mres + pos_base[s] + G.base;
  // inserted positions of the window (deflate.ts:1367-1370: p <= n - 3), and the bytes their hashes read
  const uint32_t m = nrel > 2 ? min(nrel - 2, G.ohi) : 0u;
  const uint32_t n = min(nrel, m + 2u);
  if (nrel - m <= 2u)  // the window reaches the stream's end: its last positions are not inserted
    for (uint32_t p = m + tid; p < nrel; p += ZS_BK_THREADS) out[p] = make_uint2(0, 0);
  if (m == 0) return;
  for (uint32_t i = tid; i < 16384 / 4; i += ZS_BK_THREADS) reinterpret_cast<uint4*>(cnt)[i] = make_uint4(0, 0, 0, 0);
  const bool aligned = ((uintptr_t)src & 3u) == 0;
#if ZS_BK_PROF
  unsigned long long bk_t = wall_clock64();
  if (threadIdx.x == 0) atomicAdd(&zs_bk_stat[3], 1ull);
#endif
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
  BK_MARK(0);
  // exclusive scan: thread i owns words [WPT i, WPT i + WPT) (buckets 2 WPT i ...)
  {
    uint32_t sum = 0;
    for (uint32_t j = 0; j < ZS_BK_WPT; j++) {
      const uint32_t w = cnt[ZS_BK_WPT * tid + ((j + tid) & (ZS_BK_WPT - 1u))];  // rotated: threads hit different banks
      sum += (w & 0xffffu) + (w >> 16);
    }
    part[tid] = sum;
    __syncthreads();
    if (tid < 64) {  // scan of the partial sums, one wave
      uint32_t v[ZS_BK_PPL], t = 0;
#pragma unroll
      for (uint32_t j = 0; j < ZS_BK_PPL; j++) { v[j] = part[ZS_BK_PPL * tid + j]; t += v[j]; }
      uint32_t x = t;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (tid >= (uint32_t)d) x += y;
      }
      uint32_t run = x - t;
#pragma unroll
      for (uint32_t j = 0; j < ZS_BK_PPL; j++) { part[ZS_BK_PPL * tid + j] = run; run += v[j]; }
    }
    __syncthreads();
    uint32_t run = part[tid];
    for (uint32_t j = 0; j < ZS_BK_WPT; j++) {
      const uint32_t w = cnt[ZS_BK_WPT * tid + j];
      const uint32_t lo = w & 0xffffu;
      cnt[ZS_BK_WPT * tid + j] = run | ((run + lo) << 16);
      run += lo + (w >> 16);
    }
  }
  __syncthreads();
  BK_MARK(1);
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
        uint32_t a[ZS_BK_INFLIGHT], v[ZS_BK_INFLIGHT], sh[ZS_BK_INFLIGHT], e[ZS_BK_INFLIGHT], hh[ZS_BK_INFLIGHT];
#pragma unroll
        for (int j = 0; j < ZS_BK_INFLIGHT; j++) {
          const uint32_t p = g0 + 64 * j + lane;
          const uint32_t o = p - c0;
          const uint32_t h = sw_hash(__builtin_amdgcn_alignbyte(stg[(o >> 2) + 1], stg[o >> 2], o & 3u));
          hh[j] = h;
          sh[j] = 16u * (h & 1u);
          a[j] = sw_lds_addr(&cnt[h >> 1]);
          v[j] = p < c1 ? 1u << sh[j] : 0u;  // a lane past the chunk adds nothing
        }
        if (!ORD) {
          // order-independent: one add per distinct hash (its lowest lane), ranks by ballot
#pragma unroll
          for (int j = 0; j < ZS_BK_INFLIGHT; j++) {
            const uint32_t p = g0 + 64 * j + lane;
            const uint32_t h = hh[j];
            const uint64_t mm = zs_wave_match(h, p < c1);
            const uint32_t rank = (uint32_t)__builtin_popcountll(mm & ((1ull << lane) - 1ull));
            const uint32_t lead = mm ? (uint32_t)__builtin_ctzll(mm) : lane;
            uint32_t old = 0;
            if (p < c1 && lead == lane)
              old = atomicAdd(&cnt[h >> 1], (uint32_t)__builtin_popcountll(mm) << sh[j]);
            old = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead * 4u), (int)old);
            e[j] = old + (rank << sh[j]);
          }
        } else {
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
        }
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
  BK_MARK(2);
}
template __global__ void zs_k_bucket<true>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*,
                                           const zs_sweep_seg*, uint16_t*, uint2*);
template __global__ void zs_k_bucket<false>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*,
                                            const zs_sweep_seg*, uint16_t*, uint2*);

// --------------------------------------------------------------- zs_k_sweep
static __device__ __forceinline__ uint32_t sw_word(const uint32_t* win, uint32_t off) {
  const uint32_t i = off >> 2;
  return __builtin_amdgcn_alignbyte(win[i + 1], win[i], off & 3u);
}

// exact length of a candidate whose first `from` bytes match, clamped to maxc
static __device__ __forceinline__ uint32_t sw_extend(const uint32_t* win, uint32_t p, uint32_t q, uint32_t maxc,
                                                     uint32_t from) {
  uint32_t k = from;
  while (k < maxc) {
    const uint32_t y = sw_word(win, q + k) ^ sw_word(win, p + k);
    if (y) { k += (uint32_t)(__builtin_ctz(y) >> 3); break; }
    k += 4;
  }
  return k < maxc ? k : maxc;
}

// a wave-uniform 64-bit value kept in SGPRs (lane masks updated in loops with divergent bodies)
static __device__ __forceinline__ uint64_t sw_uniform(uint64_t x) {
  // (readfirstlane returns int: widen through uint32_t, not by sign extension)
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

static __device__ __forceinline__ uint32_t max3(uint32_t a, uint32_t b, uint32_t c) {
  return max(max(a, b), c);  // one v_max3_u32
}

// Candidate signatures.  A chain step compares the lane's own signature with a
// candidate's and yields the index of the first differing bit (the "matched
// bits"); its byte is the signature's matched-byte count sigma.
//
// SwSig<false>, any stream: the 11 bytes [q, q + 11) in three words.  A
// record's third word keeps bytes 8..10 (byte 11 zeroed) and the lane's own
// third word carries a sentinel bit 24, so the xor of the third words always
// has bit 24 set and the count saturates at 88 (all 11 bytes) by itself.
// sigma is the match length (>= 3 within a bucket unless the hash collides).
//
// SwSig<true>, streams whose bytes are all < 0x80 (text): two words, 8 bytes
// [X, b3 .. b9].  Bytes 0..2 hash to the bucket; of their 24 bits
// the 15-bit hash loses 9 -- b0[5:7], and b1[0:2], b1[5:7] (which the hash
// only has xor-ed with b2[5:7] and b0[0:2]) -- and with bit 7 of every byte
// clear, the 7 bits X = b0[5:6] | b1[0:2] << 2 | b1[5:6] << 5 recover them: in
// one bucket, equal X <=> equal first three bytes.  So sigma = 0 means "not a
// match" (a hash collision) and sigma >= 1 means a match of sigma + 2 bytes;
// the count saturates at 64 (min3 with 64).  A step is six VALU instead of
// nine.
static __device__ __forceinline__ uint32_t sw_x7(uint32_t w) {
  const uint32_t b0 = w & 0xffu, b1 = (w >> 8) & 0xffu;
  return ((b0 >> 5) & 3u) | ((b1 & 7u) << 2) | (((b1 >> 5) & 3u) << 5);
}
template <bool A7>
struct SwSig;
template <>
struct SwSig<false> {
  static constexpr uint32_t LONG = 88u;  // all 11 bytes: the exact length needs the window
  static constexpr uint32_t THR0 = 23u;  // sigma 2 (B << 3 | 7): no match yet
  static constexpr uint32_t EXT = 11u;   // a long candidate's known bytes
  uint32_t a, b, c;
  __device__ __forceinline__ void own(const uint32_t* win, uint32_t p) {
    a = sw_word(win, p);
    b = sw_word(win, p + 4);
    c = (sw_word(win, p + 8) & 0x00ffffffu) | 0x01000000u;
  }
  static __device__ __forceinline__ uint4 rec(const uint32_t* win, uint32_t q, uint32_t w0) {
    return make_uint4(w0, sw_word(win, q + 4), sw_word(win, q + 8) & 0x00ffffffu, 0u);
  }
  __device__ __forceinline__ uint32_t mbits(uint32_t x, uint32_t y, uint32_t z) const {
    uint32_t f0, f1, f2;
    asm("v_ffbl_b32 %0, %1" : "=v"(f0) : "v"(x ^ a));
    asm("v_ffbl_b32 %0, %1\n\tv_add_u32_e64 %0, %0, 32 clamp" : "=&v"(f1) : "v"(y ^ b));
    asm("v_ffbl_b32 %0, %1\n\tv_add_u32_e32 %0, 64, %0" : "=&v"(f2) : "v"(z ^ c));
    // ffbl(0) = ~0 and the clamped add keep "no difference" at ~0; f2 <= 88 (the sentinel)
    return min(min(f0, f1), f2);
  }
  static __device__ __forceinline__ uint32_t len(uint32_t sigma) { return sigma; }
};
template <>
struct SwSig<true> {
  static constexpr uint32_t LONG = 64u;  // all 8 signature bytes: a match of >= 10 bytes
  static constexpr uint32_t THR0 = 7u;   // sigma 0
  static constexpr uint32_t EXT = 10u;
  uint32_t a, b;
  __device__ __forceinline__ void own(const uint32_t* win, uint32_t p) {
    a = sw_x7(sw_word(win, p)) | (sw_word(win, p + 3) << 8);
    b = sw_word(win, p + 6);
  }
  // (the record's third word: the four bytes past the signature, which a long
  // candidate's first extension step compares -- from the ring, not the window)
  static __device__ __forceinline__ uint4 rec(const uint32_t* win, uint32_t q, uint32_t w0) {
    return make_uint4(sw_x7(w0) | (sw_word(win, q + 3) << 8), sw_word(win, q + 6), sw_word(win, q + EXT), 0u);
  }
  __device__ __forceinline__ uint32_t mbits(uint32_t x, uint32_t y, uint32_t) const {
    uint32_t f0, f1;
    asm("v_ffbl_b32 %0, %1" : "=v"(f0) : "v"(x ^ a));
    asm("v_ffbl_b32 %0, %1\n\tv_add_u32_e64 %0, %0, 32 clamp" : "=&v"(f1) : "v"(y ^ b));
    return min(min(f0, f1), 64u);  // one v_min3_u32
  }
  static __device__ __forceinline__ uint32_t len(uint32_t sigma) { return sigma ? sigma + 2u : 2u; }
};

// Per-wave ring of candidate records, as separate dense arrays so that the 64
// lanes of a step read 64 consecutive elements (conflict-free): signature words
// 0..1 (8 B), word 2 (the 11-byte form only) and the liveness key
// hash << 16 | q.  Member j's record lives in slot j mod 128 and again 128
// slots later, so that a block's 64 steps read slots base .. base + 63 without
// wrapping.
struct SwRing {
  uint2 ab[2 * ZS_SW_RING];
  uint32_t c[2 * ZS_SW_RING];
  uint32_t key[2 * ZS_SW_RING];
};

// The lock-step sweep of one stream (the workgroup), for signature form A7.
//
// For chain step t every lane compares its position with the t-th
// predecessor's signature.  A step's score is its matched bits with the low
// three bits (the bit within the first differing byte, which must not count)
// replaced by 7 - u, u = the step's place in its GROUP of steps (8, or 4 where
// a block end or the chain >> 2 snapshot cuts it): one v_and_or.  The group's
// maximum score is then its longest candidate and, among equally long ones,
// the earliest -- the first maximum of deflate.ts:1100-1105 -- and the lane
// keeps it when it is longer than its best so far (thr = B << 3 | 7 for a best
// of B signature bytes).  A step costs the compare and the v_and_or; the
// group's fold is max3s + a compare + three selects.
//
// A candidate whose whole signature matches is "long": its exact length needs
// the window.  Such candidates are rare; when a group holds one for any lane,
// those lanes extend it on the spot (the record's position is in the ring),
// keeping the first longest and stopping at the first nice match
// (deflate.ts:1100-1105).  Long candidates beat every short one.
//
// Liveness (deflate.ts:1109, 1376) is monotone in t, so a block of 64 steps in
// which every live lane's LAST step is live is live throughout for those lanes:
// such a block runs with the exec mask of the live lanes and no per-step test.
// A block in which some lane's chain ends runs the masked form (the step's
// ballot of `key > klim` ands into the live mask, a dead lane's score is 0).
#if ZS_SW_EXP & 64  // instrumentation (timing experiments only)
__device__ unsigned long long zs_sw_stat[8];  // chunks, fast groups, masked groups, long branches, wave steps
#define SW_STAT(i, v) do { if ((threadIdx.x & 63u) == __builtin_ctzll(__builtin_amdgcn_read_exec())) atomicAdd(&zs_sw_stat[i], (unsigned long long)(v)); } while (0)
extern "C" int zs_sw_stats(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_sw_stat), sizeof(zs_sw_stat));
}
#else
#define SW_STAT(i, v) do { } while (0)
#endif

template <bool A7, bool MW>
static __device__ __forceinline__ void sw_body(const uint32_t* win, SwRing* R, uint16_t* mw, uint32_t* next,
                                               uint32_t n, uint32_t m, uint32_t olo, uint32_t ohi,
                                               const uint16_t* mem, uint2* out, int chain, int nice_cfg) {
  // n: bytes from the window's start to the stream's end; m: the window's
  // members (inserted positions); results for the own positions [olo, ohi)
  using Sig = SwSig<A7>;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t budget = (uint32_t)chain, budget_s = (uint32_t)chain >> 2;
  // the steps swept: the full chain (a demand-driven variant that swept chain >> 2
  // steps and left the rest to the parse lost: DESIGN 4.2, tools/variants/r05_paths.patch)
#if ZS_SW_EXP & 128
  const uint32_t sbud = 4u;  // (timing: the per-chunk cost without chain steps past 4)
#else
  const uint32_t sbud = budget;
#endif
  const uint32_t nchunks = (m + 63) / 64;
  auto put_rec = [&](int j, uint4 r) {
    const uint32_t i = (uint32_t)j & (ZS_SW_RING - 1);
    R->ab[i] = make_uint2(r.x, r.y);
    R->ab[i + ZS_SW_RING] = make_uint2(r.x, r.y);
    R->c[i] = r.z;  // (A7: the bytes past the signature)
    R->c[i + ZS_SW_RING] = r.z;
    R->key[i] = r.w;
    R->key[i + ZS_SW_RING] = r.w;
  };
  auto make_rec = [&](uint32_t q) -> uint4 {
    const uint32_t w0 = sw_word(win, q);
    uint4 r = Sig::rec(win, q, w0);
    r.w = (sw_hash(w0) << 16) | q;
    return r;
  };
  // MW: the members k0 - budget .. k0 + 63 of the current chunk are kept in a
  // per-wave LDS window as their records are built, so the distances after
  // the sweep read positions from LDS instead of HBM (chain + 64 <= ZS_SW_MW)
  int mw0 = 0;  // member index of mw[0] (k0 - budget)
  auto load_rec_q = [&](int j, uint32_t q) {  // key 0 = no member: fails every liveness test
    const bool in = j >= 0 && (uint32_t)j < m;
    if (MW && (uint32_t)(j - mw0) < ZS_SW_MW) mw[j - mw0] = (uint16_t)q;  // (block 1 back reaches below k0 - budget when budget < 64)
    put_rec(j, in ? make_rec(q) : make_uint4(0, 0, 0, 0));
  };
  auto fetch = [&](int j) -> uint32_t { return j >= 0 && (uint32_t)j < m ? (uint32_t)mem[j] : 0u; };
  auto load_rec = [&](int j) { load_rec_q(j, fetch(j)); };
  auto member = [&](int j) -> uint32_t { return MW ? (uint32_t)mw[j - mw0] : (uint32_t)mem[j]; };
  auto rmbits = [&](const Sig& S, uint32_t slot) -> uint32_t {  // a ring record's matched bits
    const uint2 ab = R->ab[slot];
    return S.mbits(ab.x, ab.y, A7 ? 0u : R->c[slot]);
  };
  // chunks are claimed one ahead: the next chunk's members (its own and the
  // block before) are loaded while this one is swept
  auto claim = [&]() -> uint32_t {
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(next, 1u);
    return __builtin_amdgcn_readfirstlane(c);
  };
  uint32_t c = claim();
  uint32_t pf_p = fetch((int)(64 * c + lane)), pf_b = fetch((int)(64 * c + lane) - 64);
  for (;;) {
    if (c >= nchunks) break;
    const uint32_t cn = claim();
    const int k0 = (int)(64 * c);
    const int k = k0 + (int)lane;
    const bool mem_ok = (uint32_t)k < m;
    SW_STAT(0, 1);
    const uint32_t p = pf_p, qb = pf_b;  // (0 past the members)
    if (cn < nchunks) {
      pf_p = fetch((int)(64 * cn + lane));
      pf_b = fetch((int)(64 * cn + lane) - 64);
    }
    c = cn;
    // the lane's position is one of the window's own (a later window of a long
    // stream: its first 32,768 positions are look-back, candidates only)
    const bool own = mem_ok && p >= olo && p < ohi;
    if (__builtin_amdgcn_ballot_w64(own) == 0) continue;
    mw0 = k0 - (int)sbud;
    if (MW) mw[k - mw0] = (uint16_t)p;
    Sig S;
    S.own(win, p);
    const uint32_t h = sw_hash(sw_word(win, p));
    const uint32_t look = n - p;
    const uint32_t maxc = look < ZS_MAX_MATCH ? look : ZS_MAX_MATCH;                 // deflate.ts:1068
    const uint32_t nice = look < (uint32_t)nice_cfg ? look : (uint32_t)nice_cfg;      // deflate.ts:1078-1080
    const bool tail = maxc <= 12u;  // exact re-walk after the sweep
    const uint32_t long_m = tail ? 0xffffu : Sig::LONG;  // a tail lane records no long candidates
    const uint32_t limit = p > ZS_MAX_DIST ? p - ZS_MAX_DIST : 0u;                   // deflate.ts:1060
    const uint32_t khead = (h << 16) | (limit > 1u ? limit : 1u);
    const uint32_t klim = (h << 16) | limit;
    // ring: this chunk's block and the one before it
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    put_rec(k, mem_ok ? make_rec(p) : make_uint4(0, 0, 0, 0));
#if ZS_SW_EXP & 256
    put_rec(k - 64, make_uint4(qb, qb, qb, 0));  // (timing: the block before without its window reads)
#else
    load_rec_q(k - 64, qb);
#endif
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();

    // the best short candidate: its group's maximum score (matched bits, 7 - its place in the group) and the
    // group's first step (0: none) -- the step itself, t0 + 7 - (score & 7), is formed once at the end
    uint32_t thr = Sig::THR0, thr_s = Sig::THR0;
    uint32_t bt = 0, bt_s = 0;
    // best long candidate: its length (capped at nice) as lthr = len << 3 | 7, its step
    uint32_t lthr = 7u, lbt = 0, lthr_s = 7u, lbt_s = 0;
    const uint32_t own_ext = sw_word(win, p + Sig::EXT);  // the lane's bytes past a full signature
    uint64_t alive_m = 0;
    uint32_t head = 0;  // bit 0: head candidate valid; 0x8000: at exactly MAX_DIST
    // step t of block 0's numbering reads ring slot base - t
    auto score = [&](uint32_t mb, uint32_t u) -> uint32_t { return (mb & ~7u) | (7u - u); };  // one v_and_or_b32
    // a group's fold: the longest candidate if longer than the best so far.
    // Long candidates (a full signature match) are rare: when a group holds one
    // for any lane, those lanes compare the next four bytes of all the group's
    // long candidates at once (their positions are in the ring), a candidate
    // matching those too is extended byte-wise (rarer still).  Lengths are
    // capped at nice: the first nice candidate ends the walk (deflate.ts:1103)
    // and ties with every later one, so it stays first.
    auto fold = [&](uint32_t gm, uint32_t t0, const uint32_t* sc, uint32_t cnt, uint32_t base)
        __attribute__((always_inline)) {
#if ZS_SW_EXP & 4096  // (A/B: the step formed per group)
      const bool up = gm > thr;
      thr = max(thr, gm | 7u);
      bt = up ? t0 + 7u - (gm & 7u) : bt;
#else
      const bool up = gm > (thr | 7u);  // longer than the best so far
      thr = up ? gm : thr;
      bt = up ? t0 : bt;
#endif
#if ZS_SW_EXP & 32
      if (0) {
#else
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(gm >= long_m) != 0, 0)) {
#endif
        SW_STAT(3, 1);
        if (gm >= long_m && (lthr >> 3) < nice) {
          uint32_t gl = 0;
#if ZS_SW_EXP & 1024
#pragma unroll
          for (uint32_t u = 0; u < 8; u++) {
            if (u < cnt && sc[u] >= long_m) {
#else
          // the group's long steps as a mask, visited one by one (one to three per lane, typically)
          uint32_t lm = 0;
#pragma unroll
          for (uint32_t u = 0; u < 8; u++) lm |= (u < cnt && sc[u] >= long_m) ? 1u << u : 0u;
          while (lm) {
            const uint32_t u = (uint32_t)__builtin_ctz(lm);
            lm &= lm - 1u;
            {
#endif
              // the next four bytes: A7 records carry them (c), else from the window
              const uint32_t x = (A7 ? R->c[base - t0 - u]
                                     : sw_word(win, (R->key[base - t0 - u] & 0xffffu) + Sig::EXT)) ^ own_ext;
              uint32_t len = x ? Sig::EXT + ((uint32_t)__builtin_ctz(x) >> 3)
                               : sw_extend(win, p, R->key[base - t0 - u] & 0xffffu, maxc, Sig::EXT + 4u);
              len = min(min(len, maxc), nice);
              gl = max(gl, (len << 3) | (7u - u));
            }
          }
          const bool lup = gl > lthr;
          lthr = max(lthr, gl | 7u);
          lbt = lup ? t0 + 7u - (gl & 7u) : lbt;
        }
      }
    };
    bool snapped = budget_s <= 1u;  // wave-uniform: step chain >> 2 has been folded
    auto snap = [&](uint32_t t1) __attribute__((always_inline)) {
      if (t1 == budget_s) {  // the chain >> 2 result (deflate.ts:1075-1077)
        thr_s = thr;
        bt_s = bt;
        lthr_s = lthr;
        lbt_s = lbt;
        snapped = true;
      }
    };
    const uint32_t base0 = (((uint32_t)(k - 64)) & (ZS_SW_RING - 1)) + 64u;  // block 0: step t at slot base0 - t
    // t = 1: the head candidate (deflate.ts:1376)
    {
      const uint32_t key = R->key[base0 - 1u];
      bool a1 = false;
      uint32_t sc[1] = {0};
      if (own && key >= khead) {
        a1 = true;
        head = 1u | ((p - (key & 0xffffu)) == ZS_MAX_DIST ? 0x8000u : 0u);
        sc[0] = score(rmbits(S, base0 - 1u), 0);
      }
      alive_m = __builtin_amdgcn_ballot_w64(a1);
      fold(sc[0], 1u, sc, 1u, base0);
      snap(1u);
    }
    // masked step (blocks in which a chain ends): 0 for a lane whose chain ended
    // masked step (groups in which a chain ends): liveness is monotone in t
    // (keys fall with the member index), so a step is live iff its own key is
    // (and the lane was live when the group began); lm = the live lanes
    auto mstep = [&](uint32_t slot, uint32_t u, uint64_t& lm) -> uint32_t {
      const uint32_t key = R->key[slot];
      asm("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(lm) : "v"(key), "v"(klim));
      lm &= alive_m;
      const uint32_t v = score(rmbits(S, slot), u);
      uint32_t r;
      asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(v), "s"(lm));
      return r;
    };
    // steps 2..4 (masked)
    if (sbud >= 4u) {
      uint32_t sc[3];
      uint64_t lm = 0;
#pragma unroll
      for (uint32_t u = 0; u < 3; u++) sc[u] = mstep(base0 - 2u - u, u, lm);
      alive_m = sw_uniform(lm);  // the lanes live at step 4
      fold(max3(sc[0], sc[1], sc[2]), 2u, sc, 3u, base0);
      snap(4u);
    }
    // Steps [ta, tb] of block b (ta = 1 mod 4, tb = 0 mod 4, wave-uniform):
    // step t reads slot base - t, one address per group, immediate offsets inside.
    // (every lane runs it -- no divergent region, whose join costs register moves --
    // and a lane whose chain has ended folds nothing)
    auto group_fast = [&](uint32_t base, uint32_t t0, auto G, bool live) __attribute__((always_inline)) {
      constexpr uint32_t N = decltype(G)::value;
      // from the group's lowest slot up: one address, immediate offsets
      const uint32_t lo = base - t0 - (N - 1u);
      const uint2* const A = R->ab + lo;
      const uint32_t* const C = R->c + lo;
      uint32_t sc[N];
#pragma unroll
      for (uint32_t u = 0; u < N; u++) {
        const uint2 ab = A[N - 1u - u];
        sc[u] = score(S.mbits(ab.x, ab.y, A7 ? 0u : C[N - 1u - u]), u);
      }
      uint32_t gm;
      if constexpr (N == 8)
        gm = max(max3(sc[0], sc[1], sc[2]), max3(sc[3], sc[4], max3(sc[5], sc[6], sc[7])));
      else
        gm = max3(sc[0], sc[1], max(sc[2], sc[3]));
      fold(live ? gm : 0u, t0, sc, N, base);
    };
    // (like group_fast: one address, immediate offsets, every load issued before the first is waited for)
    auto group_masked = [&](uint32_t base, uint32_t t0, auto G) __attribute__((always_inline)) {
      constexpr uint32_t N = decltype(G)::value;
#if ZS_SW_EXP & 8192  // (A/B: step by step, an address and a wait each)
      uint32_t sc[8];
      uint64_t lm = 0, last = 0;
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) {
        sc[u] = 0u;
        if (u < N) {
          sc[u] = mstep(base - t0 - u, u, lm);
          last = lm;
        }
      }
      alive_m = sw_uniform(last);  // the lanes live at the group's last step
      fold(max(max3(sc[0], sc[1], sc[2]), max3(sc[3], sc[4], max3(sc[5], sc[6], sc[7]))), t0, sc, N, base);
#else
      const uint32_t lo = base - t0 - (N - 1u);
      const uint2* const A = R->ab + lo;
      const uint32_t* const C = R->c + lo;
      const uint32_t* const K = R->key + lo;
      uint32_t sc[N], key[N];
      uint2 ab[N];
#pragma unroll
      for (uint32_t u = 0; u < N; u++) {
        key[u] = K[N - 1u - u];
        ab[u] = A[N - 1u - u];
      }
      uint64_t lm = 0;
#pragma unroll
      for (uint32_t u = 0; u < N; u++) {
        asm("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(lm) : "v"(key[u]), "v"(klim));
        lm &= alive_m;
        const uint32_t v = score(S.mbits(ab[u].x, ab[u].y, A7 ? 0u : C[N - 1u - u]), u);
        asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(sc[u]) : "v"(v), "s"(lm));
      }
      alive_m = sw_uniform(lm);  // the lanes live at the group's last step
      uint32_t gm;
      if constexpr (N == 8)
        gm = max(max3(sc[0], sc[1], sc[2]), max3(sc[3], sc[4], max3(sc[5], sc[6], sc[7])));
      else
        gm = max3(sc[0], sc[1], max(sc[2], sc[3]));
      fold(gm, t0, sc, N, base);
#endif
    };
    using G8 = std::integral_constant<uint32_t, 8>;
    using G4 = std::integral_constant<uint32_t, 4>;
    // Steps [ta, tb] of a block in groups of 8 (4 where the range or the
    // snapshot cuts them).  A group in which every live lane is still live at
    // its last step runs unmasked with the exec mask of the live lanes;
    // otherwise masked.
    auto run = [&](uint32_t base, uint32_t ta, uint32_t tb) __attribute__((always_inline)) {
#if !(ZS_SW_EXP & 16384)
      // the next group's last key is read with this group's records: the fast-or-masked test waits on no load
      auto last_of = [&](uint32_t t0) __attribute__((always_inline)) {
        uint32_t t1 = t0 + 7u <= tb ? t0 + 7u : t0 + 3u;
        if (t0 <= budget_s && t1 > budget_s) t1 = budget_s;
        return t1;
      };
      if (ta > tb) return;
      uint32_t t0 = ta, t1 = last_of(ta);
      uint32_t kl = R->key[base - t1];
      while (alive_m) {
        const bool mine = ((alive_m >> lane) & 1u) != 0;
        const uint64_t last_live = __builtin_amdgcn_ballot_w64(mine && kl > klim);
        const uint32_t n0 = t1 + 1u, n1 = n0 <= tb ? last_of(n0) : t1;
        kl = R->key[base - n1];
        if (last_live == alive_m) {
          SW_STAT(1, 1);
          SW_STAT(4, t1 - t0 + 1u);
          if (t1 - t0 == 7u) group_fast(base, t0, G8{}, mine);
          else group_fast(base, t0, G4{}, mine);
        } else {
          SW_STAT(2, 1);
          SW_STAT(4, t1 - t0 + 1u);
          if (t1 - t0 == 7u) group_masked(base, t0, G8{});
          else group_masked(base, t0, G4{});
        }
        snap(t1);
        if (n0 > tb) break;
        t0 = n0;
        t1 = n1;
      }
#else
      for (uint32_t t0 = ta; t0 <= tb && alive_m;) {
        uint32_t t1 = t0 + 7u <= tb ? t0 + 7u : t0 + 3u;
        if (t0 <= budget_s && t1 > budget_s) t1 = budget_s;
        const bool mine = ((alive_m >> lane) & 1u) != 0;
        const uint64_t last_live = __builtin_amdgcn_ballot_w64(mine && R->key[base - t1] > klim);
#if ZS_SW_EXP & 4
        if (0) {
#elif ZS_SW_EXP & 16
        if (1) {
#else
        if (last_live == alive_m) {
#endif
          SW_STAT(1, 1);
          SW_STAT(4, t1 - t0 + 1u);
          if (t1 - t0 == 7u) group_fast(base, t0, G8{}, mine);
          else group_fast(base, t0, G4{}, mine);
        } else {
          SW_STAT(2, 1);
          SW_STAT(4, t1 - t0 + 1u);
          if (t1 - t0 == 7u) group_masked(base, t0, G8{});
          else group_masked(base, t0, G4{});
        }
        snap(t1);  // (every lane: one whose chain ended has its final best already)
        t0 = t1 + 1u;
      }
#endif
    };
    for (uint32_t b = 0; sbud > 4u && alive_m; b++) {
      // block b = steps (64b, 64b + 64]: members k0 - 64b - 64 ... k0 - 64b + 62, i.e. the blocks b and b + 1 back
      if (b >= 1) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        load_rec(k - 64 * (int)(b + 1));
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
      const uint32_t ta = b == 0 ? 5u : 64u * b + 1u;
      const uint32_t tb = min(64u * b + 64u, sbud);
      // step t of this block at slot base - t
      const uint32_t base = (((uint32_t)(k - 64 * (int)b - 64)) & (ZS_SW_RING - 1)) + 64u * b + 64u;
      run(base, ta, tb);
      if (tb >= sbud) break;
    }
    if (!snapped) {  // every chain ended before step chain >> 2
      thr_s = thr;
      bt_s = bt;
      lthr_s = lthr;
      lbt_s = lbt;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if (own) {
      uint32_t rx = 0, ry = 0;
      if (head) {
        uint32_t L = 2, D = 0, Ls = 2, Ds = 0;
        if (tail) {  // maxc <= 12: min(lcp, maxc) exactly, first maximum in chain order (deflate.ts:1082-1105)
          uint32_t b = 2u << 16, bs = 2u << 16;
          for (uint32_t t = 1; t <= budget && (int)t <= k; t++) {
            const uint32_t q = t <= sbud ? member(k - (int)t) : (uint32_t)mem[k - (int)t];
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
          L = b >> 16;
          D = L > 2u ? p - (uint32_t)mem[k - (int)(0xffffu - (b & 0xffffu))] : 0u;
          Ls = bs >> 16;
          Ds = Ls > 2u ? p - (uint32_t)mem[k - (int)(0xffffu - (bs & 0xffffu))] : 0u;
        } else {
#if ZS_SW_EXP & 4096
          const uint32_t tb = bt, tb_s = bt_s;
#else
          const uint32_t tb = bt + 7u - (thr & 7u), tb_s = bt_s + 7u - (thr_s & 7u);  // the steps
#endif
          if (bt) {
            L = Sig::len(thr >> 3);
            D = p - member(k - (int)tb);
          }
          if (bt_s) {
            Ls = Sig::len(thr_s >> 3);
            Ds = tb_s == tb ? D : p - member(k - (int)tb_s);
          }
          // long candidates beat every short one; a nice one's length was capped: measure it
          auto long_of = [&](uint32_t lt, uint32_t t, uint32_t& len, uint32_t& dist) {
            const uint32_t q = member(k - (int)t);
            len = lt >> 3;
            if (len >= nice) len = sw_extend(win, p, q, maxc, Sig::EXT);
            dist = p - q;
          };
          if (lbt) long_of(lthr, lbt, L, D);
          if (lbt_s) {
            if (lbt_s == lbt) {
              Ls = L;
              Ds = D;
            } else {
              long_of(lthr_s, lbt_s, Ls, Ds);
            }
          }
        }
        rx = (L << 16) | (L > 2u ? D : 0u) | (head & 0x8000u);
        ry = (Ls << 16) | (Ls > 2u ? Ds : 0u);
      }
#if ZS_SW_EXP & 512
      if (rx == 0x12345678u) out[p] = make_uint2(rx, ry);  // (timing: without the result stores)
#else
      out[p] = make_uint2(rx, ry);
#endif
    }
  }
}

__global__ __launch_bounds__(1024) void zs_k_sweep(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len,
                                                   const uint64_t* __restrict__ pos_base,
                                                   const zs_sweep_seg* __restrict__ segs,
                                                   const uint16_t* __restrict__ members, uint2* __restrict__ mres,
                                                   int chain, int nice_cfg) {
  __shared__ __attribute__((aligned(16))) SwRing ring[16];
  __shared__ __attribute__((aligned(16))) uint32_t win[ZS_SW_WIN_WORDS];
  __shared__ uint16_t mwin[16][ZS_SW_MW];
  __shared__ uint32_t next;
  const zs_sweep_seg G = segs[blockIdx.x];
  const int s = (int)G.s;
  const uint32_t n = in_len[s] - G.base;  // bytes from the window's start to the stream's end
  if (n < 3) return;
  const uint32_t m = min(n - 2, G.ohi);
  const uint8_t* src = in + in_off[s] + G.base;
  // the window in LDS, zero padded past the stream's end (reads run up to 16
  // bytes past a longest match); the OR of its bytes' top bits picks the
  // signature form
  uint32_t hi = 0;
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
      hi |= v.x | v.y | v.z | v.w;
      if (4 * i + 3 < ZS_SW_WIN_WORDS) *(uint4*)(win + 4 * i) = v;
      else for (uint32_t k = 0; 4 * i + k < ZS_SW_WIN_WORDS; k++) win[4 * i + k] = (&v.x)[k];
    }
  } else {
    for (uint32_t i = threadIdx.x; i < ZS_SW_WIN_WORDS; i += 1024) {
      uint32_t v = 0;
      for (uint32_t k = 0; k < 4; k++)
        if (4 * i + k < n) v |= (uint32_t)src[4 * i + k] << (8 * k);
      hi |= v;
      win[i] = v;
    }
  }
  if (threadIdx.x == 0) next = 0;
  const bool a7 = !__syncthreads_or((hi & 0x80808080u) != 0);
  SwRing* const R = &ring[threadIdx.x >> 6];
  const uint16_t* mem = members + G.mb;
  uint2* out = mres + pos_base[s] + G.base;
  uint16_t* const mw = mwin[threadIdx.x >> 6];
  const uint32_t olo = G.olo, ohi = G.ohi;
  if (chain + 64 <= (int)ZS_SW_MW) {
    if (a7) sw_body<true, true>(win, R, mw, &next, n, m, olo, ohi, mem, out, chain, nice_cfg);
    else sw_body<false, true>(win, R, mw, &next, n, m, olo, ohi, mem, out, chain, nice_cfg);
  } else {  // levels 8, 9: positions from HBM
    if (a7) sw_body<true, false>(win, R, mw, &next, n, m, olo, ohi, mem, out, chain, nice_cfg);
    else sw_body<false, false>(win, R, mw, &next, n, m, olo, ohi, mem, out, chain, nice_cfg);
  }
}
