// inflate_lane.hip -- the lane-per-member inflate path of zs_inflate_batch*
// (see the comment below); zs_k_inflate in inflate.hip is the exact path.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_inflate.h"
#include "zs_inftab.h"
#include "zs_refcalls.h"
#ifndef ZS_OPAQUE  // (the host stand-in of tools/lane_host defines these away)
#define ZS_OPAQUE(x) asm("" : "+v"(x))
#endif
#ifndef ZS_LANE_WAVES
#define ZS_LANE_WAVES(n) __attribute__((amdgpu_waves_per_eu(n)))
#endif
#ifndef ZS_IL_EXP
#define ZS_IL_EXP 0  // experiment builds (timing only; 0 in the product): 1 no stores, 2 no copy loads, 64 counters
#endif
#define IL_ST(x) do { if (!(ZS_IL_EXP & 1)) { x; } } while (0)
#if ZS_IL_EXP & 128  // per-member clock cycles, start and end (timing experiments)
__device__ unsigned long long zs_il_mcyc[2 * 65536];
extern "C" int zs_il_member_cycles(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_il_mcyc), sizeof(unsigned long long) * 2 * n);
}
#endif
#define IL_LD(x) ((ZS_IL_EXP & 2) ? 0u : (uint32_t)(x))

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
  uint16_t lens[320];  // the block's code lengths (lit/len then distance; the header's code-length code first)
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

// Canonical Huffman decoding (RFC 1951 3.2.2) with the code's shape in
// registers.  lim[l-1] is the end of the length-l codes left-justified to 15
// bits, so with the next 15 input bits read MSB first (rev), a code's length is
// one more than the number of limits <= rev, and its rank in (length, symbol)
// order is rev shifted down to that length plus D[length-1].  The symbols by
// rank are the only table, in LDS.  No memory access before the symbol itself
// and none in HBM: zlib's two-level tables (8-bit LDS roots before this) sent
// every code longer than the root to a second-level table in HBM, and some lane
// of a wave needed one in 68% of the C3 symbol steps -- a full memory latency
// for the whole wave each time.
struct zs_canon {
  uint32_t lim[15];
  uint32_t D[16];
};

// A lane's LDS: 548 B (a CU's 160 KB holds four 64-lane workgroups).
struct zs_lane_lds {
  uint32_t ring[32];  // the last 128 output bytes (zs_lane_out)
  uint8_t lsym[288];  // lit/len symbols by rank, low 8 bits
  uint32_t lhi[9];    // their bit 8, one bit per rank
  uint8_t dsym[32];   // distance symbols by rank (the header's code-length code first)
  uint32_t cnt[16];   // codes per length, then the next free rank of each length
};

// Narrow workgroups (lane_block <= 16: batches of a few thousand members) have
// LDS to spare: there each lane also keeps direct root tables -- 9-bit lit/len,
// 7-bit distance, u16 entries (length << 12 | symbol), 0 = a longer code -- so
// most codes cost one LDS read instead of the ~45-instruction compare chain;
// with few lanes per wave the VALU work per symbol is what each SIMD's lone
// wave waits on (C5-i: 8,192 members, eight lanes per wave).
#define ZS_LROOT 9u
#ifndef ZS_DROOT
#define ZS_DROOT 8u
#endif
struct zs_lane_lds_root {
  zs_lane_lds b;
  uint16_t lroot[1u << ZS_LROOT];
  uint16_t droot[1u << ZS_DROOT];
  // the canonical codes' limits too, for the LDS-canon instances (RT = 2; only
  // codes longer than the roots read them): out of registers the kernel needs
  // 68 VGPRs instead of 120 and leaves wave slots free on every SIMD, which the
  // large members' kernels of the same batch (side stream) run in
  __attribute__((aligned(16))) zs_canon cl;
  __attribute__((aligned(16))) zs_canon cd;
};

// C from lens[0..n) (the member's scratch in HBM); false unless the code is
// complete.  zlib's inflate_table rejects over-subscribed sets and incomplete
// ones but for a lone code of length 1 (inftrees.ts:128-139); a lane bails on
// every incomplete set and leaves that case to the exact path.
static __device__ bool zs_canon_build(zs_canon& C, uint32_t* cnt, uint8_t* sym8, uint32_t* hi, const uint16_t* lens,
                                      uint32_t n) {
#pragma unroll
  for (int l = 0; l < 16; l++) cnt[l] = 0;
  if (hi)
#pragma unroll
    for (int w = 0; w < 9; w++) hi[w] = 0;
#pragma unroll 8
  for (uint32_t i = 0; i < n; i++) atomicAdd(&cnt[lens[i]], 1u);
  uint32_t code = 0, rank = 0;
  int left = 1;
#pragma unroll
  for (int l = 1; l <= 15; l++) {
    const uint32_t c = cnt[l];
    left = 2 * left - (int)c;  // once negative (over-subscribed) it stays so
    C.lim[l - 1] = (code + c) << (15 - l);
    C.D[l - 1] = rank - code;
    cnt[l] = rank;
    rank += c;
    code = (code + c) << 1;
  }
  C.D[15] = 0;
  if (left != 0) return false;
#pragma unroll 8
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t l = lens[i];
    if (l) {
      const uint32_t k = atomicAdd(&cnt[l], 1u);
      sym8[k] = (uint8_t)i;
      if (hi && (i >> 8)) atomicOr(&hi[k >> 5], 1u << (k & 31u));
    }
  }
  return true;
}

// root[r] for every code of length <= rbits (after zs_canon_build: cnt[l] is
// the rank past the last length-l code, and a rank k of length l has code k - D[l-1])
static __device__ void zs_root_fill(uint16_t* root, uint32_t rbits, const zs_canon& C, const uint32_t* cnt,
                                    const uint8_t* sym8, const uint32_t* hi) {
  for (uint32_t k = 0; k < (1u << rbits) / 2u; k++) reinterpret_cast<uint32_t*>(root)[k] = 0;
  uint32_t k = 0;
#pragma unroll
  for (uint32_t l = 1; l <= ZS_LROOT; l++) {
    if (l > rbits) break;
    const uint32_t end = cnt[l];
    for (; k < end; k++) {
      const uint32_t code = k - C.D[l - 1];
      const uint32_t r = __builtin_bitreverse32(code) >> (32u - l);  // the stream sends codes MSB first
      const uint32_t sym = sym8[k] | (hi ? ((hi[k >> 5] >> (k & 31u)) & 1u) << 8 : 0u);
      for (uint32_t x = r; x < (1u << rbits); x += 1u << l) root[x] = (uint16_t)((l << 12) | sym);
    }
  }
}

// the rank of the code at the front of the bit buffer; L = its length (16: no
// such code -- the caller bails)
static __device__ __forceinline__ uint32_t zs_canon_rank(const zs_canon& C, const zs_lane_reader& R, uint32_t& L) {
  const uint32_t rev = __builtin_bitreverse32((uint32_t)R.hold) >> 17;
  // the values pass an empty asm so each select below is between registers (the
  // compiler otherwise selects an address into C and keeps C in scratch)
  uint32_t d[16];
#pragma unroll
  for (int l = 0; l < 16; l++) {
    d[l] = C.D[l];
    ZS_OPAQUE(d[l]);
  }
  uint32_t n = 1, D = d[0];
#pragma unroll
  for (int l = 0; l < 15; l++) {
    const bool c = rev >= C.lim[l];
    n += c;
    D = c ? d[l + 1] : D;
  }
  L = n;
  return (rev >> ((15u - n) & 31u)) + D;
}
// the same from a code kept in LDS: the limits in four 16-byte reads, then the
// one D[] entry of the code's length
static __device__ __forceinline__ uint32_t zs_canon_rank_lds(const zs_canon& C, const zs_lane_reader& R,
                                                             uint32_t& L) {
  const uint32_t rev = __builtin_bitreverse32((uint32_t)R.hold) >> 17;
  const uint4* l4 = reinterpret_cast<const uint4*>(C.lim);  // lim[0..14] (+ D[0], unused)
  const uint4 q0 = l4[0], q1 = l4[1], q2 = l4[2], q3 = l4[3];
  const uint32_t lim[15] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z};
  uint32_t n = 1;
#pragma unroll
  for (int l = 0; l < 15; l++) n += rev >= lim[l] ? 1u : 0u;
  L = n;
  return (rev >> ((15u - n) & 31u)) + C.D[(n - 1u) & 15u];
}
template <bool LDS>
static __device__ __forceinline__ uint32_t zs_canon_rank_t(const zs_canon& C, const zs_lane_reader& R, uint32_t& L) {
  if constexpr (LDS) return zs_canon_rank_lds(C, R, L);
  else return zs_canon_rank(C, R, L);
}
static __device__ __forceinline__ void zs_lr_drop(zs_lane_reader& R, uint32_t k) {
  R.hold >>= k;
  R.bits -= k;
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

// Output of one lane.  Bytes collect in cw (the word being filled) and each
// completed word goes to the lane's 128-byte ring in LDS; HBM sees whole
// 16-byte units, stored from the ring by flush() -- called for every lane of
// the wave at once when one of them holds 64 unstored bytes, so stores come in
// rare bursts.  (Every s_waitcnt on a load also waits for the wave's earlier
// stores; with a store in nearly every symbol step, the input refills and copy
// loads waited out store latencies: half of C3's time.)  The ring also serves
// every copy source up to ZS_RING_SRC bytes back.  P counts bytes from the
// unit-aligned base below the member's first byte (out_off is 4-aligned: the
// first unit is entered at word w0 and its earlier words -- another member's --
// are never stored); F is the start of the first unstored unit.  Writing the
// word at W overwrites the one at W - 128, so W - 124 <= F must hold: room()
// before a round of up to 16 bytes keeps P - F <= 108, and the partial word a
// sync() writes leaves [P - 124, P) readable.
#define ZS_RING 128u
#define ZS_RING_SRC 124u
struct zs_lane_out {
  uint32_t* base;  // 16-byte aligned, <= dst
  uint32_t* ring;  // LDS: output byte X at ring byte X % ZS_RING
  uint32_t P, F, w0, cw;
  __device__ __forceinline__ void init(uint8_t* dst, uint32_t* lds_ring) {
    const uintptr_t a = (uintptr_t)dst;
    // (pointer arithmetic, not an integer round trip: the compiler then knows base is global memory
    // and issues global loads / stores instead of flat ones, which also count against lgkmcnt)
    base = reinterpret_cast<uint32_t*>(dst - (a & 15u));
    ring = lds_ring;
    P = (uint32_t)(a & 15u);
    w0 = P >> 2;
    F = 0;
    cw = 0;
  }
  __device__ __forceinline__ uint32_t& slot(uint32_t x) { return ring[(x >> 2) & (ZS_RING / 4 - 1)]; }
  // n (1..4) bytes, the low bytes of v (bytes above n zero)
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    const uint32_t a = P & 3u;
    cw |= v << (8u * a);
    if (a + n >= 4u) {
      slot(P) = cw;
      cw = a ? v >> (32u - 8u * a) : 0u;  // the bytes past the word
    }
    P += n;
  }
  __device__ __forceinline__ void byte(uint32_t b) { put(b & 0xffu, 1u); }
  // the partial word into the ring too: the ring then holds every byte in [P - 124, P)
  __device__ __forceinline__ void sync() {
    if (P & 3u) slot(P) = cw;
  }
  // the complete units below P to HBM
  __device__ __forceinline__ void flush() {
    while (F + 16u <= P) {
      const uint32_t x0 = slot(F), x1 = slot(F + 4u), x2 = slot(F + 8u), x3 = slot(F + 12u);
      uint32_t* q = base + (F >> 2);
      if (F >= 16u || w0 == 0) {
        IL_ST(*reinterpret_cast<uint4*>(q) = make_uint4(x0, x1, x2, x3));
      } else {
        if (w0 <= 1) IL_ST(q[1] = x1);
        if (w0 <= 2) IL_ST(q[2] = x2);
        IL_ST(q[3] = x3);
      }
      F += 16u;
    }
  }
  // room for a round of up to 16 bytes
  __device__ __forceinline__ void room() {
    if (P - F > ZS_RING - 20u) flush();
  }
  // the member's last bytes (the last word's bytes past P are inside its capacity)
  __device__ __forceinline__ void finish() {
    sync();
    flush();
    uint32_t* q = base + (F >> 2);
    for (uint32_t i = 0; i < 4; i++)
      if (F + 4u * i < P && (F >= 16u || i >= w0)) IL_ST(q[i] = slot(F + 4u * i));
  }
  // 16 bytes from ring position x (any alignment; x + 16 <= P after a sync)
  __device__ __forceinline__ void ring16(uint32_t x, uint32_t (&w)[4]) {
    const uint32_t sh = x & 3u;
    uint32_t r[5];
#pragma unroll
    for (int k = 0; k < 5; k++) r[k] = slot(x + 4u * (uint32_t)k);
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = __builtin_amdgcn_alignbyte(r[k + 1], r[k], sh);
  }
  // up to 16 bytes of w (n of them)
  __device__ __forceinline__ void put16(const uint32_t (&w)[4], uint32_t n) {
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      if (n >= 4u * k + 4u) {
        put(w[k], 4u);
      } else if (n > 4u * k) {
        const uint32_t nb = n - 4u * k;
        put(w[k] & ((1u << (8u * nb)) - 1u), nb);
      }
    }
  }
};

#if ZS_IL_EXP & 64
// per wave (max over its lanes): symbol iterations, ones with a slow lit/len
// decode, a slow distance decode, a direct copy, a spilled copy; clock cycles in
// headers+tables, in symbols, in all
__device__ unsigned long long zs_il_stat[8];
extern "C" int zs_il_stats(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_il_stat), sizeof(zs_il_stat));
}
#define IL_ANY(c) ((__builtin_amdgcn_ballot_w64(c) != 0) ? 1ull : 0ull)
#define IL_FIRST() ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec()))
#define IL_T(v) const unsigned long long v = clock64()
#define IL_ACC(i, v) do { if (IL_FIRST()) st[i] += clock64() - v; } while (0)
#endif

// REFW: the large-member instance (launched over a list of members with more
// than inflate_wave_min input bytes): a deflate / zlib / gzip member at any
// size, the reference's inflate() calls tracked per lane (zs_refcalls) and
// their window-wrap copy reproduced -- what zs_k_inflate_wave does with a wave
// per member, here with a lane (many large members: the wave kernel's scalar
// bookkeeping shares one scalar unit per CU among its waves).
// RT: 0 no root tables (wide workgroups), 1 root tables, 2 root tables with
// the canonical limits in LDS too (batches with large members beside them)
template <int RT, bool REFW>
__global__ __launch_bounds__(64) ZS_LANE_WAVES(4) void zs_k_inflate_lane(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint32_t* __restrict__ out_cap, int wbits, uint32_t n_members,
                                                        zs_lane_tabs* __restrict__ tabs, zs_lane_res* __restrict__ res,
                                                        uint32_t* __restrict__ lens_out, int flags,
                                                        uint32_t wave_min, const uint32_t* __restrict__ list) {
  extern __shared__ __attribute__((aligned(16))) uint8_t LL[];  // blockDim.x lanes' tables
  constexpr bool ROOT = RT > 0, LCAN = RT == 2;
  constexpr uint32_t lstride = ROOT ? sizeof(zs_lane_lds_root) : sizeof(zs_lane_lds);
  const uint32_t li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= n_members) return;
  // REFW with a list: the large members; without one (retry mode): every member the
  // single-call instance bailed on that may be longer than one inflate() call of the
  // reference (a caller's cap past 64 KiB), except large ones.  A member that fails
  // for another reason fails here again and goes on to the exact path.
  const uint32_t s = REFW && list ? list[li] : li;
  // (members of 512 MB or more too: the bookkeeping's bit positions are 32-bit; the exact path takes them)
  if (REFW && !list &&
      (res[s].bail == 0 || out_cap[s] <= 65536u || zs_inf_large(in_len[s], out_cap[s], wave_min) ||
       in_len[s] >= (1u << 29)))
    return;
  // a large member: the REFW instance, zs_k_inflate_wave or the split path decodes it
  if (!REFW && zs_inf_large(in_len[s], out_cap[s], wave_min)) return;
  zs_lane_tabs& T = tabs[s];
  zs_lane_lds& F = *reinterpret_cast<zs_lane_lds*>(LL + threadIdx.x * lstride);
  uint16_t* const lroot = ROOT ? reinterpret_cast<zs_lane_lds_root*>(&F)->lroot : nullptr;
  uint16_t* const droot = ROOT ? reinterpret_cast<zs_lane_lds_root*>(&F)->droot : nullptr;
#if ZS_IL_EXP & 128
  if (s < 65536) zs_il_mcyc[2 * s] = wall_clock64();
#endif
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
#if ZS_IL_EXP & 64
  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long tk0 = clock64();
  unsigned long long tk = tk0;
#endif
  uint8_t* dst = out + out_off[s];
  zs_canon CLr, CDr;  // registers (wide workgroups); the root instance keeps them in LDS
  zs_canon& CL = *(LCAN ? &reinterpret_cast<zs_lane_lds_root*>(&F)->cl : &CLr);
  zs_canon& CD = *(LCAN ? &reinterpret_cast<zs_lane_lds_root*>(&F)->cd : &CDr);
  zs_lane_out W;
  W.init(dst, F.ring);
  // This path decodes a member in one go, without the stream layer's call
  // boundaries.  A member whose input fits one 32 KiB sub-chunk and whose
  // output fits one 64 KiB output buffer is decoded by ONE inflate() call of
  // the reference (streams.ts:6-7,78-93) that never copies from the window, so
  // the window-wrap behaviour (ZS_INF_REF_WRAP) cannot arise; any other member
  // takes the exact path, which emulates the calls.
  // deflate64 members never reach inflate_fast in the reference (inflate.ts:841),
  // so they carry no call-boundary behaviour and decode here at any size.
  const bool d64 = wbits == -16;
  const bool ref_wrap = (flags & ZS_INF_REF_WRAP) != 0 && !d64 && !REFW;
  const uint32_t cap = ref_wrap ? min(out_cap[s], 65536u) : out_cap[s];
  zs_refcalls_t<uint32_t> C;  // (the host routes members of under 512 MB here: bit positions fit 32 bits)
#if ZS_IL_EXP & 256  // timing experiments: the bookkeeping skipped (wrong bytes where the defect applies)
#define REFW_SYM(...) false
#else
#define REFW_SYM(...) C.symbol(__VA_ARGS__)
#endif
  C.init();
  const uint32_t lmask = d64 ? 31u : 15u;  // length extra-bit mask (inflate.ts:891)
  uint32_t total = 0;
  zs_lane_res r = {1u, 0u, 0u, 0u};
  const int wrap = wbits < 0 ? 0 : (wbits >> 4) + 5;  // inflate.ts:152-160
  bool bail = ref_wrap && R.n > 32768u;  // several sub-chunks: the call-tracking instance
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
    if (type == 0) {  // stored (inflate.ts:615-660)
      zs_lr_align(R);
      const uint32_t len = zs_lr_take(R, 16), nlen = zs_lr_take(R, 16);
      if (len != (nlen ^ 0xffffu) || zs_lr_over(R) || total + len > cap) { bail = true; break; }
      if (REFW) C.stored((uint32_t)(zs_lr_bitpos(R) >> 3), total, len);
      for (uint32_t i = 0; i < len; i++) {
        if (W.P - W.F > ZS_RING - 8u) W.flush();
        W.byte(zs_lr_take(R, 8));
      }
      total += len;
      if (zs_lr_over(R)) { bail = true; break; }
      continue;
    }
    uint32_t nlen, ndist;
    if (type == 1) {  // fixed codes (inflate.ts:218-280)
      nlen = 288;
      ndist = 32;
      for (uint32_t sym = 0; sym < 320; sym++)
        T.lens[sym] = sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : sym < 288 ? 8 : 5;
    } else if (type == 2) {  // dynamic (inflate.ts:662-836)
      nlen = zs_lr_take(R, 5) + 257;
      ndist = zs_lr_take(R, 5) + 1;
      const uint32_t ncode = zs_lr_take(R, 4) + 4;
      if (nlen > 286 || (!d64 && ndist > 30)) { bail = true; break; }
      uint32_t i;
      for (i = 0; i < ncode; i++) T.lens[ZS_BL_ORDER[i]] = (uint16_t)zs_lr_take(R, 3);
      for (; i < 19; i++) T.lens[ZS_BL_ORDER[i]] = 0;
      if (!zs_canon_build(CD, F.cnt, F.dsym, nullptr, T.lens, 19)) { bail = true; break; }
      i = 0;
      uint32_t prev = 0;
      while (i < nlen + ndist) {
        if (R.bits < 32) zs_lr_fill(R);
        uint32_t L;
        const uint32_t k = zs_canon_rank_t<LCAN>(CD, R, L);
        if (L > 15) { bail = true; break; }
        zs_lr_drop(R, L);
        const uint32_t v = F.dsym[k];
        if (v < 16) {
          T.lens[i++] = (uint16_t)v;
          prev = v;
          continue;
        }
        uint32_t rep, val = 0;
        if (v == 16) {
          if (i == 0) { bail = true; break; }
          val = prev;
          rep = 3 + zs_lr_take(R, 2);
        } else if (v == 17) {
          rep = 3 + zs_lr_take(R, 3);
        } else {
          rep = 11 + zs_lr_take(R, 7);
        }
        if (i + rep > nlen + ndist) { bail = true; break; }
        while (rep--) T.lens[i++] = (uint16_t)val;
        prev = val;
      }
      if (bail || zs_lr_over(R) || T.lens[256] == 0) { bail = true; break; }
    } else {
      bail = true;  // "invalid block type"
      break;
    }
    if (!zs_canon_build(CL, F.cnt, F.lsym, F.lhi, T.lens, nlen)) {
      bail = true;
      break;
    }
    if (ROOT) zs_root_fill(lroot, ZS_LROOT, CL, F.cnt, F.lsym, F.lhi);
    if (!zs_canon_build(CD, F.cnt, F.dsym, nullptr, T.lens + nlen, ndist)) {
      bail = true;
      break;
    }
    if (ROOT) zs_root_fill(droot, ZS_DROOT, CD, F.cnt, F.dsym, nullptr);
#if ZS_IL_EXP & 64
    { const unsigned long long t = clock64(); st[5] += t - tk; tk = t; }
#endif
    // symbols (inffast.ts:5-228 semantics, without the call boundaries)
    for (;;) {
      // stores in bursts: every lane flushes when one holds 64 unstored bytes
      if (__builtin_amdgcn_ballot_w64(W.P - W.F >= 64u)) {
#if ZS_IL_EXP & 64
        IL_T(tf);
#endif
        W.flush();
#if ZS_IL_EXP & 64
        IL_ACC(2, tf);
#endif
      }
      if (R.bits < 32) zs_lr_fill(R);
#if ZS_IL_EXP & 64
      st[0]++;
      st[1] += IL_FIRST();  // wave steps (summed)
#endif
      uint32_t L, k, sym;
      const uint32_t b0 = REFW ? R.pos * 8u - R.bits : 0u;  // the symbol's first bit (zs_refcalls)
      const uint32_t le = ROOT ? lroot[(uint32_t)R.hold & ((1u << ZS_LROOT) - 1u)] : 0u;
      if (le) {
        L = le >> 12;
        sym = le & 0x1ffu;
      } else {
        k = zs_canon_rank_t<LCAN>(CL, R, L);
        if (L > 15) { bail = true; break; }  // "invalid literal/length code"
        sym = F.lsym[k] | (((F.lhi[k >> 5] >> (k & 31u)) & 1u) << 8);
      }
      zs_lr_drop(R, L);
      const uint32_t l1 = L;
      if (sym >= 286) { bail = true; break; }  // fixed codes 286/287: "invalid literal/length code"
      zcode here = zs_lit_entry(sym, d64);
      uint32_t op = C_OP(here);
      if (op == 0) {
        if (total >= cap) { bail = true; break; }
        if (REFW) REFW_SYM(b0, total, 1u, l1, 0u, 0u, 0u, false);
        W.byte(C_VAL(here));
        total++;
        continue;
      }
      if (op & 32) {  // end of block
        if (REFW) REFW_SYM(b0, total, 0u, l1, 0u, 0u, 0u, true);
        break;
      }
      if (op & 64) { bail = true; break; }  // "invalid literal/length code"
      const uint32_t e1 = op & lmask;
      uint32_t len = C_VAL(here) + zs_lr_take(R, e1);
      if (R.bits < 32) zs_lr_fill(R);
      uint32_t dsym;
      const uint32_t de = ROOT ? droot[(uint32_t)R.hold & ((1u << ZS_DROOT) - 1u)] : 0u;
      if (de) {
        L = de >> 12;
        dsym = de & 0x1fu;
      } else {
        k = zs_canon_rank_t<LCAN>(CD, R, L);
        if (L > 15) { bail = true; break; }  // "invalid distance code"
        dsym = F.dsym[k];
      }
      zs_lr_drop(R, L);
      if (!d64 && dsym >= 30) { bail = true; break; }  // fixed codes 30/31 likewise
      here = zs_dist_entry(dsym, d64);
      op = C_OP(here);
      const uint32_t dist0 = C_VAL(here) + zs_lr_take(R, op & 15u);
      if (dist0 > total || total + len > cap) { bail = true; break; }  // too far back / capacity
      // REFW: a copy inflate_fast runs may end with the reference's window-wrap
      // copy -- its last `tail` bytes taken from the current call's first output
      // bytes (C.B on), i.e. a second copy at distance total + head - C.B
      uint32_t tail = 0;
      if (REFW && REFW_SYM(b0, total, len, l1, e1, L, op & 15u, false)) tail = C.wrap(total, len, dist0);
      const uint32_t len_all = len;
      for (uint32_t part = 0; part < (REFW ? 2u : 1u); part++) {
      const uint32_t dist = part == 0 ? dist0 : total - C.B;  // (total has moved past the head)
      if (part == 0) len -= tail;
      else len = tail;
      if (len == 0) continue;
      const uint32_t src = W.P - dist;
#if ZS_IL_EXP & 64
      IL_T(tc);
#endif
      if (dist > ZS_RING_SRC) {
        // older than the ring: in HBM (room() keeps P - F <= 108 before every
        // round, so the round's source lies below F), 16 bytes per round trip;
        // aligned words funnel-shifted into place
        const uint32_t fsh = src & 3u;
        const uint32_t* fw = W.base + (src >> 2);
        for (uint32_t i = 0; i < len; i += 16) {
          W.room();
          uint32_t x[5], w[4];
#pragma unroll
          for (int k = 0; k < 5; k++) x[k] = IL_LD(fw[(i >> 2) + (uint32_t)k]);
#pragma unroll
          for (int k = 0; k < 4; k++) w[k] = __builtin_amdgcn_alignbyte(x[k + 1], x[k], fsh);
          W.put16(w, min(16u, len - i));
        }
#if ZS_IL_EXP & 64
        IL_ACC(3, tc);
#endif
      } else if (dist >= 16) {  // from the ring, 16 bytes a round
        for (uint32_t i = 0; i < len; i += 16) {
          W.room();
          W.sync();
          uint32_t w[4];
          W.ring16(src + i, w);
          W.put16(w, min(16u, len - i));
        }
#if ZS_IL_EXP & 64
        IL_ACC(4, tc);
#endif
      } else {
        // overlapping (period dist < 16): a round copies the md bytes before P,
        // md a multiple of dist that doubles up to the largest one within 16
        const uint32_t mmax = (uint32_t)((0xedcba98fdbefeffull >> (4u * (dist - 1u))) & 15u) + 1u;
        uint32_t md = dist;
        for (uint32_t i = 0; i < len;) {
          W.room();
          W.sync();
          uint32_t w[4];
          W.ring16(W.P - md, w);
          const uint32_t n = min(md, len - i);
          W.put16(w, n);
          i += n;
          md = min(2u * md, mmax);
        }
#if ZS_IL_EXP & 64
        IL_ACC(5, tc);
#endif
      }
      total += len;
      }  // part
      (void)len_all;
    }
    if (zs_lr_over(R)) bail = true;
#if ZS_IL_EXP & 64
    { const unsigned long long t = clock64(); st[6] += t - tk; tk = t; }
#endif
  }
  if (!bail) W.finish();  // the last unit's bytes
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
#if ZS_IL_EXP & 128
  if (s < 65536) zs_il_mcyc[2 * s + 1] = wall_clock64();
#endif
  lens_out[s] = r.out_len;  // for the checksum pass over the decoded bytes
#if ZS_IL_EXP & 64
  st[7] = clock64() - tk0;
  for (int i = 0; i < 8; i++) {
    unsigned long long v = st[i];
    for (int o = 32; o; o >>= 1) {
      const unsigned long long w = __shfl_xor(v, o);
      v = (i >= 1 && i <= 5) ? v + w : w > v ? w : v;
    }
    if ((threadIdx.x & 63u) == 0) atomicAdd(&zs_il_stat[i], v);
  }
#endif
}

size_t zs_inflate_lane_scratch_bytes() { return sizeof(zs_lane_tabs); }
size_t zs_inflate_lane_lds_bytes(bool root) { return root ? sizeof(zs_lane_lds_root) : sizeof(zs_lane_lds); }

#define ZS_LANE_INST(R, W)                                                                                           \
  template __global__ void zs_k_inflate_lane<R, W>(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,       \
                                                   const uint64_t*, const uint32_t*, int, uint32_t, zs_lane_tabs*,    \
                                                   zs_lane_res*, uint32_t*, int, uint32_t, const uint32_t*);
ZS_LANE_INST(0, false)
ZS_LANE_INST(1, false)
ZS_LANE_INST(2, false)
ZS_LANE_INST(0, true)
ZS_LANE_INST(2, true)

