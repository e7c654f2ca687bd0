// zs_wave.h -- the wave-uniform bit reader shared by the wave-per-member inflate
// kernel (inflate_wave.hip) and the split decode of large members
// (inflate_split.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zs_inftab.h"
#include "zs_refcalls.h"

#ifndef ZS_WIN_IN
#define ZS_WIN_IN 256u  // staged input words
#endif

static __device__ __forceinline__ uint32_t zs_u(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// wave-uniform bit reader: the zs_lane_reader scheme (clamped aligned words,
// one refill ahead) with every value in SGPRs.  The input words are staged in
// LDS, 1 KiB at a time by the whole wave: a refill is then an LDS read, which
// the table lookups' waits cover, where a direct load would wait behind the
// output stores (vmcnt) or -- as a scalar load -- make every table lookup's
// lgkmcnt wait for it.
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
