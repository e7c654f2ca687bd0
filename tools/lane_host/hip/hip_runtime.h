// Host stand-in for the few HIP names inflate_lane.hip uses, so that the lane
// kernel's own source compiles as plain C++ and runs one lane at a time on the
// CPU (tools/lane_host/lane_host.cpp).  Test tooling only: the product is the
// gfx950 build of the same file.
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#define ZS_HOST_BUILD 1  // (zs_inftab.h: the wave-parallel table builder needs a real wave)
#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(x)
#define __shared__
struct uint4 {
  uint32_t x, y, z, w;
};
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
struct zs_dim3 {
  uint32_t x, y, z;
};
extern zs_dim3 threadIdx, blockIdx, blockDim;
using std::max;
using std::min;
static inline uint32_t zs_host_alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (s & 3u)));
}
#define __builtin_amdgcn_alignbyte(hi, lo, s) zs_host_alignbyte(hi, lo, s)
// one lane: a ballot is the lane's own bit, LDS atomics are plain read-modify-writes
#define __builtin_amdgcn_ballot_w64(c) ((c) ? 1ull : 0ull)
#define __builtin_amdgcn_readlane(v, l) (v)  // (one lane)
static inline uint32_t atomicAdd(uint32_t* p, uint32_t v) {
  const uint32_t o = *p;
  *p = o + v;
  return o;
}
static inline uint32_t atomicOr(uint32_t* p, uint32_t v) {
  const uint32_t o = *p;
  *p = o | v;
  return o;
}
#define ZS_OPAQUE(x) ((void)0)
#define ZS_LANE_WAVES(n)
typedef int hipError_t;
