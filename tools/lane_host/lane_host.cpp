// Runs the lane-per-member inflate kernel (zlib-streams-ts_amd/csrc/inflate_lane.hip)
// on the CPU, one member at a time, from its own source (host stand-ins for the
// HIP names in hip/hip_runtime.h next to this file).  Test tooling: lets the CPU
// suite check the lane decoder's logic against the oracle without a GPU.
//
// The instances run on every member -- zs_k_inflate_lane<0, .> (canonical
// decode only), <1, .> (with the per-lane root tables) and <2, false> (root
// tables, canonical limits in LDS) -- and must agree.
// FLAGS bit 2 selects the large-member instances <., true> (the reference's
// inflate() calls tracked per lane, its window-wrap copy reproduced).
//
// usage: lane_host WBITS FLAGS < members > results
//   stdin:  u32 count, then per member: u32 in_len, u32 out_cap, in_len bytes
//   stdout: per member: u32 bail, u32 out_len, u32 consumed, u32 want, out_len bytes
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "hip/hip_runtime.h"
zs_dim3 threadIdx, blockIdx, blockDim;
#include "../../zlib-streams-ts_amd/csrc/inflate_lane.hip"
alignas(16) uint8_t LL[sizeof(zs_lane_lds_root)];

static void rd(void* p, size_t n) {
  if (fread(p, 1, n, stdin) != n) {
    fprintf(stderr, "lane_host: short input\n");
    exit(2);
  }
}
int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int wbits = atoi(argv[1]), flags = atoi(argv[2]);
  uint32_t n;
  rd(&n, 4);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t len, cap;
    rd(&len, 4);
    rd(&cap, 4);
    // 16-byte aligned buffers with slack, as device allocations are; the member
    // starts at a varying misalignment to exercise the reader's edges
    const uint32_t mis = i % 16;
    std::vector<uint4> ib((len + mis + 64) / 16 + 1), ob((cap + mis + 64) / 16 + 1);
    uint8_t* in = (uint8_t*)ib.data();
    rd(in + mis, len);
    uint64_t ioff = mis, ooff = ((i * 5) % 16) & ~3u;  // output offsets are 4-aligned (the C-ABI's contract)
    zs_lane_res r;
    uint32_t lo;
    threadIdx = {0, 0, 0};
    blockIdx = {0, 0, 0};
    blockDim = {1, 1, 1};
    std::vector<zs_lane_tabs> tabs(1);
    uint8_t* ob8 = (uint8_t*)ob.data();
    const size_t obn = ob.size() * sizeof(uint4);
    for (size_t k = 0; k < obn; k++) ob8[k] = 0xa5;  // guard pattern around the member's output
    const uint32_t zero = 0;
    const bool refw = (flags & 2) != 0;
    if (refw)
      zs_k_inflate_lane<2, true>(in, &ioff, &len, ob8, &ooff, &cap, wbits, 1, tabs.data(), &r, &lo, flags & 1, 0u,
                                    &zero);
    else
      zs_k_inflate_lane<1, false>(in, &ioff, &len, ob8, &ooff, &cap, wbits, 1, tabs.data(), &r, &lo, flags, 0u,
                                     nullptr);
    const std::vector<uint8_t> out_root(ob8, ob8 + obn);
    const zs_lane_res r_root = r;
    for (size_t k = 0; k < obn; k++) ob8[k] = 0xa5;
    if (refw)
      zs_k_inflate_lane<0, true>(in, &ioff, &len, ob8, &ooff, &cap, wbits, 1, tabs.data(), &r, &lo, flags & 1, 0u,
                                     &zero);
    else
      zs_k_inflate_lane<0, false>(in, &ioff, &len, ob8, &ooff, &cap, wbits, 1, tabs.data(), &r, &lo, flags, 0u,
                                      nullptr);
    if (r.bail != r_root.bail || (!r.bail && (r.out_len != r_root.out_len || r.consumed != r_root.consumed ||
                                              memcmp(ob8 + ooff, out_root.data() + ooff, r.out_len)))) {
      fprintf(stderr, "lane_host: member %u: root and canonical decoders differ\n", i);
      exit(4);
    }
    if (!refw) {  // the instance with the canonical limits in LDS too
      const std::vector<uint8_t> out_c(ob8, ob8 + obn);
      const zs_lane_res r_c = r;
      for (size_t k = 0; k < obn; k++) ob8[k] = 0xa5;
      zs_k_inflate_lane<2, false>(in, &ioff, &len, ob8, &ooff, &cap, wbits, 1, tabs.data(), &r, &lo, flags, 0u,
                                  nullptr);
      if (r.bail != r_c.bail || (!r.bail && (r.out_len != r_c.out_len || r.consumed != r_c.consumed ||
                                             memcmp(ob8, out_c.data(), obn)))) {
        fprintf(stderr, "lane_host: member %u: the LDS-canon instance differs\n", i);
        exit(4);
      }
    }
    for (size_t k = 0; k < obn; k++)
      if ((k < ooff || k >= ooff + cap) && ob8[k] != 0xa5) {
        fprintf(stderr, "lane_host: member %u wrote byte %zu outside [%lu, %lu)\n", i, k, (unsigned long)ooff,
                (unsigned long)(ooff + cap));
        exit(3);
      }
    fwrite(&r, 4, 4, stdout);
    fwrite((uint8_t*)ob.data() + ooff, 1, r.bail ? 0 : r.out_len, stdout);
  }
  return 0;
}
