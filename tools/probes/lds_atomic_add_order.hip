// Probe: are same-address LDS atomic adds (ds_add_rtn_u32) within ONE wave
// instruction applied in increasing lane order on gfx950?  Each lane does
// old = atomicAdd(&cnt[key], 1); lane order means old == count before the
// instruction + number of lower lanes with the same key.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void probe(const uint32_t* keys, uint32_t* bad, int rounds, uint32_t mask) {
  __shared__ uint32_t cnt[256];
  const uint32_t lane = threadIdx.x & 63;
  for (int i = lane; i < 256; i += 64) cnt[i] = 0;
  __syncthreads();
  uint32_t errs = 0;
  for (int r = 0; r < rounds; r++) {
    const uint32_t* kr = keys + (size_t)(blockIdx.x * rounds + r) * 64;
    const uint32_t k = kr[lane] & mask;
    const uint32_t before = cnt[k];
    __syncthreads();
    const uint32_t old = atomicAdd(&cnt[k], 1u);
    uint32_t lower = 0;
    for (uint32_t l = 0; l < lane; l++) lower += (kr[l] & mask) == k;
    if (old != before + lower) errs++;
    __syncthreads();
  }
  atomicAdd(bad, errs);
}
int main() {
  const int blocks = 2048, rounds = 64;
  size_t nk = (size_t)blocks * rounds * 64;
  uint32_t* hk = (uint32_t*)malloc(nk * 4);
  srand(7);
  for (size_t i = 0; i < nk; i++) hk[i] = rand();
  uint32_t *dk, *db;
  hipMalloc(&dk, nk * 4); hipMalloc(&db, 4);
  hipMemcpy(dk, hk, nk * 4, hipMemcpyHostToDevice);
  for (uint32_t mask : {0u, 3u, 15u, 255u}) {
    hipMemset(db, 0, 4);
    probe<<<blocks, 64>>>(dk, db, rounds, mask);
    uint32_t bad = 0;
    hipMemcpy(&bad, db, 4, hipMemcpyDeviceToHost);
    printf("key mask %3u: lane-order violations %u of %zu adds\n", mask, bad, nk);
  }
  return 0;
}
