// Probe: are same-address LDS atomic exchanges within ONE wave instruction
// applied in increasing lane order on gfx950?  For random keys per lane, each
// lane does old = atomicExch(&tab[key], lane + 1 + 64*round); lane-order
// semantics means old == (previous lower lane with the same key) or the value
// left by the previous round.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void probe(const uint32_t* keys, uint32_t* bad, int rounds) {
  __shared__ uint32_t tab[64];
  const uint32_t lane = threadIdx.x & 63;
  for (int i = lane; i < 64; i += 64) tab[i] = 0;
  __syncthreads();
  uint32_t errs = 0;
  __shared__ uint32_t last[64];
  if (lane < 64) last[lane] = 0;
  for (int r = 0; r < rounds; r++) {
    const uint32_t k = keys[(blockIdx.x * rounds + r) * 64 + lane] & 15;  // few keys -> many collisions
    const uint32_t val = 1 + lane + 64u * r;
    const uint32_t old = atomicExch(&tab[k], val);
    // expected: the highest lower lane with the same key in this round, else the table before the round
    uint32_t expect = 0xffffffffu;
    for (int l = (int)lane - 1; l >= 0; l--) {
      const uint32_t kl = keys[(blockIdx.x * rounds + r) * 64 + l] & 15;
      if (kl == k) { expect = 1 + l + 64u * r; break; }
    }
    if (expect == 0xffffffffu) expect = last[k];
    if (old != expect) errs++;
    __syncthreads();
    // last[k] = value of the highest lane with key k this round
    if (tab[k] == val) last[k] = val;
    __syncthreads();
  }
  atomicAdd(bad, errs);
}
int main() {
  const int blocks = 1024, rounds = 64;
  size_t nk = (size_t)blocks * rounds * 64;
  uint32_t* hk = (uint32_t*)malloc(nk * 4);
  srand(1);
  for (size_t i = 0; i < nk; i++) hk[i] = rand();
  uint32_t *dk, *db;
  hipMalloc(&dk, nk * 4); hipMalloc(&db, 4);
  hipMemcpy(dk, hk, nk * 4, hipMemcpyHostToDevice);
  hipMemset(db, 0, 4);
  probe<<<blocks, 64>>>(dk, db, rounds);
  uint32_t bad = 0;
  hipMemcpy(&bad, db, 4, hipMemcpyDeviceToHost);
  printf("lane-order violations: %u of %zu exchanges\n", bad, nk);
  return 0;
}
