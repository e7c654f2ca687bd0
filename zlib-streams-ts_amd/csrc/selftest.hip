// selftest.hip -- run-time check of the one hardware property the chain
// builders (zs_k_prev, zs_k_bucket, zs_k_fast) rely on beyond the ISA manual:
// same-address LDS atomics (ds_wrxchg_rtn_b32, ds_mskor_rtn_b32 on 16-bit
// halves, and ds_add_rtn_u32 on whole words and on 16-bit halves) issued by
// ONE wave instruction are applied in increasing lane order on gfx950.  Probed
// off-line (tools/probes/lds_atomic_order.hip, lds_atomic_add_order.hip); the
// context re-checks it at creation so a part that behaves differently fails
// loudly instead of producing wrong hash chains.
#include <hip/hip_runtime.h>
#include <stdint.h>

// Keys come from a fixed xorshift sequence (many same-key lanes per instruction).
static __device__ __forceinline__ uint32_t zs_st_key(uint32_t i, uint32_t mask) {
  uint32_t x = i * 0x9e3779b9u + 0x7f4a7c15u;
  x ^= x << 13; x ^= x >> 17; x ^= x << 5;
  return x & mask;
}

__global__ __launch_bounds__(64) void zs_k_selftest(uint32_t* __restrict__ bad, int rounds) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t keys[64];
  __shared__ uint32_t half[128];  // 256 u16 buckets, two per word (zs_k_fast's head[])
  __shared__ uint32_t hcnt[128];  // 256 u16 counters, two per word (zs_k_bucket)
  const uint32_t lane = threadIdx.x;
  const uint32_t mask = (blockIdx.x & 3u) == 0 ? 0u : (blockIdx.x & 3u) == 1 ? 3u : (blockIdx.x & 3u) == 2 ? 15u : 255u;
  for (uint32_t i = lane; i < 256; i += 64) { tab[i] = 0; cnt[i] = 0; }
  for (uint32_t i = lane; i < 128; i += 64) { half[i] = 0; hcnt[i] = 0; }
  __syncthreads();
  uint32_t errs = 0;
  for (int r = 0; r < rounds; r++) {
    const uint32_t k = zs_st_key((blockIdx.x * rounds + r) * 64 + lane, mask);
    keys[lane] = k;
    const uint32_t sh = 16u * (k & 1u);
    const uint32_t before_x = tab[k], before_c = cnt[k], before_h = (half[k >> 1] >> sh) & 0xffffu;
    const uint32_t before_hc = (hcnt[k >> 1] >> sh) & 0xffffu;
    __syncthreads();
    const uint32_t val = 1 + lane + 64u * (uint32_t)r;
    const uint32_t old_x = atomicExch(&tab[k], val);
    const uint32_t old_c = atomicAdd(&cnt[k], 1u);
    uint32_t old_w, old_hc;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(old_hc)
                 : "v"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)&hcnt[k >> 1]), "v"(1u << sh)
                 : "memory");
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(old_w)
                 : "v"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)&half[k >> 1]),
                   "v"(0xffffu << sh), "v"((val & 0xffffu) << sh)
                 : "memory");
    // lane order: the exchange returns the value of the highest lower lane with
    // the same key (else the table before the instruction); the add returns the
    // count before plus the number of lower lanes with the same key
    uint32_t lower = 0, last_lower = 0;
    for (uint32_t l = 0; l < lane; l++)
      if (keys[l] == k) { lower++; last_lower = 1 + l + 64u * (uint32_t)r; }
    if (old_x != (lower ? last_lower : before_x)) errs++;
    if (old_c != before_c + lower) errs++;
    if (((old_w >> sh) & 0xffffu) != (lower ? (last_lower & 0xffffu) : before_h)) errs++;
    if (((old_hc >> sh) & 0xffffu) != ((before_hc + lower) & 0xffffu)) errs++;
    __syncthreads();
  }
  if (errs) atomicAdd(bad, errs);
}
