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

// ---------------------------------------------------------------------------
// zs_inflate_table_wave (zs_inftab.h) against zlib's serial inflate_table: one
// wave per block builds random complete code sets (a leaf split at random until
// the set has its symbol count; lengths <= 15, shuffled over the alphabet) with
// both and compares the return value, root bits, table size and every entry.
// Test infrastructure (tests/test_gpu_inflate.py); not used by the decoders.
#include "zs_inftab.h"

// the first failing set: type, d64, codes, returns, roots, sizes, lens[320], both tables
__device__ uint32_t zs_inftab_dbg[16 + 320 + 2 * (ENOUGH_LENS + 8)];
__device__ uint32_t zs_inftab_dbg_taken;
extern "C" int zs_inftab_dbg_fetch(void* out, unsigned long long bytes) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_inftab_dbg), bytes < sizeof(zs_inftab_dbg) ? bytes : sizeof(zs_inftab_dbg));
}
__global__ __launch_bounds__(64) void zs_k_inftab_check(uint32_t seed, uint32_t sets, unsigned long long* bad) {
  __shared__ uint16_t lens[320], work[320], work2[320];
  __shared__ zcode ta[ENOUGH_LENS + 8], tb[ENOUGH_LENS + 8];
  __shared__ uint8_t depth[320];
  const uint32_t lane = threadIdx.x;
  uint32_t x = seed * 0x9e3779b9u + blockIdx.x * 0x85ebca6bu + 1u;
  auto rnd = [&]() {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    return x;
  };
  __shared__ uint32_t s_kind, s_codes;
  unsigned long long errs = 0;
  for (uint32_t t = 0; t < sets; t++) {
    if (lane == 0) {  // (lane 0 draws everything: the generator below draws a varying number of times)
      s_kind = rnd() % 4u;  // LENS, DISTS, CODES, deflate64 DISTS
      const uint32_t kd = s_kind;
      s_codes = kd == 0 ? 257u + rnd() % 30u : kd == 2 ? 19u : kd == 3 ? 32u : 2u + rnd() % 29u;
    }
    __syncthreads();
    const uint32_t kind = s_kind;
    const int type = kind == 0 ? LENS : kind == 2 ? CODES : DISTS;
    const bool d64 = kind == 3;
    const uint32_t codes = s_codes;
    const uint32_t maxd = type == CODES ? 7u : 15u;
    if (lane == 0) {
      uint32_t k = 2u + rnd() % (codes - 1u);  // symbols in the code (>= 2: a complete set)
      // leaves of a random full binary tree: split a random leaf (depth < maxd) until there are k
      uint32_t nl = 1;
      depth[0] = 0;
      while (nl < k && nl < codes) {
        uint32_t j = rnd() % nl, tries = 0;
        while (depth[j] >= maxd && tries++ < 400u) j = rnd() % nl;
        if (depth[j] >= maxd) break;
        depth[j]++;
        depth[nl++] = depth[j];
      }
      k = nl;
      for (uint32_t s = 0; s < codes; s++) lens[s] = 0;
      for (uint32_t l = 0; l < k; l++) {  // a random free symbol for each leaf
        uint32_t s = rnd() % codes;
        while (lens[s]) s = (s + 1u) % codes;
        lens[s] = depth[l];
      }
      if (type == LENS) {  // the end-of-block code present, as a valid header needs
        if (!lens[256]) {
          uint32_t s = 0;
          while (!lens[s]) s++;
          lens[256] = lens[s];
          lens[s] = 0;
        }
      }
    }
    __syncthreads();
    uint32_t ba = type == LENS ? 9u : type == CODES ? 7u : 6u, bb = ba, ua = 0, ub = 0;
    const int ra = zs_inflate_table(type, lens, codes, ta, &ba, work, d64, &ua);
    __syncthreads();
    const int rb = zs_inflate_table_wave<true>(type, lens, codes, tb, &bb, work2, d64, &ub);
    __syncthreads();
    unsigned long long e0 = 0;
    if (ra != rb || ba != bb || (ra == 0 && ua != ub)) e0 = 1;
    else if (ra == 0)
      for (uint32_t i = lane; i < ua; i += 64) e0 += ta[i] != tb[i] ? 1u : 0u;
    errs += e0;
    const bool any = __syncthreads_or(e0 != 0);
    if (any && lane == 0 && atomicExch(&zs_inftab_dbg_taken, 1u) == 0u) {
      uint32_t* g = zs_inftab_dbg;
      g[0] = (uint32_t)type; g[1] = d64; g[2] = codes; g[3] = (uint32_t)ra; g[4] = (uint32_t)rb;
      g[5] = ba; g[6] = bb; g[7] = ua; g[8] = ub;
      for (uint32_t i = 0; i < 320; i++) g[16 + i] = i < codes ? lens[i] : 0u;
      for (uint32_t i = 0; i < ENOUGH_LENS + 8; i++) {
        g[16 + 320 + i] = ta[i];
        g[16 + 320 + ENOUGH_LENS + 8 + i] = tb[i];
      }
    }
    __syncthreads();
  }
  if (errs) atomicAdd(bad, errs);
}

extern "C" int zs_inftab_selfcheck(int device, uint32_t seed, uint32_t blocks, uint32_t sets,
                                   unsigned long long* mismatches) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, sizeof(*d)) != hipSuccess) return -1;
  int r = hipMemset(d, 0, sizeof(*d)) == hipSuccess ? 0 : -1;
  if (r == 0) {
    zs_k_inftab_check<<<blocks, 64>>>(seed, sets, d);
    r = hipDeviceSynchronize() == hipSuccess && hipMemcpy(mismatches, d, sizeof(*d), hipMemcpyDeviceToHost) == hipSuccess
            ? 0 : -1;
  }
  (void)hipFree(d);
  return r;
}
