// checksum.hip -- per-stream Adler-32 / CRC-32 of the input, for the zlib and
// gzip wrappers (deflate.ts:155-159 update them in read_buf; the trailer is
// written at deflate.ts:971-983).
//
// One wave per stream; lane i owns the i-th contiguous 1/64 of the stream
// (rounded up to 16 bytes), read 16 bytes at a time with the next 16 in flight.
//   CRC-32 (common/crc32.ts:26-58): each lane computes the standard CRC of its
//   segment, four bytes per step from slice-by-4 LDS tables (the same CRC as the
//   reference's byte table, four table steps folded); lane 0 then folds the 64 segment CRCs with
//   crc32_combine arithmetic (multiplication by x^(8*len) modulo the reflected
//   polynomial 0xedb88320).
//   Adler-32 (common/adler32.ts:4-25): A = 1 + sum x_j, B = n + sum (n-j) x_j
//   (mod 65521); each lane sums its segment, a wave reduction finishes it.
// A per-stream seed continues a running checksum as crc32(crc, buf) /
// adler32(adler, buf) do: CRC(seed, data) = seed * x^(8n) + CRC(0, data) (mod P),
// and Adler with (a0, b0) = (seed & 0xffff, seed >> 16): A = a0 + sum x_j,
// B = b0 + n a0 + sum (n-j) x_j.  An empty stream returns the seed unchanged,
// unreduced, as the reference's loops never run (adler32.ts:14, crc32.ts:34-57).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"

static __device__ uint32_t zs_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0xedb88320u : b >> 1;
  }
  return p;
}

// x^(8 * len) mod P (reflected), by repeated squaring of x^8
static __device__ uint32_t zs_x8nmodp(uint64_t len) {
  uint32_t p = 1u << 31;   // x^0
  uint32_t sq = 1u << 23;  // x^8
  while (len) {
    if (len & 1) p = zs_multmodp(sq, p);
    sq = zs_multmodp(sq, sq);
    len >>= 1;
  }
  return p;
}

// Input bytes [i, i + 16) of the lane's segment as four words: five aligned
// word loads (indices clamped to the word holding the stream's last byte, so
// nothing outside the stream's pages is touched) and funnel shifts.
struct zs_ck_src {
  const uint32_t* w4;
  uint32_t sh, last;
};
static __device__ __forceinline__ uint4 zs_ck_load16(const zs_ck_src& S, uint32_t i) {
  const uint32_t q = (i + S.sh) >> 2, r = (i + S.sh) & 3u;  // (r: any byte offset i)
  uint32_t x[5];
#pragma unroll
  for (int k = 0; k < 5; k++) x[k] = S.w4[min(q + (uint32_t)k, S.last)];
  return make_uint4(__builtin_amdgcn_alignbyte(x[1], x[0], r), __builtin_amdgcn_alignbyte(x[2], x[1], r),
                    __builtin_amdgcn_alignbyte(x[3], x[2], r), __builtin_amdgcn_alignbyte(x[4], x[3], r));
}
static __device__ __forceinline__ uint32_t zs_ck_word(const uint4& d, uint32_t j) {
  return j == 0 ? d.x : j == 1 ? d.y : j == 2 ? d.z : d.w;
}

__global__ __launch_bounds__(64) void zs_k_checksum(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint32_t* __restrict__ in_len, uint32_t* __restrict__ check,
                                                    int kind, const uint32_t* __restrict__ seeds) {
  __shared__ uint32_t T[4][256];  // slice-by-4 tables: T[k][b] = CRC of byte b followed by k zero bytes
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  // Adler: lane i owns bytes [i per, (i + 1) per), per a multiple of 16.  CRC:
  // segments counted from the stream's end, lane i owns [n - (64 - i) per,
  // n - (63 - i) per) clipped at 0, so every segment but the first nonempty one
  // is full (the combine below relies on it)
  const uint32_t per = (((n + 63) / 64) + 15u) & ~15u;
  uint32_t b0 = min(n, lane * per), b1 = min(n, b0 + per);
  if (kind == 2) {
    const uint32_t back = (63u - lane) * per;
    b1 = n > back ? n - back : 0u;
    b0 = b1 > per ? b1 - per : 0u;
  }
  zs_ck_src S;
  S.sh = (uint32_t)((uintptr_t)src & 3u);
  S.w4 = n ? reinterpret_cast<const uint32_t*>(src - S.sh) : in_len;  // an empty stream reads nothing it uses
  S.last = n ? (S.sh + n - 1u) >> 2 : 0u;
  if (kind == 2) {
    for (uint32_t i = lane; i < 256; i += 64) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
      T[0][i] = c;
    }
    __syncthreads();
    for (uint32_t i = lane; i < 256; i += 64) {
      uint32_t c = T[0][i];
      for (int k = 1; k < 4; k++) {
        c = (c >> 8) ^ T[0][c & 0xff];
        T[k][i] = c;
      }
    }
    __syncthreads();
    uint32_t c = 0xffffffffu;
    if (b0 < b1) {
      uint4 d = zs_ck_load16(S, b0);
      for (uint32_t i = b0; i < b1; i += 16) {
        const uint4 cur = d;
        if (i + 16 < b1) d = zs_ck_load16(S, i + 16);  // the next 16 bytes in flight
        const uint32_t m = b1 - i;
        if (m >= 16) {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            c ^= zs_ck_word(cur, (uint32_t)j);
            c = T[3][c & 0xff] ^ T[2][(c >> 8) & 0xff] ^ T[1][(c >> 16) & 0xff] ^ T[0][c >> 24];
          }
        } else {
          for (uint32_t j = 0; j < m; j++)
            c = (c >> 8) ^ T[0][(c ^ (zs_ck_word(cur, j >> 2) >> (8 * (j & 3)))) & 0xff];
        }
      }
    }
    // crc32_combine over the 64 segments as a tree, all lanes at once: in round
    // r lane l (a multiple of 2^(r+1)) appends the 2^r segments after its own
    // run, crc = crc * x^(8 per 2^r) + crc' (mod P).  Every right-hand run is
    // full; a run holding the short or empty segments has only empty ones
    // (CRC 0) before it, so their shift does not matter.
    uint32_t crc = c ^ 0xffffffffu;  // (0 for an empty segment)
    uint32_t xp = n ? zs_x8nmodp(per) : 1u << 31;
#pragma unroll 1
    for (uint32_t r = 0; r < 6; r++) {
      const uint32_t o = (uint32_t)__shfl_down((int)crc, 1 << r, 64);
      const uint32_t cc = zs_multmodp(xp, crc) ^ o;
      if ((lane & ((2u << r) - 1u)) == 0) crc = cc;
      if (r < 5) xp = zs_multmodp(xp, xp);
    }
    if (lane == 0) {
      const uint32_t seed = seeds ? seeds[s] : 0u;
      if (!n) crc = seed;  // crc32 of nothing (crc32.ts:27-29): the seed
      else if (seed) crc ^= zs_multmodp(zs_x8nmodp(n), seed);
      check[s] = crc;
    }
  } else {
    uint64_t a = 0, w = 0;
    if (b0 < b1) {
      uint4 d = zs_ck_load16(S, b0);
      uint32_t since = 0;
      for (uint32_t i = b0; i < b1; i += 16) {
        const uint4 cur = d;
        if (i + 16 < b1) d = zs_ck_load16(S, i + 16);
        const uint32_t m = min(16u, b1 - i);
        for (uint32_t j = 0; j < m; j++) {
          const uint32_t x = (zs_ck_word(cur, j >> 2) >> (8 * (j & 3))) & 0xffu;
          a += x;
          w += (uint64_t)(n - (i + j)) * x;
        }
        if (++since == 256) { a %= 65521; w %= 65521; since = 0; }  // 4 KiB between reductions
      }
    }
    a %= 65521;
    w %= 65521;
    for (int d = 32; d >= 1; d >>= 1) {
      a += __shfl_down(a, d, 64);
      w += __shfl_down(w, d, 64);
    }
    if (lane == 0) {
      const uint32_t seed = seeds ? seeds[s] : 1u;
      const uint64_t a0 = seed & 0xffffu, b0 = seed >> 16;
      const uint32_t A = (uint32_t)((a0 + a) % 65521);
      const uint32_t B = (uint32_t)((b0 + ((uint64_t)n % 65521) * a0 + w) % 65521);
      check[s] = n ? (B << 16) | A : seed;
    }
  }
}
