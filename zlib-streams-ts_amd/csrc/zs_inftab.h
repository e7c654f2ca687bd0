// zs_inftab.h -- zlib's decoding tables for the inflate kernels: inflate_table
// (inftrees.ts:62-279) and the length / distance bases (inflate/constants.ts:8-45),
// shared by the exact stream-layer kernel (inflate.hip) and the lane-per-member
// path (inflate_lane.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ENOUGH_LENS 852u  // inflate/constants.ts:4-6
#define ENOUGH_DISTS_9 594u

typedef uint32_t zcode;  // op << 24 | bits << 16 | val (inflate/utils.ts:51-72)
#define C_OP(c) ((c) >> 24)
#define C_BITS(c) (((c) >> 16) & 0xffu)
#define C_VAL(c) ((c) & 0xffffu)

enum { CODES = 0, LENS, DISTS };

static __device__ __forceinline__ zcode zpack(uint32_t op, uint32_t bits, uint32_t val) {
  return (op << 24) | (bits << 16) | val;
}

// length/distance tables, inflate/constants.ts:8-45 (ops: 16 + extra, deflate64: 128 + extra),
// in closed form (a lookup in a constant array is a memory round trip per table entry):
//   length code i < 28: extra e = i < 8 ? 0 : i / 4 - 1, base = 3 + i below 8, else ((4 + i % 4) << e) + 3
//     (3, 4, .., 10, 11, 13, 15, 17, 19, 23, .., 227);
//   distance code i < 30: extra e = i < 4 ? 0 : i / 2 - 1, base = 1 + i below 4, else ((2 + i % 2) << e) + 1
//     (1, 2, 3, 4, 5, 7, 9, 13, .., 24577).
// zs_inftab_selfcheck (and every golden) pins them to the reference's tables.
static __device__ __forceinline__ void zs_lbase(uint32_t i, bool d64, uint32_t& base, uint32_t& op) {
  if (i < 28) {
    const uint32_t e = i < 8u ? 0u : (i >> 2) - 1u;
    base = i < 8u ? 3u + i : ((4u + (i & 3u)) << e) + 3u;
    op = (d64 ? 128u : 16u) + e;
  }
  else if (i == 28) { base = d64 ? 3u : 258u; op = d64 ? 144u : 16u; }
  else { base = 0; op = d64 ? (i == 29 ? 72u : 78u) : (i == 29 ? 73u : 200u); }
}
static __device__ __forceinline__ void zs_dbase(uint32_t i, bool d64, uint32_t& base, uint32_t& op) {
  if (i < 30) {
    const uint32_t e = i < 4u ? 0u : (i >> 1) - 1u;
    base = i < 4u ? 1u + i : ((2u + (i & 1u)) << e) + 1u;
    op = (d64 ? 128u : 16u) + e;
  }
  else if (d64) { base = i == 30 ? 32769u : 49153u; op = 128u + 14u; }
  else { base = 0; op = 64u; }
}

// inflate_table (inftrees.ts:62-279).  Returns 0 ok, -1 bad code set, 1 over ENOUGH.
// All lanes execute it on identical values (writes are duplicated, benign).
static __device__ __attribute__((unused)) int zs_inflate_table(int type, const uint16_t* lens, uint32_t codes, zcode* table, uint32_t* bits_io,
                                       uint16_t* work, bool d64, uint32_t* used_out) {
  uint32_t len, sym, min, max, root, curr, drop, used, huff, incr, fill, low, mask;
  int left;
  zcode here;
  uint32_t next = 0;
  uint16_t count[16], offs[16];
  const uint32_t enough_d = d64 ? ENOUGH_DISTS_9 : 592u;
  for (len = 0; len <= 15; len++) count[len] = 0;
  for (sym = 0; sym < codes; sym++) count[lens[sym]]++;
  root = *bits_io;
  for (max = 15; max >= 1; max--) if (count[max] != 0) break;
  if (root > max) root = max;
  if (max == 0) {
    if (!d64) {  // _createTableWhenNoCodes
      table[0] = zpack(64, 1, 0);
      table[1] = zpack(64, 1, 0);
      *bits_io = 1;
      *used_out = 0;
      return 0;
    }
    return -1;
  }
  for (min = 1; min < max; min++) if (count[min] != 0) break;
  if (root < min) root = min;
  left = 1;
  for (len = 1; len <= 15; len++) {
    left <<= 1;
    left -= count[len];
    if (left < 0) return -1;
  }
  if (left > 0 && (type == CODES || max != 1)) return -1;
  offs[1] = 0;
  for (len = 1; len < 15; len++) offs[len + 1] = (uint16_t)(offs[len] + count[len]);
  for (sym = 0; sym < codes; sym++) if (lens[sym] != 0) work[offs[lens[sym]]++] = (uint16_t)sym;
  const int match = type == CODES ? (d64 ? 19 : 20) : type == LENS ? (d64 ? 256 : 257) : (d64 ? -1 : 0);
  huff = 0;
  sym = 0;
  len = min;
  curr = root;
  drop = 0;
  low = 0xffffffffu;
  used = 1u << root;
  mask = used - 1;
#define ZS_OVER(u) ((type == LENS && (d64 ? (u) >= ENOUGH_LENS : (u) > ENOUGH_LENS)) || \
                    (type == DISTS && (d64 ? (u) >= enough_d : (u) > enough_d)))
  if (ZS_OVER(used)) return 1;
  for (;;) {
    const int w = work[sym];
    if (d64 ? w < match : w + 1 < match) {
      here = zpack(0, len - drop, (uint32_t)w);
    } else if (d64 ? w > match : w >= match) {
      uint32_t b, op;
      if (type == CODES) { b = (uint32_t)work[w - match]; op = b; }  // unreachable for valid CODES tables
      else if (type == LENS) zs_lbase((uint32_t)(w - 257), d64, b, op);
      else zs_dbase((uint32_t)(d64 ? w : w - match), d64, b, op);
      here = zpack(op, len - drop, b);
    } else {
      here = zpack(32 + 64, len - drop, 0);
    }
    incr = 1u << (len - drop);
    fill = 1u << curr;
    min = fill;
    do { fill -= incr; table[next + (huff >> drop) + fill] = here; } while (fill != 0);
    incr = 1u << (len - 1);
    while (huff & incr) incr >>= 1;
    if (incr != 0) { huff &= incr - 1; huff += incr; } else huff = 0;
    sym++;
    if (--count[len] == 0) {
      if (len == max) break;
      len = lens[work[sym]];
    }
    if (len > root && (huff & mask) != low) {
      if (drop == 0) drop = root;
      next += 1u << curr;
      curr = len - drop;
      left = 1 << curr;
      while (curr + drop < max) {
        left -= count[curr + drop];
        if (left <= 0) break;
        curr++;
        left <<= 1;
      }
      used += 1u << curr;
      if (ZS_OVER(used)) return 1;
      low = huff & mask;
      table[low] = zpack(curr, root, next);
    }
  }
  if (huff != 0) {
    here = zpack(64, len - drop, 0);
    while (huff != 0) {
      if (drop != 0 && (huff & mask) != low) {
        drop = 0;
        len = root;
        next = 0;
        curr = root;
        here = zpack(64, len, 0);
      }
      table[next + (huff >> drop)] = here;
      incr = 1u << (len - 1);
      while (huff & incr) incr >>= 1;
      if (incr != 0) { huff &= incr - 1; huff += incr; } else huff = 0;
    }
  }
#undef ZS_OVER
  *used_out = used;
  *bits_io = root;
  return 0;
}


#ifndef ZS_HOST_BUILD  // (tools/lane_host compiles the serial form on the CPU: no waves there)
// zs_inflate_table_wave: inflate_table's exact output (same return value, root
// bits, size and entries) built by the 64 lanes of one wave together, for the
// segmented walk's block headers (inflate_seg.hip; the wave and split decoders
// keep the serial form: with both forms inlined they lose occupancy, 7 -> 3
// waves per SIMD for zs_k_split_decode).  Requires all 64 lanes active and
// wave-uniform arguments.
//
// Why: the serial form makes one pass per symbol and per table entry, each a
// chain of dependent LDS round trips for ONE lane's worth of work -- measured in
// the segmented walk at ~214k core cycles for a literal/length table and ~72k
// for a distance table per dynamic header, against ~43k for decoding the ~300
// code lengths themselves (tools/dbg/seg_hdr_clock.py, profiles/r06/hdr/).
//
// How (RFC 1951 3.2.2 canonical codes, which is what inflate_table lays out):
//  * per-length values live across the lanes: lane k holds count[k], the first
//    canonical code of length k and the first sorted index of length k (three
//    VGPRs); a uniform one is a readlane, a per-lane one a __shfl;
//  * the sorted symbol list work[] (by length, then symbol: inflate_table's fill
//    order) from per-length ranks (ballot + mbcnt);
//  * every ROOT entry is the canonical decode of its own index read MSB-first:
//    the code of length L <= root whose value is the index's top L bits, or,
//    past the short codes' range r0, a pointer to a sub-table;
//  * sub-table k serves root prefix r0 + k (a complete code fills every prefix
//    past r0); its size 2^curr follows inflate_table's own rule (inftrees.ts:
//    232-242) with the counts left when the prefix's first code comes up (all
//    codes of longer lengths, the rest of its own length), its offset is a scan
//    of the sizes before it (next += 1 << curr);
//  * every long code replicates its entry in its sub-table, as the serial loop.
// Anything but a complete code set (incomplete, over-subscribed, empty, or a
// table past ENOUGH) is the serial form's business: with SERIAL it runs, and
// returns what zlib returns; without (the segmented walk, whose members then
// take the exact paths) the result is 2.  Checked entry for entry against the
// serial form on random complete code sets of every alphabet
// (zs_inftab_selfcheck, tests/test_gpu_inflate.py).
static __device__ __forceinline__ uint32_t zs_it_rev(uint32_t v, uint32_t n) {  // the low n bits of v reversed (n >= 1)
  return __builtin_bitreverse32(v) >> (32u - n);
}
// lane k's v (k a compile-time constant after unrolling): volatile, so that the
// compiler does not hoist all 45 per-length values out of the loops into SGPRs
static __device__ __forceinline__ uint32_t zs_it_rd(uint32_t v, uint32_t k) {
  k = (uint32_t)__builtin_amdgcn_readfirstlane((int)k);
  asm volatile("" : "+s"(k));  // (an opaque lane index: the read stays where it is used)
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)k);
}
static __device__ __forceinline__ zcode zs_it_here(int type, uint32_t w, uint32_t bits, bool d64) {
  // inftrees.ts:164-182 with match = 20 / 19 (CODES), 257 / 256 (LENS), 0 / -1 (DISTS)
  if (type == CODES) return zpack(0, bits, w);
  if (type == LENS) {
    if (w < 256u) return zpack(0, bits, w);
    if (w == 256u) return zpack(32 + 64, bits, 0);
    uint32_t b, op;
    zs_lbase(w - 257u, d64, b, op);
    return zpack(op, bits, b);
  }
  uint32_t b, op;
  zs_dbase(w, d64, b, op);
  return zpack(op, bits, b);
}
template <bool SERIAL>
static __device__ __attribute__((unused)) int zs_inflate_table_wave(int type, const uint16_t* lens, uint32_t codes,
                                                                     zcode* table, uint32_t* bits_io, uint16_t* work,
                                                                     bool d64, uint32_t* used_out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t lt = (1ull << lane) - 1ull;
  const bool klane = lane >= 1u && lane <= 15u;  // the lanes holding a code length's values
  auto wsync = [] {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // (LDS stores of this wave visible to its own later loads)
    __builtin_amdgcn_wave_barrier();
  };
  auto serial = [&]() -> int {
    if constexpr (SERIAL) return zs_inflate_table(type, lens, codes, table, bits_io, work, d64, used_out);
    else return 2;
  };
  // ---- counts per length: lane k
  uint32_t cntv = 0;
  for (uint32_t s0 = 0; s0 < codes; s0 += 64) {
    const uint32_t s = s0 + lane;
    const uint32_t l = s < codes ? (uint32_t)lens[s] : 0u;
#pragma unroll 1
    for (uint32_t k = 1; k < 16; k++) {
      const uint32_t c = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(l == k));
      cntv += lane == k ? c : 0u;
    }
  }
  // first canonical code fcv = sum_{j<k} count[j] << (k - j), first sorted index offv = sum_{j<k} count[j]
  uint32_t fcv = 0, offv = 0;
#pragma unroll 1
  for (uint32_t j = 1; j < 15; j++) {
    const uint32_t c = zs_it_rd(cntv, j);
    if (klane && lane > j) {
      fcv += c << (lane - j);
      offv += c;
    }
  }
  // ---- a complete code?  over-subscribed at k: fc[k] + count[k] > 2^k; complete: equal at the longest length
  const uint64_t nz = __builtin_amdgcn_ballot_w64(klane && cntv != 0u);
  const uint64_t over = __builtin_amdgcn_ballot_w64(klane && fcv + cntv > (1u << lane));
  if (nz == 0 || over != 0) return serial();
  const uint32_t mx = 63u - (uint32_t)__builtin_clzll(nz), mn = (uint32_t)__builtin_ctzll(nz);
  if (zs_it_rd(fcv + cntv, mx) != (1u << mx)) return serial();
  uint32_t root = (uint32_t)__builtin_amdgcn_readfirstlane((int)*bits_io);
  if (root > mx) root = mx;
  if (root < mn) root = mn;
  // ---- sorted symbols: work[offs[l] + rank among the symbols of length l]
  {
    uint32_t runv = offv;
    for (uint32_t s0 = 0; s0 < codes; s0 += 64) {
      const uint32_t s = s0 + lane;
      const uint32_t l = s < codes ? (uint32_t)lens[s] : 0u;
      uint32_t at = 0;
#pragma unroll 1
      for (uint32_t k = 1; k < 16; k++) {
        const uint64_t b = __builtin_amdgcn_ballot_w64(l == k);
        if (l == k) at = zs_it_rd(runv, k) + (uint32_t)__builtin_popcountll(b & lt);
        runv += lane == k ? (uint32_t)__builtin_popcountll(b) : 0u;
      }
      if (l) work[at] = (uint16_t)s;
    }
  }
  // root slots taken by the codes of length <= root
  uint32_t r0 = 0;
#pragma unroll 1
  for (uint32_t k = 1; k < 16; k++)
    if (k <= root) r0 += zs_it_rd(cntv, k) << (root - k);
  const uint32_t nroot = 1u << root, nsub = nroot - r0;
  // ---- sub-tables: prefix r0 + k for k < nsub; sizes 2^curr, offsets by a scan
  uint32_t used = nroot;
  for (uint32_t k0 = 0; k0 < nsub; k0 += 64) {
    const uint32_t k = k0 + lane;
    const uint32_t r = r0 + k;
    const bool sub = k < nsub;
    uint32_t L1 = sub ? 0u : root + 1u, rem = 1;  // (lanes past the last sub-table: a dummy)
#pragma unroll 1
    for (uint32_t L = 2; L < 16; L++) {  // the prefix's first code: the shortest length with a code under it
      if (L > root) {
        const uint32_t cL = zs_it_rd(cntv, L), fL = zs_it_rd(fcv, L);
        const uint32_t lo = r << (L - root), hi = (r + 1u) << (L - root);
        const uint32_t c = max(lo, fL);
        if (L1 == 0u && cL != 0u && c < hi && c < fL + cL) {
          L1 = L;
          rem = cL - (c - fL);  // codes of this length left, this one included
        }
      }
    }
    // inftrees.ts:232-242: curr = len - root, then grow while the codes left do not fill it
    uint32_t curr = L1 - root;
    int lf = 1 << curr;
    bool go = true;
#pragma unroll 1
    for (uint32_t L = 2; L < 16; L++) {
      if (L > root && L < mx) {
        const uint32_t cL = zs_it_rd(cntv, L);
        if (go && L == curr + root) {
          lf -= (int)(L == L1 ? rem : cL);
          if (lf <= 0) go = false;
          else {
            curr++;
            lf <<= 1;
          }
        }
      }
    }
    const uint32_t size = sub ? 1u << curr : 0u;
    uint32_t x = size;  // inclusive scan over the lanes
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
      if (lane >= d) x += y;
    }
    if (sub) table[zs_it_rev(r, root)] = zpack(curr, root, used + x - size);
    used += zs_it_rd(x, 63);
  }
  if (type == LENS ? (d64 ? used >= ENOUGH_LENS : used > ENOUGH_LENS)
                   : type == DISTS ? (d64 ? used >= ENOUGH_DISTS_9 : used > 592u) : false)
    return serial();  // (it returns 1)
  wsync();  // work[] and the sub-table pointers
  // ---- root entries of the short codes: the canonical decode of each index
  for (uint32_t i0 = 0; i0 < nroot; i0 += 64) {
    const uint32_t i = i0 + lane;
    const uint32_t r = zs_it_rev(i, root);  // the index read MSB-first
    uint32_t L1 = 0, at = 0;
#pragma unroll 1
    for (uint32_t L = 1; L < 16; L++) {
      if (L <= root) {
        const uint32_t d = (r >> (root - L)) - zs_it_rd(fcv, L);
        if (L1 == 0u && d < zs_it_rd(cntv, L)) {
          L1 = L;
          at = zs_it_rd(offv, L) + d;
        }
      }
    }
    if (i < nroot && L1) table[i] = zs_it_here(type, work[at], L1, d64);
  }
  // ---- long codes (sorted indices offs[root + 1] ..): entries replicated in their sub-table
  const uint32_t ntot = zs_it_rd(offv + cntv, mx);
  const uint32_t lfirst = root < mx ? zs_it_rd(offv, root + 1u) : ntot;
  for (uint32_t j0 = lfirst; j0 < ntot; j0 += 64) {
    const uint32_t j = j0 + lane;
    uint32_t L = 0, fL = 0, oL = 0;
#pragma unroll 1
    for (uint32_t k = 2; k < 16; k++) {
      if (k > root) {
        const uint32_t o = zs_it_rd(offv, k);
        if (j >= o && zs_it_rd(cntv, k) != 0u) {
          L = k;
          fL = zs_it_rd(fcv, k);
          oL = o;
        }
      }
    }
    if (j < ntot) {
      const uint32_t c = fL + (j - oL);
      const uint32_t ptr = table[zs_it_rev(c >> (L - root), root)];
      const uint32_t curr = C_OP(ptr), next = C_VAL(ptr);
      const zcode here = zs_it_here(type, work[j], L - root, d64);
      const uint32_t base = next + zs_it_rev(c, L - root), step = 1u << (L - root);
      for (uint32_t f = 0; f < (1u << curr); f += step) table[base + f] = here;
    }
  }
  wsync();
  *bits_io = root;
  *used_out = used;
  return 0;
}
#endif  // ZS_HOST_BUILD
