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

// length/distance tables, inflate/constants.ts:8-45 (ops: 16 + extra, deflate64: 128 + extra)
static __device__ __forceinline__ void zs_lbase(uint32_t i, bool d64, uint32_t& base, uint32_t& op) {
  static constexpr uint16_t lb[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
  static constexpr uint8_t le[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
  if (i < 28) { base = lb[i]; op = (d64 ? 128u : 16u) + le[i]; }
  else if (i == 28) { base = d64 ? 3u : 258u; op = d64 ? 144u : 16u; }
  else { base = 0; op = d64 ? (i == 29 ? 72u : 78u) : (i == 29 ? 73u : 200u); }
}
static __device__ __forceinline__ void zs_dbase(uint32_t i, bool d64, uint32_t& base, uint32_t& op) {
  static constexpr uint16_t db[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                      193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
  static constexpr uint8_t de[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  if (i < 30) { base = db[i]; op = (d64 ? 128u : 16u) + de[i]; }
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

