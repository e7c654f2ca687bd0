// zs_parse.h -- one step of deflate_slow's lazy parse over the match table
// (deflate.ts:1356-1426) and the slide schedule, used by the zs_k_parse family
// (deflate_parse.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zs_common.h"

#define ZS_NONE 0xffffffffu

struct zs_pstate {
  uint32_t p, ma, ml, ms;
};

// One iteration of deflate_slow's loop at position p (deflate.ts:1356-1426),
// given the match-table entry e of p and the byte in[p-1].  Returns the symbol
// tallied (ZS_NONE: none).  Symbols: literal = byte, match = 0x80000000 |
// (len - 3) << 16 | dist.
// Written without branches (selects only): the lanes of a wave stand at
// different points of their parses, and a branchy step costs every lane all
// paths plus the exec-mask bookkeeping.
static __device__ __forceinline__ uint32_t zs_parse_step(zs_pstate& st, uint2 e, uint32_t lit, uint32_t n, int good,
                                                         int lazy) {
  const uint32_t p = st.p, pl = st.ml, pm = st.ms;
  // head slot emptied by a slide at exactly this position
  const bool nil = ((e.x & 0x8000u) != 0) & (p >= ZS_SLIDE_AT) & (((p - ZS_SLIDE_AT) & 32767u) == 0) &
                   (n - p < (uint32_t)ZS_MIN_LOOKAHEAD);
  // (lengths are bits 16..24: the parse may carry a byte in the bits above, deflate_parse.hip)
  const bool search = (((e.x >> 16) & 0x1ffu) != 0) & (pl < (uint32_t)lazy) & !nil;  // deflate.ts:1376
  const uint32_t u = pl >= (uint32_t)good ? e.y : e.x;  // chain >> 2 when prev_length >= good (deflate.ts:1075-1077)
  const uint32_t L = (u >> 16) & 0x1ffu, D = u & 0x7fffu;
  const bool take = search & (L > pl);
  const uint32_t ms = take ? p - D : pm;
  const bool too_far = (L == ZS_MIN_MATCH) & (D > ZS_TOO_FAR);  // deflate.ts:1381-1387
  const uint32_t ml = (take & !too_far) ? L : ZS_MIN_MATCH - 1;
  const bool emit = (pl >= ZS_MIN_MATCH) & (ml <= pl);  // emit the previous match (deflate.ts:1389-1411)
  const uint32_t sym = 0x80000000u | ((pl - ZS_MIN_MATCH) << 16) | (p - 1 - pm);
  const uint32_t ret = emit ? sym : (st.ma ? lit : ZS_NONE);  // deferred literal (deflate.ts:1412-1421)
  st.p = emit ? p + pl - 1 : p + 1;
  st.ma = emit ? 0u : 1u;
  st.ml = emit ? ZS_MIN_MATCH - 1 : ml;
  st.ms = ms;
  return ret;
}

// Number of fill_window slides performed by the time the parse visits v
// (slide j happens at the first visited position >= T_j with
// T_j = max(32768 j + 65274, min(n, 32768 j + 65536) - 261), deflate.ts:180-190).
static __device__ __forceinline__ uint32_t zs_slides(uint32_t v, uint32_t n) {
  if (n <= v + 261u) return v >= ZS_SLIDE_AT ? (v - ZS_SLIDE_AT) / 32768u + 1u : 0u;
  return v >= ZS_SLIDE_AT + 1u ? (v - ZS_SLIDE_AT - 1u) / 32768u + 1u : 0u;
}

