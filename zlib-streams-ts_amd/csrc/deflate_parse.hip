// deflate_parse.hip -- the lazy-match parse of deflate_slow (deflate.ts:1352-1448)
// replayed over the per-position match table built by zs_k_match.
//
// One wave per stream.  The parse is a serial state machine,
// so all 64 lanes run it in lock-step on identical values (no divergence,
// LDS reads broadcast) and cooperate only to stage the next 2 K positions of
// match results / input bytes into LDS and to drain the symbol buffer with
// coalesced stores.  Blocks close every 16383 tallied symbols (deflate.ts:336,
// deflate/utils.ts:68,80); a block's input range ends right after its last
// symbol, as FLUSH_BLOCK_ONLY sets block_start = strstart (deflate.ts:1120-1124).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"

#define ZS_PARSE_MB 2048u  // staged positions
#define ZS_PARSE_SB 1024u  // staged symbols

// symbol encoding: literal = byte; match = 0x80000000 | (len-3) << 16 | dist
__global__ __launch_bounds__(64) void zs_k_parse(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                 const uint32_t* __restrict__ in_len,
                                                 const uint64_t* __restrict__ pos_base,
                                                 const uint32_t* __restrict__ blk_base, const uint2* __restrict__ mres,
                                                 uint32_t* __restrict__ syms, zs_block* __restrict__ blocks,
                                                 zs_stream* __restrict__ streams, int good, int lazy) {
  __shared__ uint2 mb[ZS_PARSE_MB];
  __shared__ uint8_t bb[ZS_PARSE_MB + 4];
  __shared__ uint32_t sb[ZS_PARSE_SB];
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  const uint2* M = mres + pos_base[s];
  uint32_t* sy = syms + pos_base[s] + s;  // each stream owns n+1 symbol slots
  zs_block* blk = blocks + blk_base[s];

  uint32_t p = 0, ma = 0, ml = ZS_MIN_MATCH - 1, ms = 0, base = 0;
  uint32_t nsym = 0, sbn = 0, in_blk = 0, nflush = 0, blk_start = 0;
  uint32_t c0 = 0u - ZS_PARSE_MB;  // staged range [c0, c0 + MB); forces the first stage

  auto stage = [&](uint32_t at) {
    __syncthreads();
    for (uint32_t i = lane; i < ZS_PARSE_MB; i += 64) {
      const uint32_t q = at + i;
      mb[i] = q < n ? M[q] : make_uint2(0, 0);
      bb[i + 1] = q < n ? src[q] : 0;
    }
    if (lane == 0) bb[0] = at > 0 ? src[at - 1] : 0;  // bb[i] = in[at - 1 + i]
    __syncthreads();
  };
  auto drain = [&]() {
    __syncthreads();
    const uint32_t o = nsym - sbn;
    for (uint32_t i = lane; i < sbn; i += 64) sy[o + i] = sb[i];
    sbn = 0;
    __syncthreads();
  };
  auto emit = [&](uint32_t v) {
    if (lane == 0) sb[sbn] = v;
    sbn++;
    nsym++;
    in_blk++;
    if (sbn == ZS_PARSE_SB) drain();
  };
  auto close_block = [&](uint32_t end) {  // FLUSH_BLOCK(s, 0)
    if (lane == 0) {
      zs_block b;
      b.sym_start = nsym - in_blk;
      b.sym_count = in_blk;
      b.in_start = blk_start;
      b.in_end = end;
      b.type = 0; b.hdr_bits = 0; b.data_bits = 0; b.pad = 0; b.bit_off = 0; b.bit_end = 0;
      b.last = blk_start < base ? 2u : 0u;
      blk[nflush] = b;
    }
    nflush++;
    in_blk = 0;
    blk_start = end;
  };

  while (p < n) {
    if (p - c0 >= ZS_PARSE_MB) { stage(p); c0 = p; }
    // fill_window's slide schedule (deflate.ts:180-190): only needed
    // to know whether the head candidate at exactly MAX_DIST is the NIL slot.
    bool slid = false;
    if (p - base >= ZS_SLIDE_AT && min(n, base + 65536u) - p < ZS_MIN_LOOKAHEAD) { base += 32768u; slid = true; }
    const uint32_t pl = ml, pm = ms;
    ml = ZS_MIN_MATCH - 1;
    const uint2 e = mb[p - c0];
    if ((e.x >> 16) != 0 && pl < (uint32_t)lazy && !(slid && (e.x & 0x8000u))) {
      const uint32_t u = pl >= (uint32_t)good ? e.y : e.x;  // chain >> 2 when prev_length >= good
      const uint32_t L = u >> 16, D = u & 0x7fffu;
      if (L > pl) {
        ml = L;
        ms = p - D;
        if (L == ZS_MIN_MATCH && D > ZS_TOO_FAR) ml = ZS_MIN_MATCH - 1;  // deflate.ts:1381-1387
      }
    }
    if (pl >= ZS_MIN_MATCH && ml <= pl) {  // emit the previous match (deflate.ts:1389-1411)
      emit(0x80000000u | ((pl - ZS_MIN_MATCH) << 16) | (p - 1 - pm));
      p += pl - 1;
      ma = 0;
      ml = ZS_MIN_MATCH - 1;
      if (in_blk == ZS_SYM_END) close_block(p);
    } else if (ma) {  // deferred literal (deflate.ts:1412-1421)
      emit(bb[p - c0]);
      if (in_blk == ZS_SYM_END) close_block(p);
      p++;
    } else {
      ma = 1;
      p++;
    }
  }
  if (ma) {  // final deferred literal, tallied without a flush check (deflate.ts:1429-1432)
    if (p - c0 > ZS_PARSE_MB) { stage(p - 1); c0 = p - 1; }
    emit(bb[p - c0]);
  }
  drain();
  // final block (deflate.ts:1434-1440): whatever is left, possibly empty
  if (lane == 0) {
    zs_block b;
    b.sym_start = nsym - in_blk;
    b.sym_count = in_blk;
    b.in_start = blk_start;
    b.in_end = n;
    b.type = 0; b.hdr_bits = 0; b.data_bits = 0; b.pad = 0; b.bit_off = 0; b.bit_end = 0;
    b.last = 1u | (blk_start < base ? 2u : 0u);
    blk[nflush] = b;
    streams[s].nsym = nsym;
    streams[s].nblk = nflush + 1;
  }
}
