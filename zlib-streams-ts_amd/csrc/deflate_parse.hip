// deflate_parse.hip -- the lazy-match parse of deflate_slow (deflate.ts:1352-1448)
// replayed over the per-position match table built by zs_k_match.
//
// The parse is a serial state machine whose state is (position,
// match_available, prev_length, prev_match).  Whenever prev_length is
// MIN_MATCH - 1 -- after every emitted match (deflate.ts:1408-1409), after
// every literal that found no match, and at position 0 -- prev_match is dead,
// so two parses of the same match table that reach the same (position,
// match_available) in that state produce identical symbols from there on.
// One wave per stream therefore works on rounds of 64 segments of ZS_SEG
// positions:
//
//   pass A  lane k parses segment k from the state at position 0 placed at the
//           segment's first position ("speculative"), recording its symbols
//           and the (position, match_available) pairs it passes with
//           prev_length = 2 inside the segment (sync points);
//   pass B  lane 0 replays the TRUE parse across each segment boundary only
//           until it reaches a sync point of the next segment -- from there the
//           speculative symbols are exact (2-3 steps per segment on text);
//   pass C  the wave splices catch-up + speculative symbols into the stream's
//           symbol array and closes a block after every 16383rd tallied symbol
//           (deflate.ts:336; FLUSH_BLOCK sets block_start = strstart,
//           deflate.ts:1120-1124) from a prefix sum of symbol lengths.
//
// fill_window's slide schedule (deflate.ts:180-190) enters the parse only
// through the NIL head slot at exactly MAX_DIST: that happens iff
// the slide falls on p itself, i.e. p = 32768 j + 65274 with the input ending
// within the window (n - p < 262) -- a pure function of p, so no state is needed.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"
#include "zs_parse.h"

#define ZS_SEG 1024u                        // positions per speculative segment
#define ZS_SPEC_SLOTS 1284u                 // >= ZS_SEG + MAX_MATCH - 1 symbols
#define ZS_SYNC_SLOTS 1028u                 // >= ZS_SEG sync points + sentinel
#define ZS_FIX_SLOTS 1284u
#define ZS_SEG_WORDS (ZS_SPEC_SLOTS + ZS_SYNC_SLOTS + ZS_FIX_SLOTS)
static_assert(ZS_SPEC_SLOTS % 4 == 0 && ZS_SEG_WORDS % 4 == 0, "16-byte aligned scratch regions");
static_assert(ZS_SEG == ZS_PARSE_SEG && ZS_SEG_WORDS == ZS_PARSE_SEG_WORDS, "scratch layout shared with capi.cpp");

struct zs_seg_info {
  uint32_t end;         // first position >= the segment end visited by the speculative parse
  uint32_t nspec;       // speculative symbols
  uint32_t ma, ml, ms;  // speculative state at `end`
  uint32_t start;       // position where the segment's final symbol run starts
  uint32_t nfix;        // catch-up symbols (true parse) preceding the splice
  uint32_t from;        // first speculative symbol kept (ZS_NONE: none)
};

__global__ __launch_bounds__(64) void zs_k_parse(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                 const uint32_t* __restrict__ in_len,
                                                 const uint64_t* __restrict__ pos_base,
                                                 const uint32_t* __restrict__ blk_base, const uint2* __restrict__ mres,
                                                 uint32_t* __restrict__ syms, zs_block* __restrict__ blocks,
                                                 zs_stream* __restrict__ streams, uint32_t* __restrict__ scratch,
                                                 int good, int lazy) {
  __shared__ zs_seg_info seg[64];
  __shared__ uint32_t sh_tail[1];  // true parse's match_available after the round
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  const uint2* M = mres + pos_base[s];
  uint32_t* sy = syms + pos_base[s] + s;  // each stream owns n+1 symbol slots
  uint32_t* scr = scratch + (size_t)ZS_SEG_WORDS * (pos_base[s] / ZS_SEG + s);
  zs_block* blk = blocks + blk_base[s];
  const uint32_t nseg = (n + ZS_SEG - 1) / ZS_SEG;

  zs_pstate t = {0, 0, ZS_MIN_MATCH - 1, 0};  // true parse state (lane 0)
  uint32_t total = 0;  // symbols written (wave-uniform)
  uint32_t last_start = 0;  // start position of the last symbol written (lane 63 of the last chunk)

  for (uint32_t r0 = 0; r0 < nseg; r0 += 64) {
    const uint32_t nr = min(64u, nseg - r0);
    // ---- pass A: speculative parse of segment r0 + lane
    if (lane < nr) {
      const uint32_t k = r0 + lane;
      const uint32_t a = k * ZS_SEG, b = min(n, a + ZS_SEG);
      uint32_t* spec = scr + (size_t)lane * ZS_SEG_WORDS;
      uint32_t* sync = spec + ZS_SPEC_SLOTS;
      zs_pstate st = {a, 0, ZS_MIN_MATCH - 1, 0};
      uint32_t cnt = 0, nsync = 0;
      // Symbols and sync entries are gathered four at a time and stored as one
      // 16-byte write: on gfx9 stores share vmcnt with loads, so a store in every
      // iteration would make each match-table load wait for the previous stores.
      uint4 sacc = make_uint4(0, 0, 0, 0), yacc = make_uint4(0, 0, 0, 0);
      while (st.p < b) {
        // sync key: (position - a) << 1 | match_available, with the symbol count
        if (st.ml == ZS_MIN_MATCH - 1) {
          const uint32_t y = ((st.p - a) << 17) | (st.ma << 16) | cnt, m = nsync & 3u;
          yacc.x = m == 0 ? y : yacc.x;
          yacc.y = m == 1 ? y : yacc.y;
          yacc.z = m == 2 ? y : yacc.z;
          yacc.w = m == 3 ? y : yacc.w;
          if (++nsync % 4 == 0) *reinterpret_cast<uint4*>(sync + nsync - 4) = yacc;
        }
        const uint32_t p = st.p;
        const uint32_t v = zs_parse_step(st, M[p], p > 0 ? src[p - 1] : 0u, n, good, lazy);
        if (v != ZS_NONE) {
          const uint32_t m = cnt & 3u;
          sacc.x = m == 0 ? v : sacc.x;
          sacc.y = m == 1 ? v : sacc.y;
          sacc.z = m == 2 ? v : sacc.z;
          sacc.w = m == 3 ? v : sacc.w;
          if (++cnt % 4 == 0) *reinterpret_cast<uint4*>(spec + cnt - 4) = sacc;
        }
      }
      for (uint32_t i = nsync & ~3u; i < nsync; i++) sync[i] = (i & 3u) == 0 ? yacc.x : (i & 3u) == 1 ? yacc.y : yacc.z;
      for (uint32_t i = cnt & ~3u; i < cnt; i++) spec[i] = (i & 3u) == 0 ? sacc.x : (i & 3u) == 1 ? sacc.y : sacc.z;
      sync[nsync] = ZS_NONE;
      if (b == n && st.ma) spec[cnt++] = src[n - 1];  // final deferred literal (deflate.ts:1429-1432)
      seg[lane].end = st.p;
      seg[lane].nspec = cnt;
      seg[lane].ma = st.ma;
      seg[lane].ml = st.ml;
      seg[lane].ms = st.ms;
    }
    __syncthreads();

    // ---- pass B: the true parse across each boundary, until it meets a sync point
    if (lane == 0) {
      for (uint32_t j = 0; j < nr; j++) {
        const uint32_t a = (r0 + j) * ZS_SEG, b = min(n, a + ZS_SEG);
        const uint32_t* spec = scr + (size_t)j * ZS_SEG_WORDS;
        const uint32_t* sync = spec + ZS_SPEC_SLOTS;
        uint32_t* fix = scr + (size_t)j * ZS_SEG_WORDS + ZS_SPEC_SLOTS + ZS_SYNC_SLOTS;
        uint32_t nf = 0, from = ZS_NONE, si = 0, sv = sync[0];
        uint4 facc = make_uint4(0, 0, 0, 0);
        seg[j].start = t.p - t.ma;  // a pending literal in[t.p - 1] opens the run
        while (t.p < b) {
          if (t.ml == ZS_MIN_MATCH - 1) {
            const uint32_t key = ((t.p - a) << 1) | t.ma;
            while ((sv >> 16) < key) sv = sync[++si];  // sentinel 0xffffffff stops the scan
            if ((sv >> 16) == key) { from = sv & 0xffffu; break; }
          }
          const uint32_t p = t.p;
          const uint32_t v = zs_parse_step(t, M[p], p > 0 ? src[p - 1] : 0u, n, good, lazy);
          if (v != ZS_NONE) {  // gathered four at a time (see pass A)
            const uint32_t m = nf & 3u;
            facc.x = m == 0 ? v : facc.x;
            facc.y = m == 1 ? v : facc.y;
            facc.z = m == 2 ? v : facc.z;
            facc.w = m == 3 ? v : facc.w;
            if (++nf % 4 == 0) *reinterpret_cast<uint4*>(fix + nf - 4) = facc;
          }
        }
        for (uint32_t i = nf & ~3u; i < nf; i++) fix[i] = (i & 3u) == 0 ? facc.x : (i & 3u) == 1 ? facc.y : facc.z;
        if (from != ZS_NONE) {  // continue from the speculative end state
          t.p = seg[j].end;
          t.ma = seg[j].ma;
          t.ml = seg[j].ml;
          t.ms = seg[j].ms;
        } else if (b == n && t.ma) {
          fix[nf++] = src[n - 1];  // final deferred literal
        }
        seg[j].nfix = nf;
        seg[j].from = from;
      }
      sh_tail[0] = t.ma;
    }
    __syncthreads();
    const bool last_round = r0 + nr == nseg;
    const bool final_lit = last_round && sh_tail[0] != 0;
    uint32_t round_total = 0;
    if (last_round) {
      for (uint32_t j = 0; j < nr; j++)
        round_total += seg[j].nfix + (seg[j].from == ZS_NONE ? 0u : seg[j].nspec - seg[j].from);
    }
    const uint32_t unchecked = final_lit ? total + round_total - 1 : ZS_NONE;  // global index of the final literal

    // ---- pass C: splice and cut blocks.  A segment's run is its catch-up
    // symbols followed by its speculative symbols from the sync point; they are
    // read four 64-symbol chunks at a time before any of them is stored (loads
    // wait for earlier stores on gfx9).
    for (uint32_t j = 0; j < nr; j++) {
      const zs_seg_info si = seg[j];
      uint32_t pos = si.start;
      const uint32_t* base = scr + (size_t)j * ZS_SEG_WORDS;
      const uint32_t* fx = base + ZS_SPEC_SLOTS + ZS_SYNC_SLOTS;
      const uint32_t* sp = base + (si.from == ZS_NONE ? 0u : si.from);
      const uint32_t cnt = si.nfix + (si.from == ZS_NONE ? 0u : si.nspec - si.from);
      for (uint32_t g0 = 0; g0 < cnt; g0 += 256) {
        uint32_t vv[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t i = g0 + 64 * q + lane;
          vv[q] = i < cnt ? (i < si.nfix ? fx[i] : sp[i - si.nfix]) : 0u;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t c0 = g0 + 64 * q;
          if (c0 >= cnt) break;
          const uint32_t i = c0 + lane;
          const uint32_t v = vv[q];
          const uint32_t len = i < cnt ? ((v & 0x80000000u) ? ((v >> 16) & 0xffu) + ZS_MIN_MATCH : 1u) : 0u;
          uint32_t x = len;  // inclusive scan of symbol lengths
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= (uint32_t)d) x += y;
          }
          if (i < cnt) {
            const uint32_t gi = total + lane;  // `total` already counts the previous chunks
            sy[gi] = v;
            if ((gi + 1) % ZS_SYM_END == 0 && gi != unchecked) {
              // FLUSH_BLOCK after this symbol; remember the window base for the stored-block check
              const uint32_t bi = (gi + 1) / ZS_SYM_END - 1;
              const uint32_t st0 = pos + x - len;
              blk[bi].in_end = pos + x;
              blk[bi].pad = zs_slides(st0 + 1, n);
            }
          }
          const uint32_t m = min(64u, cnt - c0);
          last_start = __shfl(pos + x - len, (int)m - 1, 64);
          pos += __shfl(x, 63, 64);
          total += m;
        }
      }
    }
    __syncthreads();
  }

  // ---- block records (deflate.ts:1434-1440: the final block takes the rest, possibly empty)
  const bool final_lit = nseg > 0 && sh_tail[0] != 0;
  const uint32_t checked = final_lit ? total - 1 : total;
  const uint32_t nflush = checked / ZS_SYM_END;
  // window base when the final block is flushed: slides up to the last visited position
  const uint32_t v_last = total == 0 ? 0u : final_lit ? n - 1 : last_start + 1;
  const uint32_t final_slides = zs_slides(v_last, n);
  __syncthreads();
  for (uint32_t b0 = 0; b0 <= nflush; b0 += 64) {
    const uint32_t b = b0 + lane;
    zs_block k;
    if (b <= nflush) {
      const uint32_t in_start = b == 0 ? 0u : blk[b - 1].in_end;
      const uint32_t in_end = b < nflush ? blk[b].in_end : n;
      const uint32_t slides = b < nflush ? blk[b].pad : final_slides;
      k.sym_start = b * ZS_SYM_END;
      k.sym_count = b < nflush ? ZS_SYM_END : total - nflush * ZS_SYM_END;
      k.in_start = in_start;
      k.in_end = in_end;
      k.type = 0; k.hdr_bits = 0; k.data_bits = 0; k.pad = 0; k.bit_off = 0; k.bit_end = 0;
      // bit 1: the block began before the slid window (matters for stored blocks)
      k.last = (b == nflush ? 1u : 0u) | ((uint64_t)in_start < 32768ull * slides ? 2u : 0u);
    }
    __syncthreads();  // every read of in_end / pad in this chunk precedes the writes
    if (b <= nflush) blk[b] = k;
    __syncthreads();
  }
  if (lane == 0) {
    streams[s].nsym = total;
    streams[s].nblk = nflush + 1;
  }
}
