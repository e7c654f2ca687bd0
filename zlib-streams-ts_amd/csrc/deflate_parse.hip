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
//   pass B  the TRUE parse across each segment boundary, only until it
//           reaches a sync point of the next segment -- from there the
//           speculative symbols are exact (2-3 steps per segment on text).
//           All boundaries at once: lane k enters segment k with the
//           speculative end state of segment k - 1, which is the true state
//           whenever segment k - 1 synced; an in-order check redoes the rare
//           boundary whose predecessor did not;
//   pass C  a gather concatenates each segment's catch-up + speculative
//           symbols into the stream's symbol array; a block closes after every
//           16383rd tallied symbol (deflate.ts:336; FLUSH_BLOCK sets
//           block_start = strstart, deflate.ts:1120-1124), its input end the
//           cut symbol's segment start plus the lengths before it.
//
// fill_window's slide schedule (deflate.ts:180-190) enters the parse only
// through the NIL head slot at exactly MAX_DIST: that happens iff
// the slide falls on p itself, i.e. p = 32768 j + 65274 with the input ending
// within the window (n - p < 262) -- a pure function of p, so no state is needed.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"
#include "zs_parse.h"

// Scratch per speculative segment of SEG positions: its speculative symbols,
// its sync points (+ sentinel) and its catch-up symbols.
template <uint32_t SEG>
struct zs_seg_cfg {
  static constexpr uint32_t SPEC = (SEG + 260u + 3u) & ~3u;  // >= SEG + MAX_MATCH - 1 symbols + final literal
  static constexpr uint32_t SYNC = SEG + 4u;                 // >= SEG sync points + sentinel
  static constexpr uint32_t FIX = SPEC;
  static constexpr uint32_t WORDS = SPEC + SYNC + FIX;
};
static_assert(zs_seg_cfg<ZS_PARSE_SEG>::WORDS == ZS_PARSE_SEG_WORDS, "scratch layout shared with capi.cpp");
static_assert(zs_seg_cfg<ZS_PARSE2W_SEG>::WORDS == ZS_PARSE2W_SEG_WORDS, "scratch layout shared with capi.cpp");
static_assert(zs_seg_cfg<ZS_PARSE4W_SEG>::WORDS == ZS_PARSE4W_SEG_WORDS, "scratch layout shared with capi.cpp");

// LDS-visible ordering among the lanes of ONE wave (the splice runs on one wave
// while the workgroup's other wave may be elsewhere: no s_barrier)
#define ZS_WAVE_SYNC()                                   \
  do {                                                   \
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); \
    __builtin_amdgcn_wave_barrier();                     \
  } while (0)

// the true parse entering a round, handed from wave to wave (two-wave parse)
struct zs_round_state {
  zs_pstate t;
  uint32_t total, last_sym;
};

// Per-lane match-table windows of pass A (WIN > 0): the wave stages, for every
// lane, the WIN table entries from its position (and the input bytes there) in
// LDS, then parses from LDS until every lane has left its window.  One memory
// round trip per stage instead of one per parse step: a step's position depends
// on the previous step's entry, so direct loads put the full memory latency on
// every step.  Entry k of lane l is at m[k / 2][l] (a lane's reads are 16 B
// apart from its neighbours': conflict-free), bytes in[w + 4 j, +4) at s[j][l].
// WIN = 32 (19 KiB of LDS: 8 workgroups per CU) halves the stages of WIN = 16
// (10 KiB) and measured faster in round 2: 1.54 vs 1.77 ms at 4096 streams,
// 2.99 ms with direct loads (WIN = 0); 0.40 / 0.42 / 0.54 ms at 512.  Only
// WIN = 32 is built.
// The input byte each step needs, in[p - 1], rides in the staged entry of p
// (round 6; before, 2 KiB of staged input words per wave: 19 KiB per workgroup,
// eight per CU, parse 1.55 ms at 4,096 streams; now 16 KiB, ten per CU, 1.47 ms).
template <uint32_t WIN>
struct zs_parse_win {
  uint4 m[WIN / 2][64];
};
template <>
struct zs_parse_win<0> {};

// per-segment values pass C looks up by segment
struct zs_seg_tab {
  uint32_t off[65];  // first run symbol of each segment in the round (exclusive prefix; off[64] = round total)
  uint32_t nf[64];   // catch-up symbols
  uint32_t from[64]; // first speculative symbol kept (ZS_NONE: none)
};

// a wave's window (pass A) and its segment table (passes B, C) are never live
// at once: the workgroup of one wave needs 16 KiB, ten per CU
template <uint32_t WIN>
union zs_parse_lds {
  zs_parse_win<WIN> W;
  zs_seg_tab T;
};

static __device__ __forceinline__ uint32_t zs_sym_len(uint32_t v) {
  return (v & 0x80000000u) ? ((v >> 16) & 0xffu) + ZS_MIN_MATCH : 1u;
}
static __device__ __forceinline__ zs_pstate zs_read_state(const zs_pstate& x, uint32_t l) {
  zs_pstate r;
  r.p = (uint32_t)__builtin_amdgcn_readlane((int)x.p, (int)l);
  r.ma = (uint32_t)__builtin_amdgcn_readlane((int)x.ma, (int)l);
  r.ml = (uint32_t)__builtin_amdgcn_readlane((int)x.ml, (int)l);
  r.ms = (uint32_t)__builtin_amdgcn_readlane((int)x.ms, (int)l);
  return r;
}

#ifndef ZS_PARSE_PROF
#define ZS_PARSE_PROF 0  // timing experiments: cycles per pass summed over waves (0 in the product)
#endif
#if ZS_PARSE_PROF
__device__ unsigned long long zs_pp_stat[16];  // pass A, phase 1 (B + counts), splice, block cuts, records, waves
extern "C" int zs_parse_stats(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_pp_stat), sizeof(zs_pp_stat));
}
#define PP_T(v) unsigned long long v = wall_clock64()
#define PP_ACC(i, v) do { if ((threadIdx.x & 63u) == 0) atomicAdd(&zs_pp_stat[i], wall_clock64() - v); } while (0)
#else
#define PP_T(v) do { } while (0)
#define PP_ACC(i, v) do { } while (0)
#endif

#define ZS_GATHER 16  // pass C: 64-symbol chunks loaded before any is stored
#ifndef ZS_PARSE_WIN
#define ZS_PARSE_WIN 32  // pass A's per-lane match-table window (A/B: 64)
#endif


template <uint32_t WIN, uint32_t SEG, uint32_t NWV>
static __device__ __forceinline__ void zs_parse_body(zs_parse_win<WIN>& W, zs_seg_tab& T, zs_round_state& RS,
                                                     const uint8_t* __restrict__ in,
                                                     const uint64_t* __restrict__ in_off,
                                                     const uint32_t* __restrict__ in_len,
                                                     const uint64_t* __restrict__ pos_base,
                                                     const uint32_t* __restrict__ blk_base,
                                                     const uint2* __restrict__ mres, uint32_t* __restrict__ syms,
                                                     zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,
                                                     uint32_t* __restrict__ scratch, int good, int lazy) {
  using CF = zs_seg_cfg<SEG>;
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  const uint2* M = mres + pos_base[s];
  uint32_t* sy = syms + pos_base[s] + s;  // each stream owns n+1 symbol slots
  // this wave's 64 segment slots (a stream owns >= min(nseg, 64 NWV) slots)
  uint32_t* scr = scratch + (size_t)CF::WORDS * (pos_base[s] / SEG + s + 64u * wave);
  zs_block* blk = blocks + blk_base[s];
  const uint32_t nseg = (n + SEG - 1) / SEG;
  const bool aligned = ((uintptr_t)src & 3u) == 0;

  zs_pstate t = {0, 0, ZS_MIN_MATCH - 1, 0};  // the true parse state entering the round (wave-uniform)
  uint32_t total = 0;     // symbols written (wave-uniform)
  uint32_t last_sym = 0;  // the last symbol written (wave-uniform)
  if (NWV > 1) {
    if (threadIdx.x == 0) RS = {t, 0u, 0u};
    __syncthreads();
  }

  // NWV waves take NWV consecutive rounds of 64 segments at once: every wave
  // runs pass A on its round in parallel, then the waves run passes B and C in
  // round order, handing the true state over through RS.
  for (uint32_t sr = 0; sr < nseg; sr += 64u * NWV) {
    const uint32_t r0 = sr + 64u * wave;
    const uint32_t nr = r0 < nseg ? min(64u, nseg - r0) : 0u;
    const bool mine = lane < nr;  // lane owns segment r0 + lane
    const uint32_t a = mine ? (r0 + lane) * SEG : n, b = mine ? min(n, a + SEG) : n;
    uint32_t* spec = scr + (size_t)lane * CF::WORDS;
    uint32_t* sync = spec + CF::SPEC;
    uint32_t* fix = sync + CF::SYNC;

    // ---- pass A: speculative parse of the lane's segment from the position-0 state
    PP_T(tA);
    zs_pstate st = {a, 0, ZS_MIN_MATCH - 1, 0};
    uint32_t cnt = 0;
    {
      uint32_t nsync = 0;
      // Symbols and sync entries are gathered four at a time and stored as one
      // 16-byte write: on gfx9 stores share vmcnt with loads, so a store in every
      // iteration would make the next load wait for the previous stores.
      uint4 sacc = make_uint4(0, 0, 0, 0), yacc = make_uint4(0, 0, 0, 0);
      auto step = [&](uint2 e, uint32_t lit) __attribute__((always_inline)) {
        // sync key: (position - a) << 1 | match_available, with the symbol count
        if (st.ml == ZS_MIN_MATCH - 1) {
          const uint32_t y = ((st.p - a) << 17) | (st.ma << 16) | cnt, m = nsync & 3u;
          yacc.x = m == 0 ? y : yacc.x;
          yacc.y = m == 1 ? y : yacc.y;
          yacc.z = m == 2 ? y : yacc.z;
          yacc.w = m == 3 ? y : yacc.w;
          if (++nsync % 4 == 0) *reinterpret_cast<uint4*>(sync + nsync - 4) = yacc;
        }
        const uint32_t v = zs_parse_step(st, e, lit, n, good, lazy);
        if (v != ZS_NONE) {
          const uint32_t m = cnt & 3u;
          sacc.x = m == 0 ? v : sacc.x;
          sacc.y = m == 1 ? v : sacc.y;
          sacc.z = m == 2 ? v : sacc.z;
          sacc.w = m == 3 ? v : sacc.w;
          if (++cnt % 4 == 0) *reinterpret_cast<uint4*>(spec + cnt - 4) = sacc;
        }
      };
      if constexpr (WIN == 0) {
        while (st.p < b) {
          const uint32_t p = st.p;
          step(M[p], p > 0 ? src[p - 1] : 0u);
        }
      } else {
        while (__ballot(st.p < b) != 0) {
          // stage: this lane's window [w, w + WIN) (entries past n are never read)
          const uint32_t w = st.p & ~3u;
          if (st.p < b) {
            // every load is issued before the first is waited for: indices are
            // clamped into the stream instead of branched around (entries past
            // n are never read; the table's rows are 8-entry aligned, pos_base)
            const uint4* g = reinterpret_cast<const uint4*>(M);
            const uint32_t glast = ((n + 7u) >> 1) & ~3u;  // the stream's uint4s (two entries each)
            uint4 mv[WIN / 2];
            auto load_m = [&]() __attribute__((always_inline)) {
#pragma unroll
              for (uint32_t j = 0; j < WIN / 2; j++) mv[j] = g[min(w / 2 + j, glast - 1u)];
            };
            auto store_m = [&]() __attribute__((always_inline)) {
#pragma unroll
              for (uint32_t j = 0; j < WIN / 2; j++) W.m[j][lane] = mv[j];
            };
            // in[p - 1] rides in the entry of p: bits 25..31 of x (L <= 258 uses bits 16..24) and bit 31 of
            // y; the parse masks them (zs_parse_step), so the window holds no input bytes
            uint32_t sv[WIN / 4], bw;
            if (aligned) {  // aligned words holding at least one byte of the stream never leave its pages
              load_m();
              const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
              const uint32_t slast = (n - 1u) >> 2;
#pragma unroll
              for (uint32_t j = 0; j < WIN / 4; j++) sv[j] = s4[min(w / 4 + j, slast)];
              bw = w ? s4[w / 4 - 1] >> 24 : 0u;
            } else {
              load_m();
#pragma unroll
              for (uint32_t j = 0; j < WIN / 4; j++) sv[j] = zs_load_word(src, n, w + 4 * j);
              bw = w ? (uint32_t)src[w - 1] : 0u;
            }
            auto byte_at = [&](uint32_t k) __attribute__((always_inline)) {  // in[w + k]
              return (sv[k >> 2] >> (8u * (k & 3u))) & 0xffu;
            };
#pragma unroll
            for (uint32_t j = 0; j < WIN / 2; j++) {
              const uint32_t l0 = j == 0 ? bw : byte_at(2 * j - 1), l1 = byte_at(2 * j);
              mv[j].x |= l0 << 25;
              mv[j].y |= (l0 >> 7) << 31;
              mv[j].z |= l1 << 25;
              mv[j].w |= (l1 >> 7) << 31;
            }
            store_m();
          }
          while (st.p < b && st.p < w + WIN) {
            const uint32_t o = st.p - w;
            const uint2 e = reinterpret_cast<const uint2*>(&W.m[o >> 1][lane])[o & 1];
            step(e, (e.x >> 25) | ((e.y >> 31) << 7));
          }
        }
      }
      if (mine) {
        for (uint32_t i = nsync & ~3u; i < nsync; i++) sync[i] = (i & 3u) == 0 ? yacc.x : (i & 3u) == 1 ? yacc.y : yacc.z;
        for (uint32_t i = cnt & ~3u; i < cnt; i++) spec[i] = (i & 3u) == 0 ? sacc.x : (i & 3u) == 1 ? sacc.y : sacc.z;
        sync[nsync] = ZS_NONE;
        if (b == n && st.ma) spec[cnt++] = src[n - 1];  // final deferred literal (deflate.ts:1429-1432)
      }
    }

    PP_ACC(0, tA);
    // Phase 1 (pass B + the round's symbol count) needs the true state entering
    // the round: the waves run it in round order.  Phase 2 (the splice) needs
    // only this round's results, so a wave's phase 2 overlaps the next wave's
    // phase 1.
    uint32_t nf = 0, from = ZS_NONE, start = 0, R = 0, tot0 = 0;
    bool final_lit_r = false;
    for (uint32_t k = 0; k < NWV + (NWV > 1 ? 1u : 0u); k++) {
    if (NWV > 1) __syncthreads();
    if (nr != 0 && k == wave) {
    PP_T(tB);
    if (NWV > 1) {
      t = RS.t;
      total = RS.total;
    }
    // ---- pass B: the true parse across each boundary until it meets a sync
    // point of the segment.  Every lane does its own boundary at once, entering
    // with the speculative end state of the segment before (which IS the true
    // state there whenever that segment synced; lane 0 enters with the true
    // state); a serial check then redoes, in order, the rare boundary whose
    // predecessor never synced.
    zs_pstate after;  // true state at the segment's end, given its entry state
    auto catch_up = [&](zs_pstate c) __attribute__((always_inline)) {
      uint32_t si = 0, sv = sync[0];
      uint4 facc = make_uint4(0, 0, 0, 0);
      nf = 0;
      from = ZS_NONE;
      start = c.p - c.ma;  // a pending literal in[c.p - 1] opens the run
      while (c.p < b) {
        if (c.ml == ZS_MIN_MATCH - 1) {
          const uint32_t key = ((c.p - a) << 1) | c.ma;
          while ((sv >> 16) < key) sv = sync[++si];  // sentinel 0xffffffff stops the scan
          if ((sv >> 16) == key) { from = sv & 0xffffu; break; }
        }
        const uint32_t p = c.p;
        const uint32_t v = zs_parse_step(c, M[p], p > 0 ? src[p - 1] : 0u, n, good, lazy);
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
      if (from == ZS_NONE && b == n && c.ma) fix[nf++] = src[n - 1];  // final deferred literal
      after = from != ZS_NONE ? st : c;  // synced: continues as the speculative parse did
    };
    {
      zs_pstate e;  // entry: the speculative end of segment lane - 1
      const int up = (int)((lane + 63u) & 63u);
      e.p = (uint32_t)__shfl((int)st.p, up, 64);
      e.ma = (uint32_t)__shfl((int)st.ma, up, 64);
      e.ml = (uint32_t)__shfl((int)st.ml, up, 64);
      e.ms = (uint32_t)__shfl((int)st.ms, up, 64);
      if (lane == 0) e = t;
      if (mine) catch_up(e);
    }
    for (uint32_t j = 0; j < nr; j++) {
      if (j > 0 && (uint32_t)__builtin_amdgcn_readlane((int)from, (int)(j - 1)) == ZS_NONE) {
        if (lane == j) catch_up(t);  // segment j - 1 never synced: t is its true end state
      }
      t = zs_read_state(after, j);
    }

    // ---- pass C: splice.  A segment's run is its catch-up symbols followed
    // by its speculative symbols from the sync point; the round's runs are
    // concatenated into the stream's symbols by a gather, ZS_GATHER chunks of
    // 64 loaded before any is stored (loads wait for earlier stores on gfx9).
    const uint32_t run = mine ? nf + (from == ZS_NONE ? 0u : cnt - from) : 0u;
    uint32_t incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    T.off[lane] = incl - run;
    if (lane == 63) T.off[64] = R;
    T.nf[lane] = nf;
    T.from[lane] = from;
    tot0 = total;
    final_lit_r = r0 + nr == nseg && t.ma != 0;
    total += R;
    if (NWV > 1 && lane == 0) {
      RS.t = t;
      RS.total = total;
    }
    PP_ACC(1, tB);
    }  // phase 1
    if (nr != 0 && k == wave + (NWV > 1 ? 1u : 0u)) {
    ZS_WAVE_SYNC();
    PP_T(tC);
    uint32_t js = 0, lastv = 0;
    for (uint32_t g0 = 0; g0 < R; g0 += 64 * ZS_GATHER) {
      uint32_t v[ZS_GATHER];
#pragma unroll
      for (int k = 0; k < ZS_GATHER; k++) {
        const uint32_t g = g0 + 64 * k + lane;
        v[k] = 0;
        if (g < R) {
          while (T.off[js + 1] <= g) js++;
          const uint32_t i = g - T.off[js], nfj = T.nf[js];
          const uint32_t* base = scr + (size_t)js * CF::WORDS;
          v[k] = i < nfj ? base[CF::SPEC + CF::SYNC + i] : base[T.from[js] + i - nfj];
        }
      }
#pragma unroll
      for (int k = 0; k < ZS_GATHER; k++) {
        const uint32_t g = g0 + 64 * k + lane;
        if (g < R) sy[tot0 + g] = v[k];
        if (g == R - 1) lastv = v[k];
      }
    }
    if (R) {
      last_sym = (uint32_t)__shfl((int)lastv, (int)((R - 1) & 63u), 64);
      if (NWV > 1 && lane == 0) RS.last_sym = last_sym;  // rounds' phases 2 run in order
    }

    PP_ACC(2, tC);
    PP_T(tD);
    // block cuts: FLUSH_BLOCK after every 16383rd tallied symbol (deflate.ts:336,
    // 1120-1124) -- but not after the final deferred literal, which is tallied
    // after the loop (deflate.ts:1429-1432)
    const uint32_t unchecked = final_lit_r ? tot0 + R - 1 : ZS_NONE;
    for (uint32_t gi = (tot0 / ZS_SYM_END + 1) * ZS_SYM_END - 1; gi < tot0 + R; gi += ZS_SYM_END) {
      if (gi == unchecked) continue;
      const uint32_t g = gi - tot0;
      uint32_t j = 0;
      while (T.off[j + 1] <= g) j++;
      const uint32_t i = g - T.off[j], nfj = T.nf[j], fj = T.from[j];
      const uint32_t* base = scr + (size_t)j * CF::WORDS;
      uint32_t acc = 0, li = 0;  // run lengths through symbol i, symbol i's length
      for (uint32_t q = lane; q <= i; q += 64) {
        const uint32_t l = zs_sym_len(q < nfj ? base[CF::SPEC + CF::SYNC + q] : base[fj + q - nfj]);
        acc += l;
        li = q == i ? l : li;
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        acc += __shfl_xor(acc, d, 64);
        li += __shfl_xor(li, d, 64);
      }
      const uint32_t end = (uint32_t)__builtin_amdgcn_readlane((int)start, (int)j) + acc;
      if (lane == 0) {  // the block's input end; its window base for the stored-block check
        const uint32_t bi = (gi + 1) / ZS_SYM_END - 1;
        blk[bi].in_end = end;
        blk[bi].pad = zs_slides(end - li + 1, n);
      }
    }
    PP_ACC(3, tD);
    ZS_WAVE_SYNC();
    }  // phase 2
    }  // handoff
  }
  if (NWV > 1) {
    __syncthreads();
    if (wave != 0) return;
    t = RS.t;
    total = RS.total;
    last_sym = RS.last_sym;
  }

  PP_T(tE);
  // ---- block records (deflate.ts:1434-1440: the final block takes the rest, possibly empty)
  const bool final_lit = nseg > 0 && t.ma != 0;
  const uint32_t checked = final_lit ? total - 1 : total;
  const uint32_t nflush = checked / ZS_SYM_END;
  // window base when the final block is flushed: slides up to the last visited
  // position (the symbols tile [0, n), so the last one starts at n - its length)
  const uint32_t v_last = total == 0 ? 0u : final_lit ? n - 1 : n - zs_sym_len(last_sym) + 1;
  const uint32_t final_slides = zs_slides(v_last, n);
  ZS_WAVE_SYNC();
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
    ZS_WAVE_SYNC();  // every read of in_end / pad in this chunk precedes the writes
    if (b <= nflush) blk[b] = k;
    ZS_WAVE_SYNC();
  }
  if (lane == 0) {
    streams[s].nsym = total;
    streams[s].nblk = nflush + 1;
  }
  PP_ACC(4, tE);
#if ZS_PARSE_PROF
  if (lane == 0) atomicAdd(&zs_pp_stat[5], 1ull);
#endif
}

#define ZS_PARSE_KERNEL(name, WIN, SEG, NWV)                                                                        \
  __global__ __launch_bounds__(64 * NWV) void name(                                                                  \
      const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,     \
      const uint64_t* __restrict__ pos_base, const uint32_t* __restrict__ blk_base, const uint2* __restrict__ mres,  \
      uint32_t* __restrict__ syms, zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,                  \
      uint32_t* __restrict__ scratch, int good, int lazy) {                                                         \
    __shared__ zs_parse_lds<WIN> U[NWV];                                                                            \
    __shared__ zs_round_state RS;                                                                                   \
    const uint32_t w_ = threadIdx.x >> 6;                                                                           \
    zs_parse_body<WIN, SEG, NWV>(U[w_].W, U[w_].T, RS, in, in_off, in_len, pos_base, blk_base, mres, syms, blocks,  \
                                 streams, scratch, good, lazy);                                                     \
  }
ZS_PARSE_KERNEL(zs_k_parse, ZS_PARSE_WIN, ZS_PARSE_SEG, 1)
// two waves per stream, 512-position segments: half the speculative pass per lane (small batches)
ZS_PARSE_KERNEL(zs_k_parse_2w, ZS_PARSE_WIN, ZS_PARSE2W_SEG, 2)
// four waves per stream, 256-position segments
ZS_PARSE_KERNEL(zs_k_parse_4w, ZS_PARSE_WIN, ZS_PARSE4W_SEG, 4)
