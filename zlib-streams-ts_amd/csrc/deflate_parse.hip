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
static_assert(zs_seg_cfg<ZS_PARSEDW_SEG>::WORDS == ZS_PARSEDW_SEG_WORDS, "scratch layout shared with capi.cpp");

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
template <uint32_t WIN>
struct zs_parse_win {
  uint4 m[WIN / 2][64];
  uint32_t s[WIN / 4][64];
  uint32_t b[64];  // in[w - 1]
};
template <>
struct zs_parse_win<0> {};

// per-segment values pass C looks up by segment
struct zs_seg_tab {
  uint32_t off[65];  // first run symbol of each segment in the round (exclusive prefix; off[64] = round total)
  uint32_t nf[64];   // catch-up symbols
  uint32_t from[64]; // first speculative symbol kept (ZS_NONE: none)
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
// zs_k_parse_dw: per-wave accumulators, added once at the end of the wave
#define DP_T(v) unsigned long long v = wall_clock64()
#define DP_ADD(i, v) (dp[i] += wall_clock64() - v)
#define DP_CNT(i, x) (dp[i] += (x))
#define PP_ACC(i, v) do { if ((threadIdx.x & 63u) == 0) atomicAdd(&zs_pp_stat[i], wall_clock64() - v); } while (0)
#else
#define PP_T(v) do { } while (0)
#define PP_ACC(i, v) do { } while (0)
#define DP_T(v) do { } while (0)
#define DP_ADD(i, v) do { } while (0)
#define DP_CNT(i, x) do { } while (0)
#endif

// ---- demand walks (zs_k_parse_dw)
// With the sweep in demand mode (zs_k_sweep, demand = 1) an entry whose
// full-budget result the first chain >> 2 steps do not settle is ZS_MORE | k
// (k = the position's member index in the bucket-sorted member array).  The
// parse asks for the full budget only when prev_length < good_match
// (deflate.ts:1075-1077); there it continues longest_match (deflate.ts:
// 1053-1115) from step chain >> 2 + 1 with the chain >> 2 result as the best so
// far: member k - t is step t's candidate, and the walk stops at the budget, at
// the first member at or below limit (deflate.ts:1109), or where member
// positions stop falling (the bucket's first member has been passed; a member
// of another bucket differs in its first three bytes and cannot win, so a late
// stop only costs steps).  First strictly longer wins, nice ends the walk
// (deflate.ts:1100-1105).  CPU model: tools/emu/emu_demand.c.
#define ZS_DW_WIN_WORDS ((65537u + 20u + 3u) / 4u + 2u)  // the stream in LDS, zero padded

static __device__ __forceinline__ uint32_t zs_dw_word(const uint32_t* win, uint32_t off) {
  const uint32_t i = off >> 2;
  return __builtin_amdgcn_alignbyte(win[i + 1], win[i], off & 3u);
}

#ifndef ZS_DW_EXP
#define ZS_DW_EXP 0  // timing experiments only (wrong output): 1 no extension, 2 no walk
#endif
#ifndef ZS_DW_BATCH
#define ZS_DW_BATCH 4  // 16-byte member loads (8 members each) in flight per walk round trip
#endif
// the stream's walk context
struct zs_dw_ctx {
  const uint32_t* win;  // LDS: the stream, zero padded
  const uint16_t* mem;  // HBM: the stream's member array (16-B aligned)
  uint32_t n, chain, cs, nice;
#if ZS_PARSE_PROF
  unsigned long long* prof;  // walks, members walked (per lane)
#endif
};

// longest_match at p (member k) continued from step cs + 1 (cs = chain >> 2)
// from the chain >> 2 result ey; returns the full-budget entry (len << 16 |
// dist).  Members are read 8 ZS_DW_BATCH at a time (16-byte loads in flight).
// Per 8 members the stop test and a first filter -- the candidate's byte at
// the best length so far, which must match for it to be longer -- are
// computed without branches into a mask; only candidates passing it are
// compared in full, in chain order (a later, longer best only tightens the
// filter: a candidate that failed it cannot be longer).
static __device__ __forceinline__ uint32_t zs_lcp(const uint32_t* win, uint32_t q, uint32_t p, uint32_t maxc) {
  uint32_t L = 0;
  while (L < maxc) {  // eight bytes per round
    const uint32_t y0 = zs_dw_word(win, q + L) ^ zs_dw_word(win, p + L);
    const uint32_t y1 = zs_dw_word(win, q + L + 4) ^ zs_dw_word(win, p + L + 4);
    if (y0 | y1) {
      L += y0 ? (uint32_t)__builtin_ctz(y0) >> 3 : 4u + ((uint32_t)__builtin_ctz(y1) >> 3);
      break;
    }
    L += 8;
  }
  return min(L, maxc);
}

static __device__ __forceinline__ uint32_t zs_walk(const zs_dw_ctx& X, uint32_t p, uint32_t k, uint32_t ey) {
#if ZS_DW_EXP & 2
  return ey;
#endif
  const uint8_t* wb = reinterpret_cast<const uint8_t*>(X.win);
  const uint32_t look = X.n - p;
  const uint32_t maxc = min(look, (uint32_t)ZS_MAX_MATCH), nice = min(look, X.nice);  // deflate.ts:1068,1078-1080
  const uint32_t limit = p > ZS_MAX_DIST ? p - ZS_MAX_DIST : 0u;                        // deflate.ts:1060
  uint32_t bl = ey >> 16, bq = 0;
  bool up = false;
  uint32_t own = wb[p + bl];
  const int jtop = (int)k - (int)X.cs;             // step cs's member: the candidates fall below its position
  const int jend = max((int)k - (int)X.chain, 0);  // step chain's member (or member 0)
  const int cend = jend >> 3;
  uint32_t qprev = 0;
  const uint4* m4 = reinterpret_cast<const uint4*>(X.mem);
  bool go = true;
  uint32_t steps = 0;
  for (int cb = jtop >> 3; go && cb >= cend; cb -= ZS_DW_BATCH) {
    uint4 v[ZS_DW_BATCH];
#pragma unroll
    for (int i = 0; i < ZS_DW_BATCH; i++) v[i] = cb - i >= cend ? m4[cb - i] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < ZS_DW_BATCH; i++) {
      const int c0 = 8 * (cb - i);
      const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      uint32_t qs[8], pm = 0;
#pragma unroll
      for (int u = 0; u < 8; u++) {  // member c0 + 7 - u (descending)
        const uint32_t q = (w[(7 - u) >> 1] >> (16 * ((7 - u) & 1))) & 0xffffu;
        qs[u] = q;
        const uint32_t bu = wb[min(q + bl, X.n)];
        const int idx = c0 + 7 - u;
        qprev = idx == jtop ? q : qprev;
        const bool inr = idx < jtop && idx >= jend;
        go = go && !(inr && (q <= limit || q > qprev));  // deflate.ts:1109; or the bucket's first member was passed
        const bool cand = inr && go;
        qprev = cand ? q : qprev;
        steps += cand ? 1u : 0u;
        pm |= (cand && bu == own) ? 1u << u : 0u;
      }
      // the candidates that passed, in chain order: first strictly longer wins,
      // nice ends the walk (deflate.ts:1100-1105)
      while (pm) {
        const uint32_t u = (uint32_t)__builtin_ctz(pm);
        pm &= pm - 1u;
        uint32_t q = qs[0];
#pragma unroll
        for (uint32_t x = 1; x < 8; x++) q = u == x ? qs[x] : q;
        if (wb[q + bl] == own) {
#if ZS_DW_EXP & 1
          const uint32_t L = maxc;
#else
          const uint32_t L = zs_lcp(X.win, q, p, maxc);
#endif
          if (L > bl) {
            bl = L;
            bq = q;
            up = true;
            own = wb[p + bl];
            if (bl >= nice) {
              go = false;
              pm = 0;
            }
          }
        }
      }
    }
  }
#if ZS_PARSE_PROF
  X.prof[0] += 1;
  X.prof[1] += steps;
#endif
  (void)steps;
  return up ? (bl << 16) | (p - bq) : ey;
}

#define ZS_GATHER 16  // pass C: 64-symbol chunks loaded before any is stored


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
            if (aligned) {  // aligned words holding at least one byte of the stream never leave its pages
              load_m();
              const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
              const uint32_t slast = (n - 1u) >> 2;
              uint32_t sv[WIN / 4];
#pragma unroll
              for (uint32_t j = 0; j < WIN / 4; j++) sv[j] = s4[min(w / 4 + j, slast)];
              const uint32_t bw = s4[w ? w / 4 - 1 : 0u] >> 24;
              store_m();
#pragma unroll
              for (uint32_t j = 0; j < WIN / 4; j++) W.s[j][lane] = sv[j];
              W.b[lane] = w ? bw : 0u;
            } else {
              load_m();
#pragma unroll
              for (uint32_t j = 0; j < WIN / 4; j++) W.s[j][lane] = zs_load_word(src, n, w + 4 * j);
              W.b[lane] = w ? (uint32_t)src[w - 1] : 0u;
              store_m();
            }
          }
          while (st.p < b && st.p < w + WIN) {
            const uint32_t o = st.p - w, q = o - 1;  // in[p - 1] is staged byte o - 1 (o > 0)
            const uint2 e = reinterpret_cast<const uint2*>(&W.m[o >> 1][lane])[o & 1];
            const uint32_t lb = reinterpret_cast<const uint8_t*>(&W.s[(q >> 2) & (WIN / 4 - 1)][lane])[q & 3];
            step(e, o == 0 ? W.b[lane] : lb);
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
    __shared__ zs_parse_win<WIN> W[NWV];                                                                            \
    __shared__ zs_seg_tab T[NWV];                                                                                   \
    __shared__ zs_round_state RS;                                                                                   \
    const uint32_t w_ = threadIdx.x >> 6;                                                                           \
    zs_parse_body<WIN, SEG, NWV>(W[w_], T[w_], RS, in, in_off, in_len, pos_base, blk_base, mres, syms, blocks,      \
                                 streams, scratch, good, lazy);                                                     \
  }
ZS_PARSE_KERNEL(zs_k_parse, 32, ZS_PARSE_SEG, 1)
// two waves per stream, 512-position segments: half the speculative pass per lane (small batches)
ZS_PARSE_KERNEL(zs_k_parse_2w, 32, ZS_PARSE2W_SEG, 2)
// four waves per stream, 256-position segments
ZS_PARSE_KERNEL(zs_k_parse_4w, 32, ZS_PARSE4W_SEG, 4)

// ---------------------------------------------------------- zs_k_parse_dw
// The lazy parse over a demand-mode match table (zs_k_sweep, demand = 1): an
// entry left open (ZS_MORE) gets its full-budget result from a walk (zs_walk)
// where the parse asks for it.  One workgroup of NWV waves per stream, the
// stream in LDS (the walks' candidate bytes), rounds of 64 NWV segments of SEG
// positions (one round for a 64 KiB stream at SEG = 64, NWV = 16):
//   pass A  every lane parses its segment speculatively (as zs_k_parse); a lane
//           that reaches an open entry it must walk stops there, and once every
//           lane has stopped or left its stage the stopped lanes walk together;
//   pass B  every segment's catch-up at once, entered with the speculative end
//           state of the segment before (the round's first with the true
//           state); wave 0 then redoes, in order, the rare segment whose
//           predecessor never synced;
//   pass C  run offsets by a scan over the round, every wave gathers its
//           segments' symbols and cuts blocks in its range.
template <uint32_t WIN, uint32_t NWV>
struct zs_dw_lds {
  uint32_t win[ZS_DW_WIN_WORDS];
  union {
    zs_parse_win<WIN> W[NWV];  // pass A stages
    struct {
      uint32_t F[64 * NWV], NF[64 * NWV], CNT[64 * NWV], START[64 * NWV];
      zs_pstate SP[64 * NWV], AFT[64 * NWV];
    } g;  // passes B, C: per segment of the round
  } u;
  uint32_t off[NWV][65];
  uint32_t WT[NWV];
  uint32_t LS[NWV];
};

struct zs_cu {
  uint32_t nf, from, start;
  zs_pstate after;
};

// the TRUE parse from state c over segment [a, b) until it meets a sync point of
// the segment's speculative parse (pass B); its symbols into fix
template <class R, class Lit>
static __device__ __forceinline__ zs_cu zs_catch_up(zs_pstate c, const zs_pstate& spec_end, uint32_t a, uint32_t b,
                                                    uint32_t n, const uint32_t* sync, uint32_t* fix, const uint2* M,
                                                    int good, int lazy, R&& resolve, Lit&& lit) {
  zs_cu r;
  uint32_t si = 0, sv = sync[0];
  uint4 facc = make_uint4(0, 0, 0, 0);
  r.nf = 0;
  r.from = ZS_NONE;
  r.start = c.p - c.ma;  // a pending literal in[c.p - 1] opens the run
  while (c.p < b) {
    if (c.ml == ZS_MIN_MATCH - 1) {
      const uint32_t key = ((c.p - a) << 1) | c.ma;
      while ((sv >> 16) < key) sv = sync[++si];  // sentinel 0xffffffff stops the scan
      if ((sv >> 16) == key) { r.from = sv & 0xffffu; break; }
    }
    const uint32_t p = c.p;
    const uint32_t v = zs_parse_step(c, resolve(M[p], p, c.ml), lit(p), n, good, lazy);
    if (v != ZS_NONE) {
      const uint32_t m = r.nf & 3u;
      facc.x = m == 0 ? v : facc.x;
      facc.y = m == 1 ? v : facc.y;
      facc.z = m == 2 ? v : facc.z;
      facc.w = m == 3 ? v : facc.w;
      if (++r.nf % 4 == 0) *reinterpret_cast<uint4*>(fix + r.nf - 4) = facc;
    }
  }
  for (uint32_t i = r.nf & ~3u; i < r.nf; i++) fix[i] = (i & 3u) == 0 ? facc.x : (i & 3u) == 1 ? facc.y : facc.z;
  if (r.from == ZS_NONE && b == n && c.ma) fix[r.nf++] = lit(n);  // final deferred literal
  r.after = r.from != ZS_NONE ? spec_end : c;
  return r;
}

template <uint32_t WIN, uint32_t SEG, uint32_t NWV>
static __device__ __forceinline__ void zs_parse_dw_body(zs_dw_lds<WIN, NWV>& S, const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint32_t* __restrict__ in_len,
                                                        const uint64_t* __restrict__ pos_base,
                                                        const uint32_t* __restrict__ blk_base,
                                                        const uint2* __restrict__ mres, uint32_t* __restrict__ syms,
                                                        zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,
                                                        uint32_t* __restrict__ scratch, int good, int lazy,
                                                        const uint16_t* __restrict__ members, int chain, int nice_cfg) {
  using CF = zs_seg_cfg<SEG>;
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  const uint2* M = mres + pos_base[s];
  uint32_t* sy = syms + pos_base[s] + s;  // each stream owns n+1 symbol slots
  uint32_t* scr0 = scratch + (size_t)CF::WORDS * (pos_base[s] / SEG + s);  // segment j of a round: scr0 + j WORDS
  zs_block* blk = blocks + blk_base[s];
  const uint32_t nseg = (n + SEG - 1) / SEG;
  const bool aligned = ((uintptr_t)src & 3u) == 0;
  const bool inwin = n <= 65537u;  // the stream is in LDS (the sweep's streams; longer ones have no open entries)
  const uint8_t* wb = reinterpret_cast<const uint8_t*>(S.win);
#if ZS_PARSE_PROF
  unsigned long long dp[16] = {0};
  unsigned long long wprof[2] = {0, 0};
  const zs_dw_ctx X = {S.win, members + pos_base[s], n, (uint32_t)chain, (uint32_t)chain >> 2, (uint32_t)nice_cfg,
                       wprof};
#else
  const zs_dw_ctx X = {S.win, members + pos_base[s], n, (uint32_t)chain, (uint32_t)chain >> 2, (uint32_t)nice_cfg};
#endif
  auto lit = [&](uint32_t p) -> uint32_t { return p == 0 ? 0u : inwin ? (uint32_t)wb[p - 1] : (uint32_t)src[p - 1]; };
  // an open entry: the walk when the step asks for the full budget, else the chain >> 2 result
  auto resolve = [&](uint2 e, uint32_t p, uint32_t pl) -> uint2 {
    if ((e.x >> 16) == 0xffffu) e.x = pl < (uint32_t)good ? zs_walk(X, p, e.x & 0xffffu, e.y) : e.y;
    return e;
  };

  zs_pstate t = {0, 0, ZS_MIN_MATCH - 1, 0};  // the true parse state entering the round (uniform)
  uint32_t total = 0;                         // symbols written (uniform)
  uint32_t last_sym = 0;                      // the last symbol written (uniform)
  for (uint32_t sr = 0; sr < nseg; sr += 64u * NWV) {
    const uint32_t NT = min(64u * NWV, nseg - sr);  // the round's segments
    const uint32_t r0 = sr + 64u * wave;
    const uint32_t nr = r0 < nseg ? min(64u, nseg - r0) : 0u;
    const bool mine = lane < nr;  // lane owns segment r0 + lane (round index j)
    const uint32_t j = 64u * wave + lane;
    const uint32_t a = mine ? (r0 + lane) * SEG : n, b = mine ? min(n, a + SEG) : n;
    uint32_t* spec = scr0 + (size_t)j * CF::WORDS;
    uint32_t* sync = spec + CF::SPEC;
    uint32_t* fix = sync + CF::SYNC;
    zs_parse_win<WIN>& W = S.u.W[wave];

    // ---- pass A
    DP_T(tA);
    zs_pstate st = {a, 0, ZS_MIN_MATCH - 1, 0};
    uint32_t cnt = 0;
    {
      uint32_t nsync = 0;
      uint4 sacc = make_uint4(0, 0, 0, 0), yacc = make_uint4(0, 0, 0, 0);
      auto step = [&](uint2 e, uint32_t lb) __attribute__((always_inline)) {
        if (st.ml == ZS_MIN_MATCH - 1) {
          const uint32_t y = ((st.p - a) << 17) | (st.ma << 16) | cnt, m = nsync & 3u;
          yacc.x = m == 0 ? y : yacc.x;
          yacc.y = m == 1 ? y : yacc.y;
          yacc.z = m == 2 ? y : yacc.z;
          yacc.w = m == 3 ? y : yacc.w;
          if (++nsync % 4 == 0) *reinterpret_cast<uint4*>(sync + nsync - 4) = yacc;
        }
        const uint32_t v = zs_parse_step(st, e, lb, n, good, lazy);
        if (v != ZS_NONE) {
          const uint32_t m = cnt & 3u;
          sacc.x = m == 0 ? v : sacc.x;
          sacc.y = m == 1 ? v : sacc.y;
          sacc.z = m == 2 ? v : sacc.z;
          sacc.w = m == 3 ? v : sacc.w;
          if (++cnt % 4 == 0) *reinterpret_cast<uint4*>(spec + cnt - 4) = sacc;
        }
      };
      while (__ballot(st.p < b) != 0) {
        const uint32_t w = st.p & ~3u;
        DP_T(tS);
        DP_CNT(8, 1);
        if (st.p < b) {  // stage [w, w + WIN): entries and input bytes (as zs_k_parse)
          const uint4* g = reinterpret_cast<const uint4*>(M);
          const uint32_t glast = ((n + 7u) >> 1) & ~3u;
          uint4 mv[WIN / 2];
#pragma unroll
          for (uint32_t q = 0; q < WIN / 2; q++) mv[q] = g[min(w / 2 + q, glast - 1u)];
          uint32_t sv[WIN / 4];
          uint32_t bw;
          if (aligned) {
            const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
            const uint32_t slast = (n - 1u) >> 2;
#pragma unroll
            for (uint32_t q = 0; q < WIN / 4; q++) sv[q] = s4[min(w / 4 + q, slast)];
            bw = w ? s4[w / 4 - 1] >> 24 : 0u;
          } else {
#pragma unroll
            for (uint32_t q = 0; q < WIN / 4; q++) sv[q] = zs_load_word(src, n, w + 4 * q);
            bw = w ? (uint32_t)src[w - 1] : 0u;
          }
#pragma unroll
          for (uint32_t q = 0; q < WIN / 2; q++) W.m[q][lane] = mv[q];
#pragma unroll
          for (uint32_t q = 0; q < WIN / 4; q++) W.s[q][lane] = sv[q];
          W.b[lane] = bw;
        }
#if ZS_PARSE_PROF
        __builtin_amdgcn_s_waitcnt(0);
#endif
        DP_ADD(10, tS);
        // drain the stage: lanes step until they reach an entry to walk or leave
        // the stage; then the stopped lanes walk together
        bool pend = false;
        uint2 pe = make_uint2(0, 0);
        uint32_t plb = 0;
        for (;;) {
          for (;;) {
            const bool act = !pend && st.p < b && st.p < w + WIN;
            if (__ballot(act) == 0) break;
            DP_CNT(9, 1);
            if (act) {
              const uint32_t o = st.p - w, q = o - 1;
              uint2 e = reinterpret_cast<const uint2*>(&W.m[o >> 1][lane])[o & 1];
              const uint32_t lb = o == 0 ? W.b[lane]
                                         : reinterpret_cast<const uint8_t*>(&W.s[(q >> 2) & (WIN / 4 - 1)][lane])[q & 3];
              if ((e.x >> 16) == 0xffffu) {
                if (st.ml < (uint32_t)good) {
                  pend = true;
                  pe = e;
                  plb = lb;
                } else {
                  step(make_uint2(e.y, e.y), lb);
                }
              } else {
                step(e, lb);
              }
            }
          }
          if (__ballot(pend) == 0) break;
          DP_T(tw);
          DP_CNT(4, 1);
          if (pend) {
            pe.x = zs_walk(X, st.p, pe.x & 0xffffu, pe.y);
            step(pe, plb);
            pend = false;
          }
          DP_ADD(3, tw);
        }
      }
      if (mine) {
        for (uint32_t i = nsync & ~3u; i < nsync; i++) sync[i] = (i & 3u) == 0 ? yacc.x : (i & 3u) == 1 ? yacc.y : yacc.z;
        for (uint32_t i = cnt & ~3u; i < cnt; i++) spec[i] = (i & 3u) == 0 ? sacc.x : (i & 3u) == 1 ? sacc.y : sacc.z;
        sync[nsync] = ZS_NONE;
        if (b == n && st.ma) spec[cnt++] = lit(n);  // final deferred literal (deflate.ts:1429-1432)
      }
    }
    DP_ADD(0, tA);
    __syncthreads();  // the stages are dead: their LDS becomes the round's segment table
    if (mine) {
      S.u.g.SP[j] = st;
      S.u.g.CNT[j] = cnt;
    }
    __syncthreads();

    // ---- pass B: every segment's catch-up at once
    DP_T(tB);
    if (mine) {
      const zs_pstate e = j == 0 ? t : S.u.g.SP[j - 1];
      const zs_cu r = zs_catch_up(e, st, a, b, n, sync, fix, M, good, lazy, resolve, lit);
      S.u.g.F[j] = r.from;
      S.u.g.NF[j] = r.nf;
      S.u.g.START[j] = r.start;
      S.u.g.AFT[j] = r.after;
    }
    __syncthreads();
    // wave 0: a segment whose predecessor never synced was entered with a
    // state that is not the true one: redo it, in order, from the true state
    if (wave == 0) {
      for (uint32_t base = 0; base + 1 < NT; base += 64) {
        uint64_t none = __ballot(base + lane + 1 < NT && S.u.g.F[base + lane] == ZS_NONE);
        while (none) {
          const uint32_t i = (uint32_t)__builtin_ctzll(none);
          const uint32_t jj = base + i + 1;
          if (lane == 0) {
            const uint32_t aa = (sr + jj) * SEG, bb = min(n, aa + SEG);
            uint32_t* sp2 = scr0 + (size_t)jj * CF::WORDS;
            const zs_cu r = zs_catch_up(S.u.g.AFT[jj - 1], S.u.g.SP[jj], aa, bb, n, sp2 + CF::SPEC,
                                        sp2 + CF::SPEC + CF::SYNC, M, good, lazy, resolve, lit);
            S.u.g.F[jj] = r.from;
            S.u.g.NF[jj] = r.nf;
            S.u.g.START[jj] = r.start;
            S.u.g.AFT[jj] = r.after;
          }
          ZS_WAVE_SYNC();
          none &= ~(1ull << i);
          if (i + 1 < 64 && jj + 1 < NT && S.u.g.F[jj] == ZS_NONE) none |= 1ull << (i + 1);
        }
      }
    }
    __syncthreads();
    DP_ADD(1, tB);

    // ---- pass C: splice and block cuts
    DP_T(tC);
    const uint32_t F = mine ? S.u.g.F[j] : 0u, NF = mine ? S.u.g.NF[j] : 0u;
    const uint32_t run = mine ? NF + (F == ZS_NONE ? 0u : cnt - F) : 0u;
    uint32_t incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    S.off[wave][lane] = incl - run;
    if (lane == 63) {
      S.off[wave][64] = R;
      S.WT[wave] = R;
    }
    __syncthreads();
    uint32_t tot0 = total, rtot = 0;
    for (uint32_t v = 0; v < NWV; v++) {
      const uint32_t x = S.WT[v];
      tot0 += v < wave ? x : 0u;
      rtot += x;
    }
    const zs_pstate tend = S.u.g.AFT[NT - 1];  // the true state leaving the round
    const bool last_round = sr + 64u * NWV >= nseg;
    const uint32_t unchecked = last_round && tend.ma ? total + rtot - 1 : ZS_NONE;  // the final deferred literal
    if (nr != 0 && R != 0) {
      uint32_t js = 0, lastv = 0;
      for (uint32_t g0 = 0; g0 < R; g0 += 64 * ZS_GATHER) {
        uint32_t v[ZS_GATHER];
#pragma unroll
        for (int k = 0; k < ZS_GATHER; k++) {
          const uint32_t g = g0 + 64 * k + lane;
          v[k] = 0;
          if (g < R) {
            while (S.off[wave][js + 1] <= g) js++;
            const uint32_t jg = 64u * wave + js;
            const uint32_t i = g - S.off[wave][js], nfj = S.u.g.NF[jg];
            const uint32_t* base = scr0 + (size_t)jg * CF::WORDS;
            v[k] = i < nfj ? base[CF::SPEC + CF::SYNC + i] : base[S.u.g.F[jg] + i - nfj];
          }
        }
#pragma unroll
        for (int k = 0; k < ZS_GATHER; k++) {
          const uint32_t g = g0 + 64 * k + lane;
          if (g < R) sy[tot0 + g] = v[k];
          if (g == R - 1) lastv = v[k];
        }
      }
      const uint32_t ls = (uint32_t)__shfl((int)lastv, (int)((R - 1) & 63u), 64);
      if (lane == 0) S.LS[wave] = ls;
      // block cuts in this wave's range (deflate.ts:336, 1120-1124)
      for (uint32_t gi = (tot0 / ZS_SYM_END + 1) * ZS_SYM_END - 1; gi < tot0 + R; gi += ZS_SYM_END) {
        if (gi == unchecked) continue;
        const uint32_t g = gi - tot0;
        uint32_t js2 = 0;
        while (S.off[wave][js2 + 1] <= g) js2++;
        const uint32_t jg = 64u * wave + js2;
        const uint32_t i = g - S.off[wave][js2], nfj = S.u.g.NF[jg], fj = S.u.g.F[jg];
        const uint32_t* base = scr0 + (size_t)jg * CF::WORDS;
        uint32_t acc = 0, li = 0;
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
        const uint32_t end = S.u.g.START[jg] + acc;
        if (lane == 0) {
          const uint32_t bi = (gi + 1) / ZS_SYM_END - 1;
          blk[bi].in_end = end;
          blk[bi].pad = zs_slides(end - li + 1, n);
        }
      }
    }
    __syncthreads();
    if (rtot) {
      uint32_t hw = 0;
      for (uint32_t v = 0; v < NWV; v++) hw = S.WT[v] ? v : hw;
      last_sym = S.LS[hw];
    }
    total += rtot;
    t = tend;
    __syncthreads();  // the round's tables are read before the next round's stages overwrite them
    DP_ADD(2, tC);
  }
#if ZS_PARSE_PROF
  {
    unsigned long long w0 = wprof[0], w1 = wprof[1];
    for (int d = 32; d >= 1; d >>= 1) {
      w0 += __shfl_xor(w0, d, 64);
      w1 += __shfl_xor(w1, d, 64);
    }
    if (lane == 0) {
      for (int i = 0; i < 16; i++)
        if (dp[i]) atomicAdd(&zs_pp_stat[i], dp[i]);
      atomicAdd(&zs_pp_stat[6], w0);
      atomicAdd(&zs_pp_stat[7], w1);
      if (wave == 0) atomicAdd(&zs_pp_stat[5], 1ull);
    }
  }
#endif
  if (wave != 0) return;

  // ---- block records (wave 0; deflate.ts:1434-1440: the final block takes the rest, possibly empty)
  const bool final_lit = nseg > 0 && t.ma != 0;
  const uint32_t checked = final_lit ? total - 1 : total;
  const uint32_t nflush = checked / ZS_SYM_END;
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
      k.last = (b == nflush ? 1u : 0u) | ((uint64_t)in_start < 32768ull * slides ? 2u : 0u);
    }
    ZS_WAVE_SYNC();
    if (b <= nflush) blk[b] = k;
    ZS_WAVE_SYNC();
  }
  if (lane == 0) {
    streams[s].nsym = total;
    streams[s].nblk = nflush + 1;
  }
}

__global__ __launch_bounds__(64 * ZS_PARSEDW_WAVES) void zs_k_parse_dw(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
    const uint64_t* __restrict__ pos_base, const uint32_t* __restrict__ blk_base, const uint2* __restrict__ mres,
    uint32_t* __restrict__ syms, zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,
    uint32_t* __restrict__ scratch, int good, int lazy, const uint16_t* __restrict__ members, int chain,
    int nice_cfg) {
  __shared__ __attribute__((aligned(16))) zs_dw_lds<8, ZS_PARSEDW_WAVES> S;
  const uint32_t n = in_len[blockIdx.x];
  if (n <= 65537u) {  // the stream in LDS (zero padded)
    const uint8_t* src = in + in_off[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < ZS_DW_WIN_WORDS; i += 64 * ZS_PARSEDW_WAVES) S.win[i] = zs_load_word(src, n, 4 * i);
  }
  __syncthreads();
  zs_parse_dw_body<8, ZS_PARSEDW_SEG, ZS_PARSEDW_WAVES>(S, in, in_off, in_len, pos_base, blk_base, mres, syms, blocks,
                                                        streams, scratch, good, lazy, members, chain, nice_cfg);
}
