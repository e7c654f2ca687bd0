// deflate_parse2.hip -- the lazy-match parse of deflate_slow (deflate.ts:1352-1448)
// for levels 4..9 as two kernels over the per-position match table.
//
// The parse is a serial state machine whose state is (position,
// match_available, prev_length, prev_match).  In a "clean" state
// (prev_length = MIN_MATCH - 1: after every emitted match, after every
// literal that found no match, and at position 0) prev_match is dead, so two
// parses that stand in the same clean state (same position and
// match_available) produce identical symbols from there on.
//
// zs_k_parse_a: one wave per RANGE of PA_LANES segments x PA_SEG positions
//   (2048 positions).  The range's match-table entries and literal bytes are
//   staged in LDS with coalesced loads (the one-wave-per-stream parse read
//   them lane by lane from 64 far-apart places and re-fetched most lines from
//   HBM), then
//     pass 1  lane j parses segment j speculatively from the fresh state at
//             its first position a_j, counting its symbols, up to the first
//             position >= a_{j+1}: end state E_j;
//     merge   lane j (< 63) continues the TRUE parse T from E_j and, in lock
//             step, re-runs lane j+1's speculative parse S from a_{j+1}, until
//             both stand in the same clean state: from there lane j+1's
//             symbols are exact.  It records that state and how many of S's
//             symbols precede it (lane j+1's skip);
//     pass 2  a wave prefix sum of the kept counts gives offsets, and the
//             lanes re-run their parses writing the kept symbols (spec from
//             skip, then T up to the meeting) into the range's compacted run.
//   A lane whose E_j is not in segment j+1 (a match longer than a segment) or
//   whose T and S do not meet inside segment j+1 makes the whole range fall
//   back to one serial parse by lane 0 (zeros-like data, where every step is
//   long).  Lane 63's continuation into the next range is zs_k_parse_b's.
// zs_k_parse_b: one wave per stream.  Lane r >= 1 continues the true parse
//   from range r-1's end state into range r until it meets range r's run
//   (lock step with segment 0's speculative parse, or a recorded clean
//   start state of a later lane), writing the catch-up ("fix") symbols.  A
//   range passed entirely (rare) makes one lane redo the boundaries in order.
//   The wave then splices fixes and runs into the stream's symbol array and
//   closes a block after every 16383rd tallied symbol (deflate.ts:336,
//   FLUSH_BLOCK deflate.ts:1120-1124) from a prefix sum of symbol lengths.
//
// fill_window's slide schedule (deflate.ts:180-190) enters the parse only
// through the NIL head slot at exactly MAX_DIST, a pure
// function of the position (zs_parse_step).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"
#include "zs_parse.h"

#define PA_SEG 32u
#define PA_LANES 64u
#define PA_RANGE (PA_SEG * PA_LANES)
#define PA_STAGE (PA_RANGE + 2u * PA_SEG)  // match-table entries staged per range (merges may run 2 segments past it)
// LDS layouts padded per 64-position segment so that lanes at the same offset
// of their segments hit different banks: 2 entries per segment in Ms, one word
// per 64 bytes in Lb
static __device__ __forceinline__ uint32_t pa_mi(uint32_t i) { return i + 2u * (i / PA_SEG); }
static __device__ __forceinline__ uint32_t pa_li(uint32_t k) { return k + 4u * (k / PA_SEG); }
#define PA_REC 200u                          // record words
#define PA_RUN (PA_RANGE + 512u)             // compacted run / fix capacity (symbols)
#define PA_WORDS (PA_REC + 2u * PA_RUN + 56u)
static_assert(PA_WORDS % 64 == 0, "range scratch blocks are 256-byte aligned");
static_assert(PA_RANGE == ZS_PARSE_RANGE && PA_WORDS == ZS_PARSE_RANGE_WORDS, "scratch layout shared with capi.cpp");
// record word offsets
#define PR_NSYM 0   // symbols in the compacted run
#define PR_FLAGS 1  // bit 0: serial fallback (no per-lane states); bit 1: the run ends with the final literal
#define PR_E 2      // end state of the range's last parse: p, ma, ml, ms
#define PR_CUT 6    // (zs_k_parse_b) first run symbol kept, ZS_NONE: range passed by the true parse
#define PR_NFIX 7   // (zs_k_parse_b) fix symbols preceding the run; bit 31: the fix ends with the final literal

static __device__ __forceinline__ bool pa_clean_eq(const zs_pstate& a, const zs_pstate& b) {
  return a.ml == ZS_MIN_MATCH - 1 && b.ml == ZS_MIN_MATCH - 1 && a.p == b.p && a.ma == b.ma;
}

__global__ __launch_bounds__(64) void zs_k_parse_a(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len,
                                                   const uint64_t* __restrict__ pos_base,
                                                   const uint32_t* __restrict__ range_base,
                                                   const uint2* __restrict__ mres, uint32_t* __restrict__ scratch,
                                                   int good, int lazy) {
  __shared__ __attribute__((aligned(16))) uint2 Ms[PA_STAGE + 2 * (PA_STAGE / PA_SEG + 1)];
  __shared__ __attribute__((aligned(16))) uint8_t Lb[PA_STAGE + 4 * (PA_STAGE / PA_SEG + 1) + 16];  // Lb[pa_li(k)] = in[r0 - 4 + k]
  const int s = blockIdx.y;
  const uint32_t n = in_len[s];
  const uint32_t r = blockIdx.x;
  const uint32_t r0 = r * PA_RANGE;
  if (r0 >= n) return;
  const uint32_t lane = threadIdx.x;
  const uint8_t* src = in + in_off[s];
  const uint2* M = mres + pos_base[s];
  uint32_t* rec = scratch + (size_t)PA_WORDS * (range_base[s] + r);
  uint32_t* run = rec + PA_REC;
  const uint32_t send = min(n, r0 + PA_STAGE);  // staged positions [r0, send)
  {
    // Every load is issued before any store (one memory latency per batch, not
    // one per 512 bytes): 16-byte pieces of the match table (pos_base is
    // 8-aligned and r0 a multiple of 4096, so M + r0 is 16-aligned) and 4-byte
    // words of the input from r0 - 4.
    constexpr uint32_t NM = (PA_STAGE / 2 + 63) / 64, NW = (PA_STAGE + 4 + 255) / 256;
    const uint4* M4 = (const uint4*)(M + r0);
    const uint32_t npair = (send - r0) / 2;
    uint4 mv[NM];
#pragma unroll
    for (uint32_t k = 0; k < NM; k++) {
      const uint32_t i = lane + 64 * k;
      mv[k] = i < npair ? M4[i] : make_uint4(0, 0, 0, 0);
    }
    const bool al = (((uintptr_t)src) & 3u) == 0;
    uint32_t bv[NW];
#pragma unroll
    for (uint32_t k = 0; k < NW; k++) {
      const uint32_t w = lane + 64 * k;  // bytes [r0 - 4 + 4w, +4)
      const int at = (int)r0 - 4 + 4 * (int)w;
      uint32_t v = 0;
      if (4 * w < PA_STAGE + 4) {
        if (al && at >= 0 && (uint32_t)at + 4 <= n) v = *(const uint32_t*)(src + at);
        else
          for (int q = 0; q < 4; q++)
            if (at + q >= 0 && (uint32_t)(at + q) < n) v |= (uint32_t)src[at + q] << (8 * q);
      }
      bv[k] = v;
    }
#pragma unroll
    for (uint32_t k = 0; k < NM; k++) {
      const uint32_t i = lane + 64 * k;
      if (i < npair) *(uint4*)(Ms + pa_mi(2 * i)) = mv[k];
    }
    if ((send - r0) & 1u) Ms[pa_mi(send - r0 - 1)] = M[send - 1];
#pragma unroll
    for (uint32_t k = 0; k < NW; k++) {
      const uint32_t w = lane + 64 * k;
      if (4 * w < PA_STAGE + 4) *(uint32_t*)(Lb + pa_li(4 * w)) = bv[k];
    }
  }
  __syncthreads();
  auto step = [&](zs_pstate& st) -> uint32_t {  // one deflate_slow iteration at st.p (staged)
    const uint32_t p = st.p;
    const uint2 e = Ms[pa_mi(p - r0)];
    asm volatile("" ::"v"(e.x), "v"(e.y));  // both halves in one read, before the branches
    return zs_parse_step(st, e, Lb[pa_li(p - r0 + 3)], n, good, lazy);
  };
  const uint32_t rend = min(n, r0 + PA_RANGE);
  const uint32_t a = r0 + lane * PA_SEG;  // this lane's segment [a, b)
  const uint32_t b = min(n, a + PA_SEG);
  const bool act = a < n;
  // ---- pass 1: speculative parse, counting
  zs_pstate E = {a, 0, ZS_MIN_MATCH - 1, 0};
  uint32_t nspec = 0;
  if (act) {
    while (E.p < b) nspec += step(E) != ZS_NONE;
    if (b == n && E.ma) nspec++;  // final deferred literal (deflate.ts:1429-1432)
  }
  // ---- merge: T (this lane's parse continued from E) meets the next lane's
  // parse S (from its first position, continued past its segment if need be)
  const uint32_t a1 = a + PA_SEG;
  const bool merges = act && lane < PA_LANES - 1 && a1 < rend;
  uint32_t sy = E.p, sk = 0, nt = 0;  // meeting position, S symbols before it, T symbols
  zs_pstate Tm = E;                   // the meeting state
  bool ok = true;
  if (merges) {
    const uint32_t cap = min(min(n, a1 + 3 * PA_SEG), r0 + PA_STAGE);
    zs_pstate T = E, S = {a1, 0, ZS_MIN_MATCH - 1, 0};
    ok = false;
    for (;;) {
      if (pa_clean_eq(T, S) || (T.p >= n && S.p >= n && T.ma == S.ma)) { ok = true; break; }
      if (S.p >= cap || T.p >= cap) break;
      const bool adv_t = T.p <= S.p, adv_s = S.p <= T.p;
      if (adv_t) nt += step(T) != ZS_NONE;
      if (adv_s) sk += step(S) != ZS_NONE;
    }
    sy = S.p;
    Tm = T;
  }
  const uint32_t out = nspec + nt;  // this lane's path: spec, then T up to the meeting
  // ---- where the true path enters each lane's path (wave-uniform scan over
  // the lanes): position Y and the number of the path's symbols before it.
  // If Y lies past lane k's own meeting, lane k's path has already merged into
  // lane k+1's: lane k contributes nothing and the entry moves on.
  // Common case: every meeting lies inside the next lane's path, so lane k
  // is entered at lane k-1's meeting (two shuffles); otherwise one serial pass.
  const uint32_t sk_up = __shfl_up(sk, 1, 64), sy_up = __shfl_up(sy, 1, 64);  // every lane shuffles
  uint32_t my_skip = lane == 0 ? 0u : sk_up;
  const uint32_t my_y = lane == 0 ? r0 : sy_up;
  bool contrib = act;
  if (__builtin_amdgcn_ballot_w64(act && my_y > (merges ? sy : E.p)) != 0) {
    uint32_t Y = r0, skip = 0;
    contrib = false;
    for (uint32_t k = 0; k < PA_LANES; k++) {
      const uint32_t k_act = __builtin_amdgcn_readlane((uint32_t)act, k);
      if (!k_act) break;
      const uint32_t k_merges = __builtin_amdgcn_readlane((uint32_t)merges, k);
      const uint32_t k_y = __builtin_amdgcn_readlane(sy, k), k_sk = __builtin_amdgcn_readlane(sk, k);
      const uint32_t k_out = __builtin_amdgcn_readlane(out, k);
      if (Y <= k_y) {
        if (lane == k) { my_skip = skip; contrib = true; }
        if (k_merges) { Y = k_y; skip = k_sk; }
      } else {
        if (!k_merges) ok = false;  // the true path would join past the range's end
        skip = k_sk + (skip - k_out);
      }
    }
  }
  if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
    const uint32_t cnt = contrib ? out - my_skip : 0u;
    uint32_t x = cnt;  // inclusive scan of the kept counts
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    const uint32_t off = x - cnt;
    const uint32_t total = __builtin_amdgcn_readlane(x, 63);
    // ---- pass 2: re-run, writing the kept symbols of the path
    if (act) {
      zs_pstate st = {a, 0, ZS_MIN_MATCH - 1, 0};
      uint32_t i = 0, o = off;
      const uint32_t skip = contrib ? my_skip : 0xffffffffu;
      while (st.p < b) {
        const uint32_t v = step(st);
        if (v != ZS_NONE) {
          if (i >= skip) run[o++] = v;
          i++;
        }
      }
      const bool fin = b == n && st.ma;
      if (fin) {
        if (i >= skip) run[o++] = src[n - 1];
        i++;
      }
      if (nt) {  // T from E to the meeting state
        zs_pstate T = st;
        while (!(T.p == Tm.p && T.ma == Tm.ma && T.ml == Tm.ml)) {
          const uint32_t v = step(T);
          if (v != ZS_NONE) {
            if (i >= skip) run[o++] = v;
            i++;
          }
        }
      }
      if (b >= rend) {  // the range's last segment: end state and final-literal flag
        rec[PR_NSYM] = total;
        rec[PR_FLAGS] = fin ? 2u : 0u;
        rec[PR_E] = st.p;
        rec[PR_E + 1] = st.ma;
        rec[PR_E + 2] = st.ml;
        rec[PR_E + 3] = st.ms;
      }
    }
    return;
  }
  // ---- serial fallback: lane 0 parses the whole range from its first position
  if (lane == 0) {
    zs_pstate st = {r0, 0, ZS_MIN_MATCH - 1, 0};
    uint32_t o = 0;
    while (st.p < rend) {
      const uint32_t v = step(st);
      if (v != ZS_NONE) run[o++] = v;
    }
    const bool fin = rend == n && st.ma;
    if (fin) run[o++] = src[n - 1];
    rec[PR_NSYM] = o;
    rec[PR_FLAGS] = 1u | (fin ? 2u : 0u);
    rec[PR_E] = st.p;
    rec[PR_E + 1] = st.ma;
    rec[PR_E + 2] = st.ml;
    rec[PR_E + 3] = st.ms;
  }
}

__global__ __launch_bounds__(64) void zs_k_parse_b(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len,
                                                   const uint64_t* __restrict__ pos_base,
                                                   const uint32_t* __restrict__ blk_base,
                                                   const uint32_t* __restrict__ range_base,
                                                   const uint2* __restrict__ mres, uint32_t* __restrict__ syms,
                                                   zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,
                                                   uint32_t* __restrict__ scratch, int good, int lazy) {
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  const uint2* M = mres + pos_base[s];
  uint32_t* sy = syms + pos_base[s] + s;  // each stream owns n+1 symbol slots
  uint32_t* scr = scratch + (size_t)PA_WORDS * range_base[s];
  zs_block* blk = blocks + blk_base[s];
  const uint32_t nr = (n + PA_RANGE - 1) / PA_RANGE;
  auto R = [&](uint32_t r) -> uint32_t* { return scr + (size_t)PA_WORDS * r; };
  auto step = [&](zs_pstate& st) -> uint32_t {
    const uint32_t p = st.p;
    return zs_parse_step(st, M[p], p > 0 ? src[p - 1] : 0u, n, good, lazy);
  };
  // Continues the true parse T into range r, writing fix symbols to range r's
  // fix region, until it meets range r's run.  Returns the run offset to
  // resume at, or ZS_NONE when T passed the whole range (T then stands at
  // the range's end).  fin: T emitted the final literal.
  auto join = [&](zs_pstate& T, uint32_t r, uint32_t& nf, bool& fin) -> uint32_t {
    uint32_t* rec = R(r);
    uint32_t* fix = rec + PA_REC + PA_RUN;
    const uint32_t r0 = r * PA_RANGE, rend = min(n, r0 + PA_RANGE);
    nf = 0;
    fin = false;
    zs_pstate S = {r0, 0, ZS_MIN_MATCH - 1, 0};  // the range's run is the parse from r0, continued
    uint32_t sk = 0;
    for (;;) {
      if (pa_clean_eq(T, S)) return sk;
      if (T.p >= rend) break;
      const bool adv_t = T.p <= S.p, adv_s = S.p <= T.p;
      if (adv_t) {
        const uint32_t v = step(T);
        if (v != ZS_NONE) fix[nf++] = v;
      }
      if (adv_s) sk += step(S) != ZS_NONE;
    }
    if (rend == n && T.ma) {
      fix[nf++] = src[n - 1];
      fin = true;
    }
    return ZS_NONE;
  };
  // ---- boundaries, one lane each
  bool bad = false;
  for (uint32_t r = 1 + lane; r < nr; r += 64) {
    const uint32_t* prv = R(r - 1);
    zs_pstate T = {prv[PR_E], prv[PR_E + 1], prv[PR_E + 2], prv[PR_E + 3]};
    uint32_t nf;
    bool fin;
    const uint32_t c = join(T, r, nf, fin);
    R(r)[PR_CUT] = c;
    R(r)[PR_NFIX] = nf | (fin ? 0x80000000u : 0u);
    bad |= c == ZS_NONE;
  }
  if (lane == 0 && nr > 0) {
    R(0)[PR_CUT] = 0;
    R(0)[PR_NFIX] = 0;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (__builtin_amdgcn_ballot_w64(bad) != 0) {
    // a range was passed entirely: redo the boundaries in order from the
    // first such one, carrying the true state across passed ranges
    if (lane == 0) {
      uint32_t r = 1;
      while (r < nr && R(r)[PR_CUT] != ZS_NONE) r++;
      const uint32_t* prv = R(r - 1);
      zs_pstate T = {prv[PR_E], prv[PR_E + 1], prv[PR_E + 2], prv[PR_E + 3]};
      for (; r < nr; r++) {
        uint32_t nf;
        bool fin;
        const uint32_t c = join(T, r, nf, fin);
        R(r)[PR_CUT] = c;
        R(r)[PR_NFIX] = nf | (fin ? 0x80000000u : 0u);
        if (c != ZS_NONE) {
          const uint32_t* rec = R(r);
          T = {rec[PR_E], rec[PR_E + 1], rec[PR_E + 2], rec[PR_E + 3]};
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  // ---- splice: fix_r then run_r[cut_r, nsym_r) for every range, in order
  uint32_t grand = 0;
  bool final_lit = false;  // the stream's last symbol is the final deferred literal (deflate.ts:1429-1432)
  for (uint32_t r = 0; r < nr; r++) {
    const uint32_t* rec = R(r);
    const uint32_t c = rec[PR_CUT], nf = rec[PR_NFIX] & 0x7fffffffu;
    const uint32_t kept = c == ZS_NONE ? 0u : rec[PR_NSYM] - c;
    grand += nf + kept;
    if (r == nr - 1) final_lit = c == ZS_NONE ? (rec[PR_NFIX] >> 31) != 0 : ((rec[PR_FLAGS] & 2u) != 0 && kept > 0);
  }
  const uint32_t unchecked = final_lit ? grand - 1 : ZS_NONE;  // global index of the final literal
  uint32_t total = 0, pos = 0, last_start = 0;
  for (uint32_t r = 0; r < nr; r++) {
    const uint32_t* rec = R(r);
    const uint32_t c = rec[PR_CUT];
    for (int piece = 0; piece < 2; piece++) {
      const uint32_t* base = piece == 0 ? rec + PA_REC + PA_RUN : rec + PA_REC + (c == ZS_NONE ? 0u : c);
      const uint32_t cnt = piece == 0 ? (rec[PR_NFIX] & 0x7fffffffu) : (c == ZS_NONE ? 0u : rec[PR_NSYM] - c);
      for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
        const uint32_t i = c0 + lane;
        const uint32_t v = i < cnt ? base[i] : 0u;
        const uint32_t len = i < cnt ? ((v & 0x80000000u) ? ((v >> 16) & 0xffu) + ZS_MIN_MATCH : 1u) : 0u;
        uint32_t x = len;  // inclusive scan of symbol lengths
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(x, d, 64);
          if (lane >= (uint32_t)d) x += y;
        }
        if (i < cnt) {
          const uint32_t gi = total + lane;
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
  // ---- block records (deflate.ts:1434-1440: the final block takes the rest, possibly empty)
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
