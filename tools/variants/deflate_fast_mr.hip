// deflate_fast_mr.hip -- the greedy parser of levels 1..3 (deflate_fast,
// deflate.ts:1281-1350) without the reference's head[] / prev[] tables.
//
// zs_k_fast (deflate_fast.hip) keeps head[] and prev[] (64 KiB each, LDS) so
// that its chain walks follow the reference's links: with the 32 KiB input
// ring that is a whole CU's LDS, one stream per CU.  Here the chains come from
// the bucket sort of levels 4..9 instead (zs_k_bucket, with ranks): in a
// window's member array -- positions sorted by (hash, position) -- the
// predecessors of member k in its bucket are every EARLIER position with the
// same hash, most recent first: the chain of the SUPERSET in which every
// position is inserted.  deflate_fast's true chain is that chain minus the
// positions it did not insert (the insides of matches longer than max_lazy,
// deflate.ts:1310-1322), so a walk reads the superset chain as a contiguous run
// of members and filters it:
//   * positions before the group: a bitmap of the truly inserted ones (32 K
//     bits, LDS, written as each group's parse is decided) -- exact;
//   * positions inside the group: taken speculatively and recorded (vis), then
//     checked by the replay exactly as in zs_k_fast (a step is exact iff every
//     in-group position its walk met was truly inserted);
//   * the slide of fill_window (deflate.ts:180-190) only turns head / prev
//     entries below the new window base into NIL, and every candidate lies
//     within MAX_DIST, so "a candidate at or below the base ends the chain" is
//     the whole of it.
// Each lane loads the first ZS_FM_R superset entries of its position (a 68-byte
// run of u16 members); a walk needing more is left to the replay's slow step
// (rare at levels 1..2: tools/emu/emu_fast_rec.c counts them), which walks the
// true chain with the whole wave, 64 entries per round.  LDS: the input ring and
// the bitmap, 37 KiB, so four streams share a CU.  Group structure, replay and
// block cuts are zs_k_fast's (deflate_fast.hip); CPU model of the walks:
// tools/emu/emu_fast_rec.c (tests/test_emu_fast.py).
#include <hip/hip_runtime.h>
#include <type_traits>
#include "zs_common.h"
#include "zs_kernels.h"

#define ZS_FM_R 32u            // superset entries a lane walk holds
#define ZS_FM_LONG 0xffffu     // a lane result longer than nice + 32: extended by the replay

#ifdef ZS_FM_PROF  // cycle profile per phase (timing experiments only; tools/dbg/fm_prof.py)
#define FM_T(k)                                                   \
  do {                                                            \
    const unsigned long long t_ = __builtin_readcyclecounter();   \
    fm_acc[k] += t_ - fm_last;                                    \
    fm_last = t_;                                                 \
  } while (0)
#else
#define FM_T(k) do {} while (0)
#endif

struct zs_fm_lds {
  uint32_t ring[8192];  // input byte x at byte (x & 32767)
  uint32_t bits[1024];  // truly inserted positions: x at bit (x & 32767)
  uint32_t scr[16];     // a slow step's first ZS_FM_R entries
};

template <int NW>
__global__ __launch_bounds__(64) void zs_k_fast_mr(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len,
                                                   const uint64_t* __restrict__ pos_base,
                                                   const uint32_t* __restrict__ blk_base, uint32_t* __restrict__ syms,
                                                   zs_block* __restrict__ blocks, zs_stream* __restrict__ streams,
                                                   int chain, int lazy, int nice_cfg,
                                                   const uint16_t* __restrict__ members,
                                                   const uint2* __restrict__ mres,
                                                   const zs_sweep_seg* __restrict__ segs,
                                                   const uint32_t* __restrict__ win0) {
  __shared__ zs_fm_lds L;
  const int s = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = in_len[s];
  const uint8_t* src = in + in_off[s];
  uint32_t* sy = syms + pos_base[s] + s;
  zs_block* blk = blocks + blk_base[s];
  const uint2* kr_of = mres + pos_base[s];
  const zs_sweep_seg* sg = segs + win0[s];
  for (uint32_t i = lane; i < 1024; i += 64) L.bits[i] = 0;
  const uint8_t* ringb = reinterpret_cast<const uint8_t*>(L.ring);

  // ring fill: E = end of the ring's bytes; pf = bytes [P, P + 256) (4 per lane), nx = [P + 256, P + 512) in flight
  uint32_t E = 0, P = 0;
  uint32_t pf = zs_load_word(src, n, 4 * lane), nx = zs_load_word(src, n, 256 + 4 * lane);
  auto fill_to = [&](uint32_t want) {
    while (E < want) {
      if ((lane >> 4) == ((E - P) >> 6)) L.ring[((P >> 2) + lane) & 8191u] = pf;
      E += 64;
      if (E == P + 256) {
        P += 256;
        pf = nx;
        nx = zs_load_word(src, n, P + 256 + 4 * lane);
      }
    }
  };
  // the window (zs_k_bucket's) holding position q's chain: its member array and first position
  auto window_of = [&](uint32_t q, const uint16_t*& mb, uint32_t& wb) {
    const uint32_t wi = (n <= 65537u || q < ZS_SEG_FIRST) ? 0u : 1u + (q - ZS_SEG_FIRST) / ZS_SEG_OWN;
    const zs_sweep_seg G = sg[wi];
    mb = members + G.mb;
    wb = G.base;
  };

  uint32_t base = 0, p = 0;
  uint32_t nsym = 0, in_blk = 0, nflush = 0, blk_start = 0;
  // prefetched runs of positions [pf0, pf0 + 128): position pf0 + 64 t + lane in set t of this lane
  uint32_t pf0 = 0xffffffffu, Pkr[2] = {0u, 0u}, Pwb[2] = {0u, 0u}, Pw[2][ZS_FM_R / 2 + 1];
#pragma unroll
  for (int i = 0; i <= (int)(ZS_FM_R / 2); i++) Pw[0][i] = Pw[1][i] = 0u;
  auto close_block = [&](uint32_t end, uint32_t last) {
    if (lane == 0) {
      zs_block b;
      b.sym_start = nsym - in_blk;
      b.sym_count = in_blk;
      b.in_start = blk_start;
      b.in_end = end;
      b.type = 0; b.hdr_bits = 0; b.data_bits = 0; b.pad = 0; b.bit_off = 0; b.bit_end = 0;
      b.last = last | (blk_start < base ? 2u : 0u);
      blk[nflush] = b;
    }
    nflush++;
    in_blk = 0;
    blk_start = end;
  };
  // exact match length at scan position a (wave-uniform) against candidate c < a, capped at maxc:
  // 64 bytes per ballot, the first 64 from the ring, further ones from memory
  auto exact_len = [&](uint32_t a, uint32_t c, uint32_t maxc) -> uint32_t {
    uint32_t k = 0;
    uint64_t neq = __ballot(ringb[(a + lane) & 32767u] != ringb[(c + lane) & 32767u] || lane >= maxc);
    while (neq == 0 && k + 64 < maxc) {
      k += 64;
      const uint32_t sb = a + k + lane < n ? src[a + k + lane] : 0x100u;
      const uint32_t mb = c + k + lane < n ? src[c + k + lane] : 0x1ffu;
      neq = __ballot(mb != sb || k + lane >= maxc);
    }
    k += neq ? (uint32_t)__builtin_ctzll(neq) : 64u;
    return k < maxc ? k : maxc;
  };
  auto inserted = [&](uint32_t c) -> bool { return ((L.bits[(c >> 5) & 1023u] >> (c & 31u)) & 1u) != 0u; };
#ifdef ZS_FM_PROF
  unsigned long long fm_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fm_last = __builtin_readcyclecounter();
  uint32_t fm_groups = 0, fm_slow = 0, fm_inc = 0, fm_miss = 0;
#endif

  while (p < n) {
    // fill_window slide (deflate.ts:180-190), same schedule as deflate_slow: only the base moves
    const uint32_t m = min(n, base + 65536u);
    if (p - base >= ZS_SLIDE_AT && m - p < ZS_MIN_LOOKAHEAD) {
      base += 32768u;
      continue;
    }
    FM_T(7);
    const uint32_t g0 = p;
#ifdef ZS_FM_PROF
    fm_groups++;
#endif
    uint32_t tslide = base + ZS_SLIDE_AT;
    if (m >= ZS_MIN_LOOKAHEAD - 1 && m - (ZS_MIN_LOOKAHEAD - 1) > tslide) tslide = m - (ZS_MIN_LOOKAHEAD - 1);
    const uint32_t g1 = min(min(g0 + 64u - (uint32_t)lazy, tslide), n);
    const uint32_t q = g0 + lane;
    const bool ok = q + 2 < n;  // INSERT_STRING needs lookahead >= MIN_MATCH (deflate.ts:1296)
    const bool walk = ok && q < g1;
    // ---- 1. the lane's superset run: member index and rank (zs_k_bucket), then ZS_FM_R entries -- from
    //         the sets prefetched during the group before (positions [pf0, pf0 + 128), lane x - pf0 mod 64),
    //         else loaded here
    uint32_t kr, wb, w[ZS_FM_R / 2 + 1];
    {
      const uint32_t o = q - pf0;
      const bool hit = pf0 != 0xffffffffu && o < 128u;
      const int sl = (int)((o & 63u) * 4u);
      const bool hi = o >= 64u;
      auto gat = [&](uint32_t v0, uint32_t v1) -> uint32_t {
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v0);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v1);
        return hi ? a1 : a0;
      };
      kr = gat(Pkr[0], Pkr[1]);
      wb = gat(Pwb[0], Pwb[1]);
#pragma unroll
      for (int i = 0; i <= (int)(ZS_FM_R / 2); i++) w[i] = gat(Pw[0][i], Pw[1][i]);
#ifdef ZS_FM_PROF
      if (walk && !hit) fm_miss++;
#endif
      if (walk && !hit) {
        const uint16_t* mbq;
        window_of(q, mbq, wb);
        kr = kr_of[q].x;
        const uint32_t kq = kr & 0xffffu;
        const uint32_t* w4 = reinterpret_cast<const uint32_t*>(mbq + (((int32_t)kq - (int32_t)ZS_FM_R) & ~1));
#pragma unroll
        for (int i = 0; i <= (int)(ZS_FM_R / 2); i++) w[i] = w4[i];  // (dword loads: the run is 4-byte aligned only)
      }
      if (!walk) kr = 0;
    }
    FM_T(0);
    fill_to(g0 + 160u);
    // the next sets' first half: member index / rank and window of positions [g1, g1 + 128)
    uint32_t Nkr[2], Nwb[2];
    const uint16_t* Nmb[2];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const uint32_t x = g1 + 64u * t + lane;
      Nkr[t] = 0;
      Nwb[t] = 0;
      Nmb[t] = members;
      if (x + 2 < n) {
        window_of(x, Nmb[t], Nwb[t]);
        Nkr[t] = kr_of[x].x;
      }
    }
    FM_T(1);
    const uint32_t k = kr & 0xffffu, rank = kr >> 16;
    uint32_t Ew[ZS_FM_R / 2];  // entry j (member k - 1 - j) in half 31 - j
    {
      // the 17 words from the even member index at or below k - 32 (the array is padded by 32 members below)
      const uint32_t sh = 16u * (k & 1u);
#pragma unroll
      for (int i = 0; i < (int)(ZS_FM_R / 2); i++) Ew[i] = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
    }
    auto entry = [&](uint32_t j) -> uint32_t {  // j compile-time after unrolling
      const uint32_t h = ZS_FM_R - 1u - j;
      return (Ew[h >> 1] >> (16u * (h & 1u))) & 0xffffu;
    };

    // ---- 2. the walks: the superset run filtered (bitmap before the group, speculative inside it)
    const uint32_t look = n - q;  // wraps for lanes past the end; they are inactive
    const uint32_t srel = q - base;
    const uint32_t maxc = min(look, (uint32_t)ZS_MAX_MATCH), nice = min(look, (uint32_t)nice_cfg);
    const uint32_t capn = min(nice, maxc);
    uint32_t best = ZS_MIN_MATCH - 1, bms = 0;
    uint64_t vis = 0;
    uint32_t sw[NW];
    {
      uint32_t A[NW + 1];
#pragma unroll
      for (int j = 0; j <= NW; j++) A[j] = L.ring[((q >> 2) + j) & 8191u];
#pragma unroll
      for (int j = 0; j < NW; j++) sw[j] = __builtin_amdgcn_alignbyte(A[j + 1], A[j], q & 3u);
    }
    // first differing byte of the W words at scan S and candidate c, 4 W if none (all loads issued first)
    auto diff_at = [&](uint32_t c, const uint32_t* S, auto Wc) -> uint32_t {
      constexpr int W = decltype(Wc)::value;
      uint32_t A[W + 1];
#pragma unroll
      for (int j = 0; j <= W; j++) A[j] = L.ring[((c >> 2) + j) & 8191u];
      uint32_t len = 4u * W;
#pragma unroll
      for (int j = W - 1; j >= 0; j--) {
        const uint32_t x = __builtin_amdgcn_alignbyte(A[j + 1], A[j], c & 3u) ^ S[j];
        len = x ? 4u * j + ((uint32_t)__builtin_ctz(x) >> 3) : len;
      }
      return len;
    };
    using NWc = std::integral_constant<int, NW>;
    // (a) every entry's status at once (ZS_FM_R bitmap reads in flight): the truly inserted ones, where the
    //     chain ends (the bucket's end, NIL at or below the base, past MAX_DIST: later entries are older still),
    //     and entries at exactly MAX_DIST (the head may be there, deflate.ts:1376; a later step may not,
    //     deflate.ts:1109: pos > limit)
    uint32_t tmask = 0, emask = 0, dmask = 0;
    {
      uint32_t bw[ZS_FM_R];  // (all the bitmap words read before any is tested)
#pragma unroll
      for (uint32_t j = 0; j < ZS_FM_R; j++) bw[j] = L.bits[((wb + entry(j)) >> 5) & 1023u];
#pragma unroll
      for (uint32_t j = 0; j < ZS_FM_R; j++) {
        const uint32_t c = wb + entry(j);
        const bool valid = walk && j < rank && c > base;
        const uint32_t d = q - c;
        const bool tr = valid && (c >= g0 || ((bw[j] >> (c & 31u)) & 1u) != 0u);
        tmask |= tr ? 1u << j : 0u;
        emask |= (!valid || d > ZS_MAX_DIST) ? 1u << j : 0u;
        dmask |= (valid && d == ZS_MAX_DIST) ? 1u << j : 0u;
      }
    }
    FM_T(2);
    const uint32_t e0 = emask ? (uint32_t)__builtin_ctz(emask) : ZS_FM_R;
    uint32_t cand = tmask & (e0 >= 32u ? 0xffffffffu : (1u << e0) - 1u);
    if (cand) {  // after the head, the first entry at exactly MAX_DIST ends the chain
      const uint32_t f = (uint32_t)__builtin_ctz(cand);
      const uint32_t dl = dmask & ~((2u << f) - 1u);
      if (dl) cand &= ((1u << __builtin_ctz(dl)) - 1u) | (1u << f);
    }
    // the run ran out with the chain still live (no end among the ZS_FM_R entries, more in the bucket): unless
    // the steps below end it first (nice, budget), the replay re-walks it
    const bool open = walk && e0 >= ZS_FM_R && rank > ZS_FM_R && (dmask & ~(cand ? (2u << __builtin_ctz(cand)) - 1u : 0u)) == 0u;
    // (b) the steps: each lane's candidates in order, one per round (the entry by a select tree over Ew)
    auto entry_rt = [&](uint32_t j) -> uint32_t {
      const uint32_t h = ZS_FM_R - 1u - j, x = h >> 1;
      uint32_t l1[8], l2[4], l3[2];
#pragma unroll
      for (int i = 0; i < 8; i++) l1[i] = (x & 1u) ? Ew[2 * i + 1] : Ew[2 * i];
#pragma unroll
      for (int i = 0; i < 4; i++) l2[i] = (x & 2u) ? l1[2 * i + 1] : l1[2 * i];
#pragma unroll
      for (int i = 0; i < 2; i++) l3[i] = (x & 4u) ? l2[2 * i + 1] : l2[2 * i];
      const uint32_t wv = (x & 8u) ? l3[1] : l3[0];
      return (wv >> (16u * (h & 1u))) & 0xffffu;
    };
    bool act = cand != 0u;
    bool budget_left = true;
    for (uint32_t t = 0; t < (uint32_t)chain; t++) {
      if (__ballot(act) == 0) break;
      const uint32_t j = act ? (uint32_t)__builtin_ctz(cand) : 0u;
      cand &= cand - 1u;
      const uint32_t c = wb + entry_rt(j);
      const uint32_t len = min(diff_at(c, sw, NWc{}), capn);
      vis |= act && c >= g0 ? 1ull << ((c - g0) & 63u) : 0ull;
      const bool better = act && len > best;
      best = better ? len : best;
      bms = better ? c - base : bms;
      const bool stop = better && len >= nice;
      budget_left = budget_left && !(act && t + 1u == (uint32_t)chain);
      act = act && !stop && cand != 0u;
      if (stop) budget_left = false;
    }
    const bool inc = open && budget_left;
    FM_T(3);
    // the next sets' second half: the runs themselves (they arrive during the replay)
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const uint32_t kx = Nkr[t] & 0xffffu;
      const uint32_t* w4 = reinterpret_cast<const uint32_t*>(Nmb[t] + (((int32_t)kx - (int32_t)ZS_FM_R) & ~1));
#pragma unroll
      for (int i = 0; i <= (int)(ZS_FM_R / 2); i++) Pw[t][i] = Nkr[t] ? w4[i] : 0u;
      Pkr[t] = Nkr[t];
      Pwb[t] = Nwb[t];
    }
    pf0 = g1;
    FM_T(4);
    // a result at nice: its exact length from 32 more bytes per lane; ZS_FM_LONG if they all match too
    if (best >= nice && best >= ZS_MIN_MATCH && nice < maxc) {
      const uint32_t o = 4u * NW;
      uint32_t S2[8], A2[9];
#pragma unroll
      for (int j = 0; j < 9; j++) A2[j] = L.ring[(((q + o) >> 2) + j) & 8191u];
#pragma unroll
      for (int j = 0; j < 8; j++) S2[j] = __builtin_amdgcn_alignbyte(A2[j + 1], A2[j], (q + o) & 3u);
      const uint32_t e = o + diff_at(base + bms + o, S2, std::integral_constant<int, 8>{});
      best = e >= maxc ? maxc : (e < o + 32u ? e : ZS_FM_LONG);
    }

    // ---- 3. replay of the group (zs_k_fast's): pointer doubling over the lanes' next-step links, the
    //         path's insertions, the first step whose result does not hold, a slow step there
    const uint32_t hw = L.ring[(q >> 2) & 8191u] >> (8u * (q & 3u));  // the literal (ring bytes up to g0 + 160)
    const bool isM = best >= ZS_MIN_MATCH;
    const uint32_t sym = isM ? 0x80000000u | ((best - ZS_MIN_MATCH) << 16) | (srel - bms) : (hw & 0xffu);
    const uint32_t shortc = isM && best != ZS_FM_LONG && best <= (uint32_t)lazy && n - (q + best) >= ZS_MIN_MATCH
                                ? best - 1u : 0u;
    const uint32_t pk = min(lane + (isM ? best : 1u), 511u) | (shortc << 10) |
                        (best == ZS_FM_LONG || inc ? 0x4000u : 0u);
    const uint32_t vlo = (uint32_t)vis, vhi = (uint32_t)(vis >> 32);
    const uint64_t okm = __ballot(ok);
    uint64_t tm = 0;  // truly inserted lanes
    const uint32_t j1 = g1 - g0;
    const uint32_t nextv = pk & 511u, shc = (pk >> 10) & 15u;
    const bool slow_lane = (pk & 0x4000u) != 0u;
    auto put = [&](uint32_t v) {  // one symbol of a slow step
      if (lane == 0) sy[nsym] = v;
      nsym++;
      in_blk++;
    };
    auto flush = [&](uint64_t path) {  // store the path's symbols in order; close a block on its 16383rd
      const uint32_t cnt = (uint32_t)__builtin_popcountll(path);
      if (cnt == 0) return;
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(path >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)path, 0u));
      if ((path >> lane) & 1ull) sy[nsym + rk] = sym;
      if (in_blk + cnt >= ZS_SYM_END) {
        const uint32_t kk = ZS_SYM_END - in_blk;  // symbols up to and including the cut
        uint64_t mm = path;
        for (uint32_t t = 1; t < kk; t++) mm &= mm - 1;
        const uint32_t c = (uint32_t)__builtin_ctzll(mm);
        nsym += kk;
        in_blk += kk;
        close_block(g0 + (uint32_t)__builtin_amdgcn_readlane((int)nextv, (int)c), 0);
        nsym += cnt - kk;
        in_blk += cnt - kk;
      } else {
        nsym += cnt;
        in_blk += cnt;
      }
    };
    uint32_t slo, shi;
    {
      uint64_t S = 1ull << lane;
      uint32_t J = nextv < j1 ? nextv : lane;
#pragma unroll
      for (int t = 0; t < 6; t++) {
        const int a = (int)(J * 4u);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)S);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(S >> 32));
        J = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)J);
        S |= ((uint64_t)hi << 32) | lo;
      }
      slo = (uint32_t)S;
      shi = (uint32_t)(S >> 32);
    }
    uint32_t j = p - g0;
    while (j < j1) {
      const uint64_t path = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)shi, (int)j) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)slo, (int)j);
      const uint32_t jj = (uint32_t)__builtin_amdgcn_readlane((int)nextv, (int)(63u - (uint32_t)__builtin_clzll(path)));
      const bool onp = (path >> lane) & 1ull;
      const uint64_t le = path & (lane == 63u ? ~0ull : (2ull << lane) - 1ull);
      const uint32_t owner = le ? 63u - (uint32_t)__builtin_clzll(le) : 0u;
      const uint32_t osc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(owner * 4u), (int)shc);
      const bool inside = !onp && le != 0 && lane - owner <= osc;
      const uint64_t tmn = tm | __ballot((onp && ok) || inside);
      const uint64_t bad = __ballot(onp && (slow_lane || (vis & ~tmn) != 0));
      if (bad == 0) {
        flush(path);
        tm = tmn;
        j = jj;
        break;
      }
      const uint32_t f = (uint32_t)__builtin_ctzll(bad);
      const uint64_t below = (1ull << f) - 1ull;
      flush(path & below);
      tm = tmn & below;
      // slow step at lane f
      const uint32_t i = f;
      p = g0 + i;
      const uint32_t lk = n - p, sr = p - base;
      tm |= okm & (1ull << i);
      const uint64_t vi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)vhi, (int)i) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)vlo, (int)i);
      uint32_t ml = 0, ms = 0;
      const uint32_t mx = min(lk, (uint32_t)ZS_MAX_MATCH), nc = min(lk, (uint32_t)nice_cfg);
      const bool inc_i = __builtin_amdgcn_readlane((int)(inc ? 1u : 0u), (int)i) != 0;
#ifdef ZS_FM_PROF
      fm_slow++;
      fm_inc += inc_i ? 1u : 0u;
#endif
      if ((vi & ~tm) == 0 && !inc_i) {
        // the lane's walk holds; only its length needs more than nice + 32 bytes
        ms = (uint32_t)__builtin_amdgcn_readlane((int)bms, (int)i);
        ml = exact_len(p, base + ms, mx);
      } else {
        const uint32_t ki = (uint32_t)__builtin_amdgcn_readlane((int)kr, (int)i);
        // re-walk the true chain with the wave: entries 64 at a time, the truly inserted ones (tm inside the
        // group, the bitmap before it) in order
        const uint32_t kk = ki & 0xffffu, rk = ki >> 16;
        // lane i's first ZS_FM_R entries through LDS, the rest from memory
        if (lane == i) {
#pragma unroll
          for (int t = 0; t < (int)(ZS_FM_R / 2); t++) L.scr[t] = Ew[t];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const uint16_t* mbi;
        uint32_t wbi;
        window_of(p, mbi, wbi);
        const uint32_t lim = sr > ZS_MAX_DIST ? sr - ZS_MAX_DIST : 0u;
        uint32_t cl2 = (uint32_t)chain, b2 = ZS_MIN_MATCH - 1;
        bool fst = true, done = false;
        for (uint32_t r0 = 0; r0 < rk && !done; r0 += 64) {
          const uint32_t t = r0 + lane;  // this lane's entry
          uint32_t e = 0;
          if (t < rk) {
            if (t < ZS_FM_R) {
              const uint32_t h = ZS_FM_R - 1u - t;
              e = (L.scr[h >> 1] >> (16u * (h & 1u))) & 0xffffu;
            } else {
              e = mbi[kk - 1u - t];
            }
          }
          const uint32_t c = wbi + e;
          const bool valid = t < rk && c > base;
          const bool tru = valid && (c >= g0 ? ((tm >> ((c - g0) & 63u)) & 1ull) != 0 : inserted(c));
          const uint64_t endm = __ballot(!valid || p - c > ZS_MAX_DIST);  // (older entries are further still)
          const uint32_t e0 = endm ? (uint32_t)__builtin_ctzll(endm) : 64u;
          uint64_t cm = __ballot(tru) & (e0 >= 64u ? ~0ull : ((1ull << e0) - 1ull));
          while (cm && !done) {
            const uint32_t l = (uint32_t)__builtin_ctzll(cm);
            cm &= cm - 1;
            const uint32_t cc = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)l);
            if (!fst && cc - base <= lim) {
              done = true;
              break;
            }
            fst = false;
            const uint32_t len = exact_len(p, cc, mx);
            if (len > b2) {
              ms = cc - base;
              b2 = len;
              if (len >= nc) {
                done = true;
                break;
              }
            }
            if (--cl2 == 0) done = true;
          }
          if (e0 < 64u) done = true;
        }
        ml = b2 >= ZS_MIN_MATCH ? b2 : 0u;
      }
      if (ml >= ZS_MIN_MATCH) {
        put(0x80000000u | ((ml - ZS_MIN_MATCH) << 16) | (sr - ms));
        const uint32_t after = p + ml;
        if (ml <= (uint32_t)lazy && n - after >= ZS_MIN_MATCH)  // insert inside short matches
          tm |= ((1ull << (after - g0)) - 1ull) & ~((2ull << i) - 1ull);
        j = after - g0;
      } else {
        put((uint32_t)__builtin_amdgcn_readlane((int)hw, (int)i) & 0xffu);
        j = i + 1;
      }
      if (in_blk == ZS_SYM_END) close_block(g0 + j, 0);
    }
    p = g0 + j;
    FM_T(5);

    // ---- 4. the decided positions [g0, p) into the bitmap: tm's bits, 0 past the group (a long match's inside)
    {
      const uint32_t w = (g0 >> 5) + lane, x0 = 32u * w;
      if (x0 < p) {
        const uint32_t lo = max(g0, x0), hi = min(p, x0 + 32u);
        const uint32_t mask = (uint32_t)(((hi - x0 >= 32u ? 0xffffffffull : (1ull << (hi - x0)) - 1ull)) &
                                         ~((1ull << (lo - x0)) - 1ull));
        const uint64_t t = x0 >= g0 ? (x0 - g0 < 64u ? tm >> (x0 - g0) : 0ull) : tm << (g0 - x0);
        uint32_t* bw = &L.bits[w & 1023u];
        *bw = (*bw & ~mask) | ((uint32_t)t & mask);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }
  FM_T(6);
#ifdef ZS_FM_PROF
  if (lane == 0 && s < 4)
    printf("fmprof s=%d n=%u groups=%u slow=%u inc=%u miss=%u gather=%llu fill=%llu bits=%llu steps=%llu "
           "pf2=%llu replay=%llu ins=%llu\n", s, n, fm_groups, fm_slow, fm_inc, fm_miss, fm_acc[0], fm_acc[1],
           fm_acc[2], fm_acc[3], fm_acc[4], fm_acc[5], fm_acc[7]);
#endif
  close_block(n, 1);
  if (lane == 0) {
    streams[s].nsym = nsym;
    streams[s].nblk = nflush;
  }
}

#define ZS_FM_INST(NW)                                                                                            \
  template __global__ void zs_k_fast_mr<NW>(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*,     \
                                            const uint32_t*, uint32_t*, zs_block*, zs_stream*, int, int, int,      \
                                            const uint16_t*, const uint2*, const zs_sweep_seg*, const uint32_t*);
ZS_FM_INST(2)
ZS_FM_INST(4)
ZS_FM_INST(8)
