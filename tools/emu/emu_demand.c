// emu_demand.c -- CPU model of the demand-driven L4..L9 match search for
// streams of at most 65,537 bytes (zs_k_sweep in its chain>>2 mode +
// zs_k_parse_dw, deflate_sweep.hip / deflate_parse.hip), checked against a
// serial deflate_slow (deflate.ts:1352-1448) with a direct longest_match
// (deflate.ts:1053-1115).
//
// The model follows the kernels' data flow:
//   * members: the positions p <= n-3 sorted by (15-bit hash, position)
//     (zs_k_bucket); member k's chain is members k-1, k-2, ... of its bucket.
//   * phase 1 (the sweep, budget chain>>2 for every position): the exact
//     chain>>2 result S(p) (deflate.ts:1075-1077), and the full-budget result
//     when the first chain>>2 steps already settle it (the chain ended, or a
//     nice match).  Otherwise the entry is MORE with p's member index k.
//   * the parse: deflate_slow's loop; a search at full budget (prev_length <
//     good) on a MORE entry continues the walk from step chain>>2 + 1 with the
//     best so far S(p) -- over members k - t, stopping at the budget, at the
//     first member at or below limit (deflate.ts:1109), or where the member
//     positions stop falling (the bucket's first member was passed: a member
//     of another bucket differs from p in its first three bytes and never wins,
//     so a late stop only costs steps).
// Every walk's result is also compared with the direct longest_match.
// Test infrastructure (tests/test_emu_sweep.py); the kernels themselves are
// pinned by the reference goldens on the GPU.
//
// usage: emu_demand FILE CHAIN NICE GOOD LAZY; FILE = u32 count, u32 sizes[count], bytes
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define MAXD 32506u

static uint8_t buf[65536 + 300];
static int32_t head[32768], prev[65536];
static uint32_t cnt[32768], off[32768];
static uint16_t mem[65536];
static uint32_t rank_[65536];

static uint32_t hash3(uint32_t p) { return ((buf[p] << 10) ^ (buf[p + 1] << 5) ^ buf[p + 2]) & 0x7fff; }

// direct longest_match from best = 2 with a budget: len << 16 | dist (0: not called)
static uint32_t ref_lm(uint32_t n, uint32_t p, uint32_t budget, uint32_t nice_cfg, int* more) {
  int32_t cur = prev[p];
  *more = 0;
  if (p + 2 >= n || cur <= 0 || p - (uint32_t)cur > MAXD) return 0;
  uint32_t look = n - p, maxc = look < 258 ? look : 258, nice = look < nice_cfg ? look : nice_cfg;
  int limit = p > MAXD ? (int)(p - MAXD) : 0;
  uint32_t bl = 2, bd = 0, st = 0;
  for (;;) {
    st++;
    uint32_t k = 0;
    while (k < maxc && buf[cur + k] == buf[p + k]) k++;
    if (k > bl) { bl = k; bd = p - cur; if (k >= nice) break; }
    int32_t nx = prev[cur];
    if (nx <= limit) break;
    if (st >= budget) { *more = 1; break; }
    cur = nx;
  }
  return (bl << 16) | (bl > 2 ? bd : 0);
}

// the continuation walk (zs_k_parse_dw): steps cs+1 .. chain from S(p)
static long walk_steps;
static uint32_t walk(uint32_t n, uint32_t p, uint32_t k, uint32_t s, uint32_t chain, uint32_t cs, uint32_t nice_cfg) {
  const uint32_t look = n - p, maxc = look < 258 ? look : 258, nice = look < nice_cfg ? look : nice_cfg;
  const uint32_t limit = p > MAXD ? p - MAXD : 0;
  uint32_t bl = s >> 16, bd = s & 0xffff;
  uint32_t qprev = mem[k - cs];
  for (uint32_t t = cs + 1; t <= chain && t <= k; t++) {
    const uint32_t q = mem[k - t];
    if (q <= limit || q > qprev) break;
    qprev = q;
    walk_steps++;
    if (buf[q + bl] != buf[p + bl]) continue;  // the kernel's first test: the byte that must match to be longer
    uint32_t L = 0;
    while (L < maxc && buf[q + L] == buf[p + L]) L++;
    if (L > bl) { bl = L; bd = p - q; if (L >= nice) break; }
  }
  return (bl << 16) | (bl > 2 ? bd : 0);
}

int main(int argc, char** argv) {
  if (argc < 6) { fprintf(stderr, "usage: %s FILE CHAIN NICE GOOD LAZY\n", argv[0]); return 2; }
  FILE* f = fopen(argv[1], "rb");
  const uint32_t chain = atoi(argv[2]), nice_cfg = atoi(argv[3]), good = atoi(argv[4]), lazy = atoi(argv[5]);
  const uint32_t cs = chain >> 2 ? chain >> 2 : 1;
  if (!f) return 2;
  uint32_t ns = 0, sizes[4096];
  if (fread(&ns, 4, 1, f) != 1 || ns > 4096 || fread(sizes, 4, ns, f) != ns) return 2;
  static uint32_t ex[65536], ey[65536], sref[70000], sgot[70000];
  long bad = 0, badsym = 0, walks = 0, positions = 0, nmore = 0;
  for (uint32_t si = 0; si < ns; si++) {
    const uint32_t n = sizes[si];
    if (n > 65537) return 2;
    memset(buf, 0, sizeof buf);
    if (fread(buf, 1, n, f) != n) return 2;
    for (int i = 0; i < 32768; i++) head[i] = -1;
    for (uint32_t p = 0; p < n; p++) {
      prev[p] = 0;
      if (p + 2 >= n) continue;
      const uint32_t h = hash3(p);
      if (head[h] > 0) prev[p] = head[h];
      head[h] = (int32_t)p;
    }
    const uint32_t m = n > 2 ? n - 2 : 0;
    memset(cnt, 0, sizeof cnt);
    for (uint32_t p = 0; p < m; p++) cnt[hash3(p)]++;
    uint32_t run = 0;
    for (int h = 0; h < 32768; h++) { off[h] = run; run += cnt[h]; }
    for (uint32_t p = 0; p < m; p++) { rank_[p] = off[hash3(p)]; mem[off[hash3(p)]++] = (uint16_t)p; }
    // phase 1: the chain>>2 result everywhere; the full one where it is settled
    for (uint32_t p = 0; p < n; p++) {
      int more = 0, mf;
      positions++;
      ey[p] = ref_lm(n, p, cs, nice_cfg, &more);
      ex[p] = more ? 0xffff0000u | rank_[p] : ref_lm(n, p, chain, nice_cfg, &mf);
      nmore += more;
    }
    // the parse, serial, twice: with the demand walks and with the direct longest_match
    uint32_t nsym[2] = {0, 0};
    for (int pass = 0; pass < 2; pass++) {
      uint32_t* out = pass ? sref : sgot;
      uint32_t p = 0, ml = 2, ms = 0, ma = 0;
      while (p < n) {
        const uint32_t pl = ml, pm = ms;
        ml = 2;
        const uint32_t ph = p + 2 < n ? (uint32_t)prev[p] : 0;
        if (p + 2 < n && prev[p] > 0 && pl < lazy && p - ph <= MAXD) {
          uint32_t e;
          if (pl >= good) e = ey[p];
          else if (pass == 0 && (ex[p] >> 16) == 0xffffu) {
            walks++;
            e = walk(n, p, ex[p] & 0xffffu, ey[p], chain, cs, nice_cfg);
            int mf;
            const uint32_t want = ref_lm(n, p, chain, nice_cfg, &mf);
            if (e != want) {
              if (bad < 10) printf("stream %u pos %u: walk %08x want %08x\n", si, p, e, want);
              bad++;
            }
          } else if (pass == 0) e = ex[p];
          else { int mf; e = ref_lm(n, p, chain, nice_cfg, &mf); }
          const uint32_t L = e >> 16, D = e & 0xffff;
          // longest_match starts from best = prev_length: only a longer match replaces it
          if (L > pl) {
            ml = L;
            ms = p - D;
          }
          if (ml == 3 && p - ms > 4096) ml = 2;  // TOO_FAR (deflate.ts:1381-1387)
          if (ml > n - p) ml = n - p;
        }
        if (pl >= 3 && ml <= pl) {
          out[nsym[pass]++] = 0x80000000u | ((pl - 3) << 16) | (p - 1 - pm);
          p += pl - 1;
          ma = 0;
          ml = 2;
        } else if (ma) {
          out[nsym[pass]++] = buf[p - 1];
          p++;
        } else {
          ma = 1;
          p++;
        }
      }
      if (ma) out[nsym[pass]++] = buf[n - 1];
    }
    if (nsym[0] != nsym[1] || memcmp(sgot, sref, 4 * nsym[0])) {
      if (badsym < 10) printf("stream %u: symbols differ (%u vs %u)\n", si, nsym[0], nsym[1]);
      badsym++;
    }
  }
  printf("positions %ld, more %ld, walks %ld (%.2f steps each), walk mismatches %ld, streams with other symbols %ld\n",
         positions, nmore, walks, walks ? (double)walk_steps / walks : 0.0, bad, badsym);
  return bad != 0 || badsym != 0;
}
