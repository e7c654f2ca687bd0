// emu_demand_fixpoint.c -- CPU model of the fixed-point resolution of the
// demand-mode match search (VERDICT r05 "next" item 1), used to decide whether
// to build it.  CPU analysis tool only; nothing here is shipped.
//
// Round 0: the sweep gives every position its chain>>2 result S(p) and a flag
// more(p) (the chain is still live after chain>>2 steps below nice,
// deflate.ts:1075-1077,1100-1109).  Round r >= 1: deflate_slow's parse
// (deflate.ts:1352-1448) runs over a table whose full-budget entries are exact
// only on the set K resolved so far (S(p) elsewhere); every entry it consumes at
// full budget (prev_length < good_match) with more(p) and p not in K is listed;
// a continuation kernel would resolve the list (K grows) and the next round
// re-parses.  The fixed point is reached when a round lists nothing: that
// parse IS the true parse.  Reported per level: rounds to the fixed point
// (max over streams = the batch's round count, since every round is a
// batch-wide parse), entries listed per round, and the continuation's
// chain steps per listed entry.
//
// usage: emu_demand_fixpoint FILE STREAM_BYTES LEVEL   (FILE = raw concatenated streams)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static const int CFG[10][4] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32},{4,4,16,16},{8,16,32,32},{8,16,128,128},{8,32,128,256},{32,128,258,1024},{32,258,258,4096}};
#define MAXD 32506u
#define NIL 0xffffffffu
#define MAXR 64
static uint8_t* buf;
static uint32_t* prv;

// longest_match (deflate.ts:1053-1115) from best = start with budget ch; *steps = candidates compared
static uint32_t lm(uint32_t p, uint32_t n, uint32_t start, uint32_t ch, uint32_t nicec, uint32_t* ms, uint32_t* steps,
                   int* live_after) {
  const uint32_t look = n - p;
  uint32_t best = start, nice = nicec < look ? nicec : look, bm = *ms;
  const uint32_t lim = p > MAXD ? p - MAXD : 0;
  uint32_t c = prv[p], t = 0;
  *live_after = 0;
  for (;;) {
    t++;
    uint32_t l = 0, mx = look < 258 ? look : 258;
    while (l < mx && buf[c + l] == buf[p + l]) l++;
    if (l > best) { best = l; bm = c; if (l >= nice) break; }
    c = prv[c];
    if (c == NIL || c <= lim) break;
    if (t == ch) { *live_after = 1; break; }
  }
  *steps = t;
  *ms = bm;
  return best;
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s FILE STREAM_BYTES LEVEL\n", argv[0]); return 2; }
  FILE* f = fopen(argv[1], "rb");
  const uint32_t S = (uint32_t)atoi(argv[2]);
  const int level = atoi(argv[3]);
  const uint32_t good = CFG[level][0], lazy = CFG[level][1], nicec = CFG[level][2], chain = CFG[level][3];
  buf = malloc(S + 300);
  prv = malloc(4 * S);
  uint8_t* more = malloc(S);
  uint8_t* known = malloc(S);
  uint32_t head[32768];
  double listed[MAXR + 1] = {0}, cont_steps = 0, npos = 0, true_demand = 0;
  int hist[MAXR + 2] = {0}, ns = 0, maxr = 0;
  while (fread(buf, 1, S, f) == S) {
    const uint32_t n = S;
    memset(buf + n, 0, 300);
    for (int i = 0; i < 32768; i++) head[i] = NIL;
    for (uint32_t p = 0; p + 2 < n; p++) {
      const uint32_t h = ((buf[p] << 10) ^ (buf[p + 1] << 5) ^ buf[p + 2]) & 0x7fff;
      prv[p] = head[h];
      head[h] = p;
    }
    for (uint32_t p = 0; p < n; p++) {
      more[p] = 0;
      known[p] = 0;
      if (p + 2 < n && prv[p] != NIL && p - prv[p] <= MAXD) {
        uint32_t st, ms = 0; int live;
        lm(p, n, 2, chain >> 2, nicec, &ms, &st, &live);
        more[p] = (uint8_t)live;
      }
      npos++;
    }
    int r = 0;
    for (r = 1; r <= MAXR; r++) {
      uint32_t q = 0, ml = 2, ms = 0, ma = 0, added = 0, dem = 0;
      while (q < n) {
        const uint32_t pl = ml, pm = ms;
        (void)pm;
        ml = 2;
        if (q + 2 < n && prv[q] != NIL && pl < lazy && q - prv[q] <= MAXD) {
          const int full = pl < good;
          uint32_t ch = full ? chain : chain >> 2;
          if (full && more[q]) {
            dem++;
            if (!known[q]) { known[q] = 2; added++; ch = chain >> 2; }  // listed: this round parses on S(q)
          }
          uint32_t st; int live;
          ml = lm(q, n, pl, ch, nicec, &ms, &st, &live);
          if (ml > n - q) ml = n - q;
          if (ml == 3 && q - ms > 4096) ml = 2;  // TOO_FAR
        }
        if (pl >= 3 && ml <= pl) { q += pl; ma = 0; ml = 2; }
        else if (ma) q++;
        else { ma = 1; q++; }
      }
      listed[r] += added;
      for (uint32_t i = 0; i < n; i++)
        if (known[i] == 2) {  // the continuation: steps chain>>2+1 .. chain
          uint32_t st1, st2, m1 = 0, m2 = 0; int l1, l2;
          lm(i, n, 2, chain, nicec, &m1, &st1, &l1);
          lm(i, n, 2, chain >> 2, nicec, &m2, &st2, &l2);
          cont_steps += st1 - st2;
          known[i] = 1;
        }
      if (!added) { true_demand += dem; break; }
    }
    hist[r > MAXR ? MAXR + 1 : r]++;
    if (r > maxr) maxr = r;
    ns++;
  }
  double tot = 0;
  for (int r = 1; r <= MAXR; r++) tot += listed[r];
  printf("level %d, %d streams of %u B: parses to the fixed point (the last lists nothing): max %d\n", level, ns, S, maxr);
  printf("streams by parse count:");
  for (int r = 1; r <= MAXR + 1; r++) if (hist[r]) printf(" %d:%d", r, hist[r]);
  printf("\nlisted per parse (%% of positions):");
  for (int r = 1; r <= maxr && r <= MAXR; r++) printf(" %.3f", 100 * listed[r] / npos);
  printf("\nlisted in total %.2f %% of positions (true demand %.2f %%), continuation steps %.2f per listed entry, %.2f per position\n",
         100 * tot / npos, 100 * true_demand / npos, cont_steps / (tot > 0 ? tot : 1), cont_steps / npos);
  return 0;
}
