// sweep_demand2.c -- which full-budget results does the lazy parse need that
// the first chain>>2 steps do not already settle?  CPU analysis tool only.
//
// Per position p (levels 4..9, deflate.ts:1053-1115 with the parse's own
// prev_length): S(p) = the longest_match result after chain>>2 steps from a
// start of MIN_MATCH-1, and more(p) = the chain still live after those steps
// with S(p) below nice (so steps chain>>2+1 .. chain can change the result).
// The true parse (deflate.ts:1352-1448) then says which positions it searches
// at the full budget; of those, the ones with more(p) are the demand.  The
// candidate superset D0 = { p : more(p) and S(p-1) < good } (p-1 searched at any
// budget returns >= S(p-1), so prev_length >= good there unless p-1 was not
// searched) is compared with the demand: misses are demanded positions outside
// D0 (p right after an emitted match whose p-1 had a long S).
// usage: sweep_demand2 FILE STREAM_BYTES [level]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static const int CFG[10][4] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32},{4,4,16,16},{8,16,32,32},{8,16,128,128},{8,32,128,256},{32,128,258,1024},{32,258,258,4096}};
#define MAXD 32506u
#define NIL 0xffffffffu
static uint8_t* buf;
static uint32_t* prv;
// longest_match from best = start, budget ch; returns best, *steps, *live_after (chain continues past the budget)
static uint32_t lm(uint32_t p, uint32_t n, uint32_t start, uint32_t ch, uint32_t nicec, uint32_t* steps, int* live_after) {
  const uint32_t look = n - p;
  uint32_t best = start, nice = nicec < look ? nicec : look;
  const uint32_t lim = p > MAXD ? p - MAXD : 0;
  uint32_t c = prv[p], t = 0;
  *live_after = 0;
  if (c == NIL || p - c > MAXD) { *steps = 0; return best; }
  for (;;) {
    t++;
    uint32_t l = 0, mx = look < 258 ? look : 258;
    while (l < mx && buf[c + l] == buf[p + l]) l++;
    if (l > best) { best = l; if (l >= nice) break; }
    c = prv[c];
    if (c == NIL || c <= lim) break;
    if (t == ch) { *live_after = 1; break; }
  }
  *steps = t;
  return best;
}
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  const uint32_t S = (uint32_t)atoi(argv[2]);
  const int level = argc > 3 ? atoi(argv[3]) : 6;
  const uint32_t good = CFG[level][0], lazy = CFG[level][1], nicec = CFG[level][2], chain = CFG[level][3];
  buf = malloc(S + 300);
  prv = malloc(4 * S);
  uint32_t* Sl = malloc(4 * S);
  uint8_t* more = malloc(S);
  uint8_t* need = malloc(S);
  uint32_t head[32768];
  double pred_tot[3] = {0, 0, 0}, pred_miss[3] = {0, 0, 0}, nsurp = 0, npos = 0, nmore = 0, nsearch = 0, nfull = 0, ndem = 0, nd0 = 0, nmiss = 0, st_all = 0, st_s = 0, st_dem = 0,
         st_d0 = 0, nd1 = 0, nmiss1 = 0;
  int ns = 0;
  while (fread(buf, 1, S, f) == S) {
    const uint32_t n = S;
    memset(buf + n, 0, 300);
    for (int i = 0; i < 32768; i++) head[i] = NIL;
    for (uint32_t p = 0; p + 2 < n; p++) {
      const uint32_t h = ((buf[p] << 10) ^ (buf[p + 1] << 5) ^ buf[p + 2]) & 0x7fff;
      prv[p] = head[h];
      head[h] = p;
    }
    for (uint32_t p = 0; p < n; p++) { Sl[p] = 2; more[p] = 0; need[p] = 0; }
    for (uint32_t p = 0; p + 2 < n; p++) {
      uint32_t st, stf;
      int live, livef;
      Sl[p] = lm(p, n, 2, chain >> 2, nicec, &st, &live);
      more[p] = (uint8_t)live;
      lm(p, n, 2, chain, nicec, &stf, &livef);
      st_all += stf;
      st_s += st;
      npos++;
      nmore += live;
      if (live) {
        const int in_d0 = p == 0 || Sl[p - 1] < good || n - p < 262;
        // D1: also the positions where some match found at q could end (q + S(q)), i.e. p - 1's
        // S is long but the p-th byte ends a run: any q < p with q + Sl[q] == p and Sl[q] >= 3
        nd0 += in_d0;
        if (in_d0) st_d0 += stf - st;
      }
    }
    // the true parse
    uint32_t p = 0, ml = 2, ms = 0, ma = 0;
    while (p < n) {
      const uint32_t look = n - p;
      const uint32_t pl = ml, pm = ms;
      (void)pm;
      ml = 2;
      if (p + 2 < n && prv[p] != NIL && pl < lazy && p - prv[p] <= MAXD) {
        const uint32_t ch = pl >= good ? chain >> 2 : chain;
        uint32_t st;
        int live;
        // the result as the reference computes it (start at prev_length)
        uint32_t c = prv[p], best = pl, nice = nicec < look ? nicec : look, t = 0, bms = ms;
        const uint32_t lim = p > MAXD ? p - MAXD : 0;
        for (;;) {
          t++;
          uint32_t l = 0, mx = look < 258 ? look : 258;
          while (l < mx && buf[c + l] == buf[p + l]) l++;
          if (l > best) { bms = c; best = l; if (l >= nice) break; }
          c = prv[c];
          if (c == NIL || c <= lim || t == ch) break;
        }
        (void)st; (void)live;
        ml = best <= look ? best : look;
        ms = bms;
        if (ml == 3 && p - ms > 4096) ml = 2;
        nsearch++;
        if (ch == chain) {
          nfull++;
          if (more[p]) {
            ndem++;
            need[p] = 1;
            uint32_t stf; int lf;
            uint32_t sts; int ls;
            lm(p, n, 2, chain, nicec, &stf, &lf);
            lm(p, n, 2, chain >> 2, nicec, &sts, &ls);
            st_dem += stf - sts;
            {
              uint32_t a1, a2; int b1, b2;
              const uint32_t lf = lm(p, n, 2, chain, nicec, &a1, &b1), ls = lm(p, n, 2, chain >> 2, nicec, &a2, &b2);
              nsurp += lf > ls;
            }
            const int in_d0 = p == 0 || Sl[p - 1] < good || n - p < 262;
            if (!in_d0) nmiss++;
          }
        }
      }
      if (pl >= 3 && ml <= pl) {
        p += pl - 1;
        ma = 0;
        ml = 2;
        p++;
      } else if (ma) {
        p++;
      } else {
        ma = 1;
        p++;
      }
    }
    // predicted demand: parses over tables whose full-budget entries are exact only on the set
    // computed so far (the chain>>2 result elsewhere); each round adds the demand it sees
    {
      uint8_t* known = calloc(n, 1);
      for (int round = 0; round < 3; round++) {
        uint32_t q = 0, ml2 = 2, ms2 = 0, ma2 = 0;
        double added = 0;
        while (q < n) {
          const uint32_t look2 = n - q, pl2 = ml2;
          ml2 = 2;
          if (q + 2 < n && prv[q] != NIL && pl2 < lazy && q - prv[q] <= MAXD) {
            const int full = pl2 < good;
            const uint32_t ch = full ? chain : chain >> 2;
            const int kn = known[q] == 1 || !more[q];  // the full result is exact here (or equals the short one)
            if (full && more[q] && !known[q]) { known[q] = 2; added++; }
            uint32_t useful = full && kn ? ch : (chain >> 2);
            uint32_t c = prv[q], best = pl2, nice = nicec < look2 ? nicec : look2, t = 0, bms = ms2;
            const uint32_t lim = q > MAXD ? q - MAXD : 0;
            for (;;) {
              t++;
              uint32_t l = 0, mx = look2 < 258 ? look2 : 258;
              while (l < mx && buf[c + l] == buf[q + l]) l++;
              if (l > best) { bms = c; best = l; if (l >= nice) break; }
              c = prv[c];
              if (c == NIL || c <= lim || t == useful) break;
            }
            ml2 = best <= look2 ? best : look2;
            ms2 = bms;
            if (ml2 == 3 && q - ms2 > 4096) ml2 = 2;
          }
          if (pl2 >= 3 && ml2 <= pl2) { q += pl2; ma2 = 0; ml2 = 2; }
          else if (ma2) q++;
          else { ma2 = 1; q++; }
        }
        double miss = 0, tot = 0;
        for (uint32_t i = 0; i < n; i++) { tot += known[i] != 0; miss += need[i] && !known[i]; }
        pred_tot[round] += tot;
        pred_miss[round] += miss;
        (void)added;
        for (uint32_t i = 0; i < n; i++) if (known[i] == 2) known[i] = 1;
      }
      free(known);
    }
    (void)nd1; (void)nmiss1;
    ns++;
  }
  printf("streams %d level %d: positions %.0f\n", ns, level, npos);
  printf("sweep steps: full %.1f / pos, first chain>>2 %.1f / pos, rest %.1f / pos\n", st_all / npos, st_s / npos,
         (st_all - st_s) / npos);
  printf("more (chain live past chain>>2, below nice): %.1f %%\n", 100 * nmore / npos);
  printf("parse: searched %.1f %%, at full budget %.1f %%, demand (full budget and more) %.1f %% with %.2f rest steps / pos\n",
         100 * nsearch / npos, 100 * nfull / npos, 100 * ndem / npos, st_dem / npos);
  printf("surprises (full result longer than the chain>>2 one) %.1f %% of the demand, %.2f per 1 KiB\n", 100 * nsurp / ndem, 1024 * nsurp / npos);
  for (int r = 0; r < 3; r++)
    printf("predicted demand after %d parse(s): %.1f %% of positions, true demand missed %.2f %% of positions (%.1f %% of the demand)\n",
           r + 1, 100 * pred_tot[r] / npos, 100 * pred_miss[r] / npos, 100 * pred_miss[r] / ndem);
  printf("superset D0 (more and S(p-1) < good): %.1f %% with %.2f rest steps / pos; demand misses %.0f (%.3f %% of positions)\n",
         100 * nd0 / npos, st_d0 / npos, nmiss, 100 * nmiss / npos);
  return 0;
}
