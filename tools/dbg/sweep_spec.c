// sweep_spec.c -- how well does a lazy parse over a cheap match table (chain
// budget cb instead of the level's) predict the positions the exact parse
// searches (deflate.ts:1352-1448)?  CPU analysis tool only.
// usage: sweep_spec FILE STREAM_BYTES level cb
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static const int CFG[10][4] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32},{4,4,16,16},{8,16,32,32},{8,16,128,128},{8,32,128,256},{32,128,258,1024},{32,258,258,4096}};
#define MAXD 32506u
static uint8_t* buf; static uint32_t* prv; static uint32_t n;
static uint32_t lm(uint32_t p, uint32_t chain, uint32_t prev_len, int good, int nicec, uint32_t* ms, uint32_t* steps) {
  uint32_t look = n - p, ch = chain, best = prev_len, nice = (uint32_t)nicec < look ? (uint32_t)nicec : look;
  if (prev_len >= (uint32_t)good) ch >>= 2;
  if (ch == 0) ch = 1;
  const uint32_t lim = p > MAXD ? p - MAXD : 0;
  uint32_t c = prv[p];
  *steps = 0;
  do {
    (*steps)++;
    uint32_t l = 0, mx = look < 258 ? look : 258;
    while (l < mx && buf[c + l] == buf[p + l]) l++;
    if (l > best) { *ms = c; best = l; if (l >= nice) break; }
    c = prv[c];
  } while (c != 0xffffffffu && c > lim && --ch != 0);
  return best;
}
// the parse; mark[p] |= bit for searched positions; returns the count
static uint32_t parse(int level, uint32_t chain, uint8_t* mark, uint8_t bit, double* stp) {
  const int good = CFG[level][0], lazy = CFG[level][1], nicec = CFG[level][2];
  uint32_t p = 0, prev_len, ml = 2, ms = 0, avail = 0, cnt = 0;
  while (p < n) {
    uint32_t hh = p + 2 < n ? prv[p] : 0xffffffffu;
    prev_len = ml; ml = 2;
    if (hh != 0xffffffffu && prev_len < (uint32_t)lazy && p - hh <= MAXD) {
      uint32_t st;
      ml = lm(p, chain, prev_len, good, nicec, &ms, &st);
      *stp += st;
      if (ml > n - p) ml = n - p;
      if (ml == 3 && p - ms > 4096) ml = 2;
      mark[p] |= bit;
      cnt++;
    }
    if (prev_len >= 3 && ml <= prev_len) { p += prev_len - 1; avail = 0; ml = 2; p++; }
    else { avail = 1; p++; }
  }
  (void)avail;
  return cnt;
}
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  n = (uint32_t)atoi(argv[2]);
  const int level = atoi(argv[3]);
  const uint32_t cb = (uint32_t)atoi(argv[4]);
  buf = malloc(n + 300); prv = malloc(4 * n);
  uint8_t* mark = malloc(n);
  uint32_t head[32768];
  double ex = 0, ap = 0, miss = 0, both = 0, st_ex = 0, st_ap = 0;
  while (fread(buf, 1, n, f) == n) {
    memset(buf + n, 0, 300);
    for (int i = 0; i < 32768; i++) head[i] = 0xffffffffu;
    for (uint32_t p = 0; p + 2 < n; p++) {
      const uint32_t h = ((buf[p] << 10) ^ (buf[p + 1] << 5) ^ buf[p + 2]) & 0x7fff;
      prv[p] = head[h]; head[h] = p;
    }
    memset(mark, 0, n);
    ex += parse(level, CFG[level][3], mark, 1, &st_ex);
    ap += parse(level, cb, mark, 2, &st_ap);
    for (uint32_t p = 0; p < n; p++) { miss += mark[p] == 1; both += mark[p] == 3; }
  }
  printf("level %d cb %u: exact searched %.0f, approx %.0f, exact not in approx %.0f (%.2f %%), approx steps %.0f vs exact %.0f\n",
         level, cb, ex, ap, miss, 100 * miss / ex, st_ap, st_ex);
  return 0;
}
