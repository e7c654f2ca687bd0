// sweep_demand.c -- how much of zs_k_sweep's work does the lazy parse use?
// For each stream: the chain steps the sweep evaluates (every inserted
// position, min(budget, live chain)) against the steps longest_match takes at
// the positions deflate_slow actually searches (deflate.ts:1352-1448, budget
// >> 2 after a good match, early exit at nice).  CPU analysis tool only.
// usage: sweep_demand FILE STREAM_BYTES [level]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static const int CFG[10][4] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32},{4,4,16,16},{8,16,32,32},{8,16,128,128},{8,32,128,256},{32,128,258,1024},{32,258,258,4096}};
#define MAXD 32506u
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  const uint32_t S = (uint32_t)atoi(argv[2]);
  const int level = argc > 3 ? atoi(argv[3]) : 6;
  const int good = CFG[level][0], lazy = CFG[level][1], nicec = CFG[level][2], chain = CFG[level][3];
  uint8_t* buf = malloc(S + 300);
  uint32_t* prev = malloc(4 * S);
  uint32_t head[32768];
  double all_steps = 0, srch_steps = 0, npos = 0, nsrch = 0, all_steps_s = 0, hist_all[8] = {0}, hist_srch[8] = {0};
  int ns = 0;
  while (fread(buf, 1, S, f) == S) {
    const uint32_t n = S;
    memset(buf + n, 0, 300);
    for (int i = 0; i < 32768; i++) head[i] = 0xffffffffu;
    for (uint32_t p = 0; p + 2 < n; p++) {
      const uint32_t h = ((buf[p] << 10) ^ (buf[p + 1] << 5) ^ buf[p + 2]) & 0x7fff;
      prev[p] = head[h];
      head[h] = p;
    }
    // the sweep's cost per position: live chain steps up to the budget
    uint32_t* live = malloc(4 * n);
    for (uint32_t p = 0; p + 2 < n; p++) {
      uint32_t c = prev[p], t = 0;
      const uint32_t lim = p > MAXD ? p - MAXD : 0;
      while (c != 0xffffffffu && c > lim && t < (uint32_t)chain) { t++; c = prev[c]; }
      live[p] = t;
      all_steps += t;
      all_steps_s += t < (uint32_t)(chain >> 2) ? t : (uint32_t)(chain >> 2);
      npos++;
      hist_all[t == 0 ? 0 : t < 4 ? 1 : t < 16 ? 2 : t < 64 ? 3 : t < 128 ? 4 : 5]++;
    }
    // deflate_slow's parse with the real longest_match, counting its steps
    uint32_t p = 0, prev_len = 2, prev_match = 0, match_avail = 0, ml = 2, ms = 0;
    while (p < n) {
      uint32_t look = n - p;
      uint32_t hh = p + 2 < n ? prev[p] : 0xffffffffu;
      prev_len = ml; prev_match = ms; ml = 2;
      if (p + 2 < n && hh != 0xffffffffu && prev_len < (uint32_t)lazy && p - hh <= MAXD) {
        uint32_t ch = chain, best = prev_len, nice = nicec < (int)look ? nicec : look, steps = 0;
        if (prev_len >= (uint32_t)good) ch >>= 2;
        const uint32_t lim = p > MAXD ? p - MAXD : 0;
        uint32_t c = hh;
        do {
          steps++;
          uint32_t l = 0, mx = look < 258 ? look : 258;
          while (l < mx && buf[c + l] == buf[p + l]) l++;
          if (l > best) { ms = c; best = l; if (l >= nice) break; }
          c = prev[c];
        } while (c != 0xffffffffu && c > lim && --ch != 0);
        ml = best <= look ? best : look;
        if (ml <= 5 && ml == 3 && p - ms > 4096) ml = 2;
        srch_steps += steps;
        nsrch++;
        uint32_t t = live[p];
        hist_srch[t == 0 ? 0 : t < 4 ? 1 : t < 16 ? 2 : t < 64 ? 3 : t < 128 ? 4 : 5]++;
      }
      if (prev_len >= 3 && ml <= prev_len) {
        p += prev_len - 1;  // (the inserts inside the match happen above for every position)
        match_avail = 0; ml = 2;
        p++;
      } else if (match_avail) {
        p++;
      } else {
        match_avail = 1;
        p++;
      }
    }
    free(live);
    ns++;
  }
  printf("streams %d level %d: positions %.0f, sweep steps %.0f (%.1f / pos; chain>>2 part %.1f)\n", ns, level, npos, all_steps,
         all_steps / npos, all_steps_s / npos);
  printf("searched %.0f (%.1f %%), their steps %.0f (%.1f %% of the sweep's)\n", nsrch, 100 * nsrch / npos, srch_steps,
         100 * srch_steps / all_steps);
  printf("live-chain histogram (0,1-3,4-15,16-63,64-127,128): all");
  for (int i = 0; i < 6; i++) printf(" %.1f%%", 100 * hist_all[i] / npos);
  printf("  searched");
  for (int i = 0; i < 6; i++) printf(" %.1f%%", 100 * hist_srch[i] / nsrch);
  printf("\n");
  return 0;
}
