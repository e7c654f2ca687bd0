// sweep_window_chunks.c -- lock-step cost of the windowed sweep (streams over 65,537 B): aligned chunks vs chunks
// starting at own members vs fully compacted own chunks.  CPU analysis tool only.
// usage: sweep_window_chunks RAWFILE STREAM_BYTES CHAIN
// lanes) vs compacted own-member chunks (64 consecutive own members)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define MAXD 32506u
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb"); uint32_t S = atoi(argv[2]); int chain = atoi(argv[3]);
  uint8_t* buf = malloc(S + 300);
  static uint32_t cnt[32768], off[32768], st[32768];
  static uint32_t mem[65536], L[65536], hh[65536];
  static double vv[4], vc[4]; double cur = 0, comp = 0, exact = 0, ownpos = 0, slots = 0, chunks_cur = 0, chunks_comp = 0, gapsum = 0;
  while (fread(buf, 1, S, f) == S) {
    memset(buf + S, 0, 300);
    for (uint32_t lo = 0; lo < S;) {
      uint32_t base = lo == 0 ? 0 : lo - 32768, olo = lo - base, ohi = lo == 0 ? 65520 : 32768 + 32752;
      uint32_t nrel = S - base, m = nrel > 2 ? (nrel - 2 < ohi ? nrel - 2 : ohi) : 0;
      const uint8_t* b = buf + base;
      memset(cnt, 0, sizeof cnt);
      for (uint32_t p = 0; p < m; p++) { hh[p] = ((b[p] << 10) ^ (b[p + 1] << 5) ^ b[p + 2]) & 0x7fff; cnt[hh[p]]++; }
      uint32_t r = 0; for (int h = 0; h < 32768; h++) { off[h] = r; r += cnt[h]; }
      memcpy(st, off, sizeof st);
      for (uint32_t p = 0; p < m; p++) mem[st[hh[p]]++] = p;
      for (uint32_t k = 0; k < m; k++) {
        uint32_t p = mem[k], h = hh[p], ap = p + base, lim = ap > MAXD ? ap - MAXD : 0, l = 0;
        for (int t = 1; t <= chain; t++) { int j = (int)k - t; if (j < (int)off[h]) break; uint32_t q = mem[j] + base; if (t == 1 ? (q < (lim > 1 ? lim : 1)) : (q <= lim)) break; l = t; }
        L[k] = l;
        int own = p >= olo && p < ohi;
        if (own) { exact += l; ownpos++; }
      }
      slots += m;
      for (uint32_t c = 0; c < m; c += 64) {
        uint32_t mx = 0, any = 0;
        for (uint32_t k = c; k < c + 64 && k < m; k++) { if (L[k] > mx) mx = L[k]; if (mem[k] >= olo && mem[k] < ohi) any = 1; }
        if (any) { cur += 64.0 * mx; chunks_cur++; }
      }
      // v2/v3: chunks start at an own member, consecutive members, cut before a look-back run longer than G
      for (int G = 0; G < 4; G++) {
        static const uint32_t GS[4] = {1000000, 32, 8, 0};
        uint32_t k = 0;
        while (k < m) {
          while (k < m && !(mem[k] >= olo && mem[k] < ohi)) k++;
          if (k >= m) break;
          uint32_t e = k, mxx = 0, lanes = 0;
          while (e < m && lanes < 64) {
            if (!(mem[e] >= olo && mem[e] < ohi)) {  // a look-back run: its length
              uint32_t r = e; while (r < m && !(mem[r] >= olo && mem[r] < ohi)) r++;
              if (r - e > GS[G] || lanes + (r - e) >= 64) break;
              for (uint32_t x = e; x < r; x++) { if (L[x] > mxx) mxx = L[x]; lanes++; }
              e = r; continue;
            }
            if (L[e] > mxx) mxx = L[e];
            lanes++; e++;
          }
          vv[G] += 64.0 * mxx; vc[G]++;
          k = e;
        }
      }
      uint32_t n = 0, mx = 0, kmin = 0;
      for (uint32_t k = 0; k < m; k++) {
        if (!(mem[k] >= olo && mem[k] < ohi)) continue;
        if (n == 0) kmin = k;
        if (L[k] > mx) mx = L[k];
        if (++n == 64) { comp += 64.0 * mx; chunks_comp++; gapsum += k - kmin - 63; n = 0; mx = 0; }
      }
      if (n) { comp += 64.0 * mx; chunks_comp++; }
      lo += lo == 0 ? 65520 : 32752;
    }
  }
  printf("own positions %.0f, member slots %.0f; steps per own position: exact %.1f, current chunks %.1f (%.0f chunks), compacted %.1f (%.0f chunks, avg member-index gap %.1f)\n",
         ownpos, slots, exact / ownpos, cur / ownpos, chunks_cur, comp / ownpos, chunks_comp, gapsum / chunks_comp);
  for (int G = 0; G < 4; G++) printf("  own-start chunks, cut at look-back runs > %d: %.1f steps per own position, %.0f chunks\n", G == 0 ? 1000000 : G == 1 ? 32 : G == 2 ? 8 : 0, vv[G] / ownpos, vc[G]);
}
