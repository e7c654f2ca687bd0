// emu_fast_group_g.c -- emu_fast_group.c with the group size G a compile-time
// parameter (-DG=64|128|256): the CPU model behind the "4-wave zs_k_fast" question
// (how often a step must re-walk when a group spans 128 or
// 256 positions, i.e. 2 or 4 waves of one stream).  CPU analysis tool only.
//
// emu_fast_group.c -- CPU model of the group-speculative deflate_fast parser
// (zs_k_fast, deflate_fast.hip) for levels 1..3, checked against a serial
// transcription of the reference's deflate_fast (deflate.ts:1281-1350) with
// the same window-relative head[] / prev[] tables and slide schedule.
//
// The model works on groups of 64 consecutive positions [g0, g0 + 64), one per
// lane.  Every lane speculatively inserts its position (the superset of what
// deflate_fast inserts: it skips the inside of matches longer than max_lazy,
// deflate.ts:1310-1322), walks its chain over that superset, and records which
// in-group positions it visited.  The serial parse then replays the group
// from lane results: a lane's result is exact iff every in-group position it
// visited was truly inserted (the true chain is the superset chain minus the
// skipped positions, so a walk that met none of them is the true walk); other
// steps re-walk the true chain.  After the group, only the truly inserted
// positions enter head[] / prev[].
//
// Input on stdin: records of u32 chain, lazy, nice, n, then n bytes.
// Output: one line per stream: "ok <steps> <rewalks>" or "MISMATCH at <sym>".
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MIN_MATCH 3u
#define MAX_MATCH 258u
#define MIN_LOOKAHEAD 262u
#define MAX_DIST 32506u
#define SLIDE_AT 65274u
#define SYM_END 16383u
#define HMASK 0x7fffu
#ifndef G
#define G 64u
#endif
#define GW (G / 64u)
static inline int bt(const uint64_t* m, uint32_t i) { return (int)((m[i >> 6] >> (i & 63u)) & 1u); }
static inline void bs(uint64_t* m, uint32_t i) { m[i >> 6] |= 1ull << (i & 63u); }
// step starts in [g0, g0 + 64 - max_lazy): short-match insides stay below g0 + 64

static uint32_t hash3(const uint8_t* s, uint32_t q) {
  return (((uint32_t)s[q] << 10) ^ ((uint32_t)s[q + 1] << 5) ^ s[q + 2]) & HMASK;
}
static uint32_t lcp(const uint8_t* s, uint32_t a, uint32_t b, uint32_t cap) {
  uint32_t k = 0;
  while (k < cap && s[a + k] == s[b + k]) k++;
  return k;
}

typedef struct {
  uint32_t* sym;
  uint32_t nsym;
  uint32_t* cut;  // block cut positions
  uint32_t ncut;
} out_t;

static void emit(out_t* o, uint32_t v, uint32_t* in_blk, uint32_t p) {
  o->sym[o->nsym++] = v;
  if (++*in_blk == SYM_END) {
    o->cut[o->ncut++] = p;
    *in_blk = 0;
  }
}
static void slide(uint16_t* head, uint16_t* prev) {
  for (uint32_t i = 0; i < 32768; i++) {
    head[i] = head[i] >= 32768u ? head[i] - 32768u : 0;
    prev[i] = prev[i] >= 32768u ? prev[i] - 32768u : 0;
  }
}
static int slide_due(uint32_t p, uint32_t base, uint32_t n) {
  const uint32_t m = n < base + 65536u ? n : base + 65536u;
  return p - base >= SLIDE_AT && m - p < MIN_LOOKAHEAD;
}

// ---------------------------------------------------------------- serial
static void serial(const uint8_t* s, uint32_t n, uint32_t chain, uint32_t lazy, uint32_t nice_cfg, out_t* o) {
  static uint16_t head[32768], prev[32768];
  memset(head, 0, sizeof head);
  memset(prev, 0, sizeof prev);
  uint32_t base = 0, p = 0, in_blk = 0;
  while (p < n) {
    if (slide_due(p, base, n)) {
      slide(head, prev);
      base += 32768u;
    }
    const uint32_t look = n - p;
    uint32_t hh = 0, ml = 0, ms = 0;
    if (look >= MIN_MATCH) {
      const uint32_t h = hash3(s, p);
      hh = head[h];
      prev[(p - base) & HMASK] = (uint16_t)hh;
      head[h] = (uint16_t)(p - base);
    }
    const uint32_t srel = p - base;
    if (hh != 0 && srel - hh <= MAX_DIST) {
      uint32_t cl = chain, best = MIN_MATCH - 1, cur = hh;
      const uint32_t maxc = look < MAX_MATCH ? look : MAX_MATCH;
      const uint32_t nice = look < nice_cfg ? look : nice_cfg;
      const uint32_t limit = srel > MAX_DIST ? srel - MAX_DIST : 0;
      do {
        const uint32_t len = lcp(s, p, base + cur, maxc);
        if (len > best) {
          ms = cur;
          best = len;
          if (len >= nice) break;
        }
        cur = prev[cur & HMASK];
      } while (cur > limit && --cl != 0);
      ml = best;
    }
    if (ml >= MIN_MATCH) {
      emit(o, 0x80000000u | ((ml - MIN_MATCH) << 16) | (srel - ms), &in_blk, p + ml);
      const uint32_t after = p + ml;
      if (ml <= lazy && n - after >= MIN_MATCH)
        for (uint32_t q = p + 1; q < after; q++) {
          const uint32_t h = hash3(s, q);
          prev[(q - base) & HMASK] = head[h];
          head[h] = (uint16_t)(q - base);
        }
      p = after;
    } else {
      emit(o, s[p], &in_blk, p + 1);
      p++;
    }
  }
}

// ---------------------------------------------------------------- groups
static uint64_t g_rewalks, g_steps, g_groups;

static void grouped(const uint8_t* s, uint32_t n, uint32_t chain, uint32_t lazy, uint32_t nice_cfg, out_t* o) {
  static uint16_t head[32768], prev[32768];
  memset(head, 0, sizeof head);
  memset(prev, 0, sizeof prev);
  uint32_t base = 0, p = 0, in_blk = 0;
  while (p < n) {
    if (slide_due(p, base, n)) {
      slide(head, prev);
      base += 32768u;
    }
    g_groups++;
    const uint32_t g0 = p, rg0 = g0 - base;
    const uint32_t m = n < base + 65536u ? n : base + 65536u;
    uint32_t tslide = base + SLIDE_AT;  // first position at which the next slide is due
    if (m >= MIN_LOOKAHEAD - 1 && m - (MIN_LOOKAHEAD - 1) > tslide) tslide = m - (MIN_LOOKAHEAD - 1);
    uint32_t g1 = g0 + G - lazy;
    if (g1 > tslide) g1 = tslide;
    if (g1 > n) g1 = n;
    // ---- lanes (parallel in the kernel)
    static uint32_t h[G], ok[G], sp[G], orig[G], best[G], bms[G];
    static uint64_t vis[G][GW];
    for (uint32_t i = 0; i < G; i++) {
      const uint32_t q = g0 + i;
      ok[i] = q + 2 < n;
      h[i] = ok[i] ? hash3(s, q) : 0;
    }
    // speculative insertion of every lane, in lane order (one lane-ordered LDS exchange)
    for (uint32_t i = 0; i < G; i++)
      if (ok[i]) {
        sp[i] = head[h[i]];
        head[h[i]] = (uint16_t)(rg0 + i);
      }
#define IN_GROUP(v) ((v) != 0 && (v) >= rg0)
    // restore: the first lane of each hash puts the original head back
    for (uint32_t i = 0; i < G; i++)
      if (ok[i] && !IN_GROUP(sp[i])) head[h[i]] = (uint16_t)sp[i];
    for (uint32_t i = 0; i < G; i++)
      if (ok[i]) orig[i] = IN_GROUP(sp[i]) ? orig[sp[i] - rg0] : sp[i];
    // walks over the superset chain, lengths capped at nice
    for (uint32_t i = 0; i < G; i++) {
      const uint32_t q = g0 + i;
      best[i] = MIN_MATCH - 1;
      bms[i] = 0;
      for (uint32_t w = 0; w < GW; w++) vis[i][w] = 0;
      if (!ok[i] || q >= g1) continue;
      const uint32_t look = n - q, srel = q - base, hh = sp[i];
      if (!(hh != 0 && srel - hh <= MAX_DIST)) continue;
      const uint32_t maxc = look < MAX_MATCH ? look : MAX_MATCH;
      const uint32_t nice = look < nice_cfg ? look : nice_cfg;
      const uint32_t limit = srel > MAX_DIST ? srel - MAX_DIST : 0;
      uint32_t cl = chain, cur = hh;
      do {
        if (IN_GROUP(cur)) bs(vis[i], cur - rg0);
        const uint32_t len = lcp(s, q, base + cur, nice < maxc ? nice : maxc);
        if (len > best[i]) {
          bms[i] = cur;
          best[i] = len;
          if (len >= nice) break;
        }
        cur = IN_GROUP(cur) ? sp[cur - rg0] : prev[cur & HMASK];
      } while (cur > limit && --cl != 0);
    }
    // ---- serial replay of the group (scalar in the kernel)
    uint64_t tmask[GW];
    for (uint32_t w = 0; w < GW; w++) tmask[w] = 0;
    while (p < g1) {
      g_steps++;
      const uint32_t i = p - g0, look = n - p, srel = p - base;
      if (ok[i]) bs(tmask, i);
      uint32_t ml = 0, ms = 0;
      int exact = 1;
      for (uint32_t w = 0; w < GW; w++) exact &= (vis[i][w] & ~tmask[w]) == 0;
      if (exact) {
        ml = best[i];
        ms = bms[i];
        const uint32_t nice = look < nice_cfg ? look : nice_cfg;
        if (ml >= nice) {
          const uint32_t maxc = look < MAX_MATCH ? look : MAX_MATCH;
          ml = lcp(s, p, base + ms, maxc);
        }
      } else {
        g_rewalks++;
        // the true chain: in-group links through the truly inserted lanes of the same hash
        uint32_t hh = orig[i];
        for (int j = (int)i - 1; j >= 0; j--)
          if (bt(tmask, (uint32_t)j) && h[j] == h[i]) {
            hh = rg0 + j;
            break;
          }
        if (hh != 0 && srel - hh <= MAX_DIST) {
          uint32_t cl = chain, best2 = MIN_MATCH - 1, cur = hh;
          const uint32_t maxc = look < MAX_MATCH ? look : MAX_MATCH;
          const uint32_t nice = look < nice_cfg ? look : nice_cfg;
          const uint32_t limit = srel > MAX_DIST ? srel - MAX_DIST : 0;
          do {
            const uint32_t len = lcp(s, p, base + cur, maxc);
            if (len > best2) {
              ms = cur;
              best2 = len;
              if (len >= nice) break;
            }
            if (IN_GROUP(cur)) {
              const uint32_t l = cur - rg0;
              uint32_t nx = orig[l];
              for (int j = (int)l - 1; j >= 0; j--)
                if (bt(tmask, (uint32_t)j) && h[j] == h[l]) {
                  nx = rg0 + j;
                  break;
                }
              cur = nx;
            } else {
              cur = prev[cur & HMASK];
            }
          } while (cur > limit && --cl != 0);
          ml = best2;
        }
      }
      if (ml >= MIN_MATCH) {
        emit(o, 0x80000000u | ((ml - MIN_MATCH) << 16) | (srel - ms), &in_blk, p + ml);
        const uint32_t after = p + ml;
        if (ml <= lazy && n - after >= MIN_MATCH)
          for (uint32_t q = p + 1; q < after; q++) bs(tmask, q - g0);
        p = after;
      } else {
        emit(o, s[p], &in_blk, p + 1);
        p++;
      }
    }
    // the truly inserted positions enter the tables, in order
    for (uint32_t i = 0; i < G; i++)
      if (bt(tmask, i)) {
        prev[(rg0 + i) & HMASK] = head[h[i]];
        head[h[i]] = (uint16_t)(rg0 + i);
      }
  }
}

int main(void) {
  uint32_t hdr[4];
  int bad = 0;
  while (fread(hdr, 4, 4, stdin) == 4) {
    const uint32_t chain = hdr[0], lazy = hdr[1], nice = hdr[2], n = hdr[3];
    uint8_t* s = calloc(n + 16, 1);
    if (fread(s, 1, n, stdin) != n) return 2;
    out_t a = {calloc(n + 1, 4), 0, calloc(n / SYM_END + 4, 4), 0};
    out_t b = {calloc(n + 1, 4), 0, calloc(n / SYM_END + 4, 4), 0};
    g_rewalks = g_steps = g_groups = 0;
    serial(s, n, chain, lazy, nice, &a);
    grouped(s, n, chain, lazy, nice, &b);
    uint32_t at = 0;
    while (at < a.nsym && at < b.nsym && a.sym[at] == b.sym[at]) at++;
    if (at != a.nsym || a.nsym != b.nsym || a.ncut != b.ncut ||
        memcmp(a.cut, b.cut, 4ull * a.ncut) != 0) {
      printf("MISMATCH n=%u at %u of %u/%u\n", n, at, a.nsym, b.nsym);
      bad = 1;
    } else {
      printf("ok n=%u syms=%u groups=%llu steps=%llu rewalks=%llu\n", n, a.nsym, (unsigned long long)g_groups,
             (unsigned long long)g_steps, (unsigned long long)g_rewalks);
    }
    free(s);
    free(a.sym), free(a.cut), free(b.sym), free(b.cut);
  }
  return bad;
}
