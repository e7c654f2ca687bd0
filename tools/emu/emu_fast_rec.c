// emu_fast_rec.c -- CPU model of deflate_fast (levels 1..3, deflate.ts:1281-1350)
// WITHOUT head[] / prev[]: the group-speculative replay of zs_k_fast
// (tools/emu/emu_fast_group.c) with every chain read from per-position
// SUPERSET records instead of the reference's tables.
//
// Superset: every position p <= n-3 inserted (what levels 4..9 insert).  The
// superset chain of q is every earlier position with q's hash, most recent
// first; deflate_fast's true chain is that chain minus the positions it did not
// insert (the insides of matches longer than max_lazy, deflate.ts:1310-1322).
// A record holds the first R superset predecessors of q as distances (0: none):
// the R members before q's in its bucket (zs_k_fast_mr loads them as a run of
// the bucket sort's member array); a lane walk that needs more is left to the
// replay's slow step (counted as "incomplete"), which walks the true chain.
// Positions before the current group are filtered through an "inserted"
// bitmap (exact: the parse has decided them); positions inside the group are
// taken speculatively and recorded (vis), as in zs_k_fast.  The slide of
// fill_window (deflate.ts:180-190) appears only as "a candidate at or below
// the window base is NIL" (head/prev entries below 32 K become 0), since every
// candidate is within MAX_DIST.
//
// Checked here against a serial transcription with the reference's tables;
// prints per stream the walks, the incomplete ones and the re-walks.
// Input on stdin: records of u32 chain, lazy, nice, n, R, then n bytes.
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
  uint32_t* cut;
  uint32_t ncut;
} out_t;
static void emit(out_t* o, uint32_t v, uint32_t* in_blk, uint32_t p) {
  o->sym[o->nsym++] = v;
  if (++*in_blk == SYM_END) {
    o->cut[o->ncut++] = p;
    *in_blk = 0;
  }
}
static int slide_due(uint32_t p, uint32_t base, uint32_t n) {
  const uint32_t m = n < base + 65536u ? n : base + 65536u;
  return p - base >= SLIDE_AT && m - p < MIN_LOOKAHEAD;
}

// ---------------------------------------------------------------- serial (the reference's tables)
static void serial(const uint8_t* s, uint32_t n, uint32_t chain, uint32_t lazy, uint32_t nice_cfg, out_t* o) {
  static uint16_t head[32768], prev[32768];
  memset(head, 0, sizeof head);
  memset(prev, 0, sizeof prev);
  uint32_t base = 0, p = 0, in_blk = 0;
  while (p < n) {
    if (slide_due(p, base, n)) {
      for (uint32_t i = 0; i < 32768; i++) {
        head[i] = head[i] >= 32768u ? head[i] - 32768u : 0;
        prev[i] = prev[i] >= 32768u ? prev[i] - 32768u : 0;
      }
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

// ---------------------------------------------------------------- records
static uint32_t R;
static uint16_t* rec;    // rec[q * R + r]: distance to q's (r+1)-th superset predecessor, 0 = none
static uint8_t* ins;     // truly inserted (decided positions)
static uint64_t g_walks, g_chases, g_rewalks, g_steps, g_cand, g_skipped, g_incomplete;

// superset walker: yields q's superset predecessors most recent first
typedef struct {
  uint32_t q;   // the record's owner
  uint32_t r;   // next entry
  uint32_t at;  // last yielded position
} sw_t;
static int sw_next(sw_t* w, uint32_t* c, int* chased) {
  if (w->r == R) {  // record exhausted: continue from the last predecessor's record
    w->q = w->at;
    w->r = 0;
    *chased = 1;
  }
  const uint16_t d = rec[(size_t)w->q * R + w->r];
  if (!d) return 0;
  w->r++;
  w->at = w->q - d;
  *c = w->at;
  return 1;
}

static void grouped(const uint8_t* s, uint32_t n, uint32_t chain, uint32_t lazy, uint32_t nice_cfg, out_t* o) {
  uint32_t base = 0, p = 0, in_blk = 0;
  memset(ins, 0, n + 64);
  while (p < n) {
    if (slide_due(p, base, n)) {
      base += 32768u;
      continue;
    }
    const uint32_t g0 = p;
    const uint32_t m = n < base + 65536u ? n : base + 65536u;
    uint32_t tslide = base + SLIDE_AT;
    if (m >= MIN_LOOKAHEAD - 1 && m - (MIN_LOOKAHEAD - 1) > tslide) tslide = m - (MIN_LOOKAHEAD - 1);
    uint32_t g1 = g0 + 64u - lazy;
    if (g1 > tslide) g1 = tslide;
    if (g1 > n) g1 = n;
    uint32_t ok[64], best[64], bms[64];
    uint64_t vis[64];
    for (uint32_t i = 0; i < 64; i++) {
      const uint32_t q = g0 + i;
      ok[i] = q + 2 < n;
    }
    // ---- lane walks over the superset chain: in-group candidates speculative, earlier ones filtered
    for (uint32_t i = 0; i < 64; i++) {
      const uint32_t q = g0 + i;
      best[i] = MIN_MATCH - 1;
      bms[i] = 0;
      vis[i] = 0;
      if (!ok[i] || q >= g1) continue;
      g_walks++;
      const uint32_t look = n - q, srel = q - base;
      const uint32_t maxc = look < MAX_MATCH ? look : MAX_MATCH;
      const uint32_t nice = look < nice_cfg ? look : nice_cfg;
      const uint32_t limit = srel > MAX_DIST ? srel - MAX_DIST : 0;
      sw_t w = {q, 0, q};
      uint32_t cl = chain, c;
      int first = 1, chased = 0;
      while (sw_next(&w, &c, &chased)) {
        if (chased) {  // past the lane's R entries: the replay re-walks it if it is on the path
          vis[i] = ~0ull;
          break;
        }
        if (c <= base) break;  // NIL (slid out, or window index 0)
        const uint32_t crel = c - base;
        const int ingrp = c >= g0;
        if (!ingrp && !ins[c]) {
          g_skipped++;
          if (srel - crel > MAX_DIST) break;  // (further ones are older still)
          continue;
        }
        if (first ? srel - crel > MAX_DIST : crel <= limit) break;
        first = 0;
        g_cand++;
        if (ingrp) vis[i] |= 1ull << (c - g0);
        const uint32_t len = lcp(s, q, c, nice < maxc ? nice : maxc);
        if (len > best[i]) {
          bms[i] = crel;
          best[i] = len;
          if (len >= nice) break;
        }
        if (--cl == 0) break;
      }
      g_chases += chased;
    }
    // ---- serial replay of the group
    uint64_t tmask = 0;
    while (p < g1) {
      g_steps++;
      const uint32_t i = p - g0, look = n - p, srel = p - base;
      if (ok[i]) tmask |= 1ull << i;
      uint32_t ml = 0, ms = 0;
      if (vis[i] == ~0ull) g_incomplete++;
      if ((vis[i] & ~tmask) == 0) {
        ml = best[i];
        ms = bms[i];
        const uint32_t nice = look < nice_cfg ? look : nice_cfg;
        if (ml >= nice) {
          const uint32_t maxc = look < MAX_MATCH ? look : MAX_MATCH;
          ml = lcp(s, p, base + ms, maxc);
        }
      } else {
        g_rewalks++;  // the true chain: the superset filtered by what is decided (tmask in the group)
        const uint32_t maxc = look < MAX_MATCH ? look : MAX_MATCH;
        const uint32_t nice = look < nice_cfg ? look : nice_cfg;
        const uint32_t limit = srel > MAX_DIST ? srel - MAX_DIST : 0;
        sw_t w = {p, 0, p};
        uint32_t cl = chain, c, best2 = MIN_MATCH - 1;
        int first = 1, chased = 0;
        while (sw_next(&w, &c, &chased)) {
          if (c <= base) break;
          const uint32_t crel = c - base;
          const int truly = c >= g0 ? (int)((tmask >> (c - g0)) & 1) : ins[c];
          if (!truly) {
            if (srel - crel > MAX_DIST) break;
            continue;
          }
          if (first ? srel - crel > MAX_DIST : crel <= limit) break;
          first = 0;
          const uint32_t len = lcp(s, p, c, maxc);
          if (len > best2) {
            ms = crel;
            best2 = len;
            if (len >= nice) break;
          }
          if (--cl == 0) break;
        }
        ml = best2;
      }
      if (ml >= MIN_MATCH) {
        emit(o, 0x80000000u | ((ml - MIN_MATCH) << 16) | (srel - ms), &in_blk, p + ml);
        const uint32_t after = p + ml;
        if (ml <= lazy && n - after >= MIN_MATCH)
          for (uint32_t q = p + 1; q < after; q++) tmask |= 1ull << (q - g0);
        p = after;
      } else {
        emit(o, s[p], &in_blk, p + 1);
        p++;
      }
    }
    for (uint32_t i = 0; i < 64; i++)
      if ((tmask >> i) & 1) ins[g0 + i] = 1;
  }
}

int main(void) {
  uint32_t hdr[5];
  int bad = 0;
  while (fread(hdr, 4, 5, stdin) == 5) {
    const uint32_t chain = hdr[0], lazy = hdr[1], nice = hdr[2], n = hdr[3];
    R = hdr[4];
    uint8_t* s = calloc(n + 16, 1);
    if (fread(s, 1, n, stdin) != n) return 2;
    // superset records
    rec = calloc((size_t)(n + 1) * R, 2);
    ins = calloc(n + 64, 1);
    static int32_t last[32768];
    for (int i = 0; i < 32768; i++) last[i] = -1;
    uint32_t* sprev = calloc(n + 1, 4);
    for (uint32_t q = 0; q + 2 < n; q++) {
      const uint32_t hq = hash3(s, q);
      sprev[q] = last[hq] < 0 ? 0xffffffffu : (uint32_t)last[hq];
      last[hq] = (int32_t)q;
      uint32_t c = q;
      for (uint32_t r = 0; r < R; r++) {
        c = c == 0xffffffffu ? c : sprev[c];
        if (c == 0xffffffffu || q - c > 32767u) break;
        rec[(size_t)q * R + r] = (uint16_t)(q - c);
      }
    }
    out_t a = {calloc(n + 1, 4), 0, calloc(n / SYM_END + 4, 4), 0};
    out_t b = {calloc(n + 1, 4), 0, calloc(n / SYM_END + 4, 4), 0};
    g_walks = g_chases = g_rewalks = g_steps = g_cand = g_skipped = g_incomplete = 0;
    serial(s, n, chain, lazy, nice, &a);
    grouped(s, n, chain, lazy, nice, &b);
    uint32_t at = 0;
    while (at < a.nsym && at < b.nsym && a.sym[at] == b.sym[at]) at++;
    if (at != a.nsym || a.nsym != b.nsym || a.ncut != b.ncut || memcmp(a.cut, b.cut, 4ull * a.ncut) != 0) {
      printf("MISMATCH n=%u at %u of %u/%u\n", n, at, a.nsym, b.nsym);
      bad = 1;
    } else {
      printf("ok n=%u R=%u syms=%u walks=%llu incomplete walks=%llu cand=%llu skipped=%llu steps=%llu rewalks=%llu "
             "(of them incomplete %llu)\n", n, R, a.nsym, (unsigned long long)g_walks, (unsigned long long)g_chases,
             (unsigned long long)g_cand, (unsigned long long)g_skipped, (unsigned long long)g_steps,
             (unsigned long long)g_rewalks, (unsigned long long)g_incomplete);
    }
    free(s), free(rec), free(ins), free(sprev);
    free(a.sym), free(a.cut), free(b.sym), free(b.cut);
  }
  return bad;
}
