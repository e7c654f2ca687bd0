// emu_match_walk.c -- CPU model of zs_k_match's walk (deflate_match.hip):
// two chains per lane in lock-step, an ended chain frozen (key masked with
// am, limit INT_MAX), the rare >= 8-byte path, the two-phase chain >> 2
// snapshot, window coordinates and 0xffff "no link" entries -- checked
// position by position against a direct longest_match (deflate.ts:1053-1115)
// for both budgets.  The model pairs a tile's positions i and cnt-1-i (chains
// of very different lengths) to exercise the freezing harder than the
// kernel's sorted pairing does.  Test infrastructure (tests/test_emu_walk.py);
// it checks the walk's logic off the GPU, not the kernel binary.
//
// usage: emu_match_walk FILE CHAIN NICE; FILE = u32 count, u32 sizes[count], bytes
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#define MAXD 32506u
typedef struct { uint32_t p, cr, best, am, ok, kx, maxc, nice, sp, s0, s1, flag; int limit; } Ch;
static uint8_t wbb[65536 + 64];
static uint16_t pv[65536];
static uint32_t win_word(uint32_t off) { uint32_t v; memcpy(&v, wbb + off, 4); return v; }
static uint32_t ffbl(uint32_t x) { return x ? (uint32_t)__builtin_ctz(x) : 0xffffffffu; }
static uint32_t sadd(uint32_t a, uint32_t b) { uint64_t s = (uint64_t)a + b; return s > 0xffffffffu ? 0xffffffffu : (uint32_t)s; }
// direct reference: longest_match with chain budget
static uint32_t ref_lm(const uint8_t* b, const int32_t* prev, uint32_t n, uint32_t p, uint32_t budget, uint32_t nice_cfg) {
  int32_t cur = prev[p];
  if (p + 2 >= n || cur <= 0 || p - (uint32_t)cur > MAXD) return 0xffffffffu;  // no head
  uint32_t look = n - p, maxc = look < 258 ? look : 258, nice = look < nice_cfg ? look : nice_cfg;
  int limit = p > MAXD ? (int)(p - MAXD) : 0; uint32_t bl = 2, bd = 0, st = 0;
  for (;;) {
    st++;
    uint32_t k = 0; while (k < maxc && b[cur + k] == b[p + k]) k++;
    if (k > bl) { bl = k; bd = p - cur; if (k >= nice) break; }
    if (st >= budget) break;
    int32_t nx = prev[cur]; if (nx <= limit) break; cur = nx;
  }
  return (bl << 16) | (bl > 2 ? bd : 0);
}
int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s FILE CHAIN NICE\n", argv[0]); return 2; }
  FILE* f = fopen(argv[1], "rb"); uint32_t chain = atoi(argv[2]), nice_cfg = atoi(argv[3]);
  if (!f) return 2;
  static uint8_t buf[65536 + 64]; static int32_t head[32768], prev[65536];
  static uint16_t lpv[65536];
  uint32_t ns = 0, sizes[4096];
  if (fread(&ns, 4, 1, f) != 1 || ns > 4096 || fread(sizes, 4, ns, f) != ns) return 2;
  long bad = 0, checked = 0;
  for (uint32_t si = 0; si < ns; si++) {
    const uint32_t n = sizes[si];
    if (n > 65536) return 2;
    memset(buf, 0, sizeof buf);
    if (fread(buf, 1, n, f) != n) return 2;
    // prev links: distance to the previous same-hash position, 0xffff = none
    // (farther than 32767, or the NIL position 0); prev[] = that position or 0
    for (int i = 0; i < 32768; i++) head[i] = -1;
    for (uint32_t p = 0; p < n; p++) {
      prev[p] = 0; pv[p] = 0xffff;
      if (p + 2 >= n) continue;
      const uint32_t h = ((buf[p] << 10) ^ (buf[p + 1] << 5) ^ buf[p + 2]) & 0x7fff;
      const int32_t q = head[h];
      head[h] = (int32_t)p;
      if (q > 0 && p - (uint32_t)q <= 32767) { prev[p] = q; pv[p] = (uint16_t)(p - (uint32_t)q); }
    }
    for (uint32_t t0 = 0; t0 < n; t0 += 8192) {
      uint32_t t1 = t0 + 8192 < n ? t0 + 8192 : n, w0 = t0 > 32768 ? t0 - 32768 : 0;
      memset(wbb, 0, sizeof wbb); uint32_t w1 = t1 + 262 < n ? t1 + 262 : n;
      memcpy(wbb, buf + w0, w1 - w0);
      for (uint32_t i = 0; i < t1 - w0; i++) lpv[i] = pv[w0 + i];
      uint32_t cnt = t1 - t0;
      // pair positions i and cnt-1-i (dissimilar on purpose)
      for (uint32_t g = 0; g < cnt; g += 2) {
        Ch c[2];
        for (int j = 0; j < 2; j++) {
          uint32_t oi = j ? cnt - 1 - g / 2 : g / 2;  // arbitrary pairing
          if (g + j >= cnt) oi = 0xffffffffu;
          Ch* h = &c[j];
          int in = oi != 0xffffffffu && oi < cnt;
          h->p = in ? t0 + oi : 0xffffffffu;
          uint32_t p = h->p;
          uint32_t d0 = (in && p + 2 < n) ? lpv[p - w0] : 0xffffu;
          uint32_t q0 = p - d0;
          h->flag = d0 == MAXD ? 0x8000u : 0u;
          h->ok = (in && q0 != 0 && d0 <= MAXD) ? 1u : 0u;
          h->am = h->ok ? 0xffffffffu : 0u;
          uint32_t look = in ? n - p : 0u;
          h->maxc = look < 258 ? look : 258; h->nice = look < nice_cfg ? look : nice_cfg;
          h->limit = h->ok ? (p > MAXD ? (int)(p - MAXD) : 0) - (int)w0 : 0x7fffffff;
          h->sp = h->ok ? p - w0 : 0u;
          h->s0 = win_word(h->sp); h->s1 = win_word(h->sp + 4);
          h->best = (2u << 16) | 0xffffu;
          h->cr = h->ok ? q0 - w0 : 0u;
          h->kx = h->ok ? (h->nice < 8u ? h->nice : 8u) : 0xffffffffu;
        }
        uint32_t budget = chain, bsmall = chain >> 2, bs[2];
        for (int phase = 0; phase < 2; phase++) {
          uint32_t rem = phase ? budget - bsmall : bsmall;
          if (phase && !(bsmall < budget && (c[0].am | c[1].am))) break;
          for (;;) {
            uint32_t d[2], k[2];
            for (int j = 0; j < 2; j++) {
              uint32_t cp = c[j].cr;
              if (cp >= 65536) { printf("chain left the window: p=%u cr=%u\n", c[j].p, cp); return 1; }
              d[j] = lpv[cp];
              uint32_t x0 = win_word(cp) ^ c[j].s0, x1 = win_word(cp + 4) ^ c[j].s1;
              uint32_t f0 = ffbl(x0), f1 = sadd(ffbl(x1), 32);
              uint32_t m = f0 < f1 ? f0 : f1; m = m < 64 ? m : 64; k[j] = m >> 3;
            }
            for (int j = 0; j < 2; j++) {
              Ch* h = &c[j];
              if (k[j] >= h->kx) {
                uint32_t kk = k[j];
                if (kk == 8u) { while (kk < h->maxc) { uint32_t y = win_word(h->cr + kk) ^ win_word(h->sp + kk); if (y) { kk += __builtin_ctz(y) >> 3; break; } kk += 4; } }
                kk = kk < h->maxc ? kk : h->maxc;
                if (kk >= h->nice) d[j] = 0xffffu;
                k[j] = kk;
              }
              uint32_t key = ((k[j] << 16) | h->cr) & h->am; if (key > h->best) h->best = key;
              int nxt = (int)h->cr - (int)d[j];
              int go = nxt > h->limit;
              h->cr = go ? (uint32_t)nxt : h->cr; h->kx = go ? h->kx : 0xffffffffu; h->am = go ? h->am : 0u; h->limit = go ? h->limit : 0x7fffffff;
            }
            if (((c[0].am | c[1].am) == 0u) | (--rem == 0)) break;
          }
          if (phase == 0) { bs[0] = c[0].best; bs[1] = c[1].best; }
        }
        for (int j = 0; j < 2; j++) {
          Ch* h = &c[j]; if (h->p == 0xffffffffu) continue;
          uint32_t bl = h->best >> 16, bsl = bs[j] >> 16, rx = 0, ry = 0;
          if (h->ok) { rx = (bl << 16) | (bl > 2 ? h->sp - (h->best & 0xffffu) : 0u); ry = (bsl << 16) | (bsl > 2 ? h->sp - (bs[j] & 0xffffu) : 0u); }
          uint32_t ex = ref_lm(buf, prev, n, h->p, budget, nice_cfg), ey = ref_lm(buf, prev, n, h->p, bsmall, nice_cfg);
          if (ex == 0xffffffffu) { ex = 0; ey = 0; }
          checked++;
          if (rx != ex || ry != ey) { if (bad < 10) printf("n=%u p=%u got %08x/%08x want %08x/%08x\n", n, h->p, rx, ry, ex, ey); bad++; }
        }
      }
    }
  }
  printf("streams %u positions %ld mismatches %ld\n", ns, checked, bad);
  return bad != 0;
}
