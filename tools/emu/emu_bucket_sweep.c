// emu_bucket_sweep.c -- CPU model of the L4..L9 match finder (zs_k_bucket +
// zs_k_sweep, deflate_sweep.hip, over the windows of capi.cpp sweep_table), checked
// position by position against a direct longest_match (deflate.ts:1053-1115)
// for both budgets the lazy parse asks for (chain, chain >> 2 when
// prev_length >= good_match, deflate.ts:1075-1077) and for the slide-NIL flag.
//
// The model follows the kernels' data flow:
//   * members: the positions p <= n-3 (every one is inserted),
//     sorted by (15-bit hash, position) -- a counting sort whose scatter keeps
//     position order inside a bucket.  Member k's chain (deflate.ts:1109) is
//     then members k-1, k-2, ... of its own bucket: the t-th predecessor is
//     the t-th chain step, no links are followed.
//   * the sweep: for t = 1, 2, ... every lane compares its position with the
//     t-th predecessor's 11-byte signature (SIG; the kernel's sentinel bit
//     saturates the matched-byte count at 11); a candidate is alive while
//     key = hash << 16 | pos passes the head test (t = 1: non-NIL, distance
//     <= MAX_DIST, deflate.ts:1376) or the chain test (t >= 2: pos > limit,
//     deflate.ts:1109) and t <= budget; liveness is monotone in t.
//   * a candidate whose 11 signature bytes all match (and maxc > 12) is "long":
//     up to 4 are recorded (t, pos) and extended afterwards in chain order
//     with the nice cut-off (deflate.ts:1100-1105); a fifth ends the lane's
//     sweep and the lane re-walks its chain from the first long candidate.
//   * short candidates keep the first max of (len, -t) (first strictly longer
//     wins), clamped to maxc (deflate.ts:1068); when any long candidate is
//     within the budget the result comes from the long ones only.
//   * lanes with maxc <= 12 (the last positions of a stream) record no long
//     candidates; their result is an exact re-walk, min(lcp, maxc), first max.
//   * windows: a stream of up to 65,537 bytes is one window; a longer one has a
//     first window owning positions [0, 65520) and then windows owning 32,752
//     positions each after a 32,768-position look-back; the members of a window
//     are its first min(65,535, bytes - 2) positions, its signature form comes
//     from its loaded bytes, and only own positions are compared.
// Test infrastructure (tests/test_emu_sweep.py); it checks the algorithm off
// the GPU, not the kernel binary (tests/test_gpu_deflate.py does that).
//
// usage: emu_bucket_sweep FILE CHAIN NICE; FILE = u32 count, u32 sizes[count], bytes
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define MAXD 32506u
#define NLONG 4
#define SIG 11u

#define MAXN (1u << 20)
#define WIN_BYTES (4u * ((65535u + 258u + 20u + 3u) / 4u + 2u))  // ZS_SW_WIN_WORDS
static uint8_t buf[MAXN + 65536 + 300];
static const uint8_t* B = buf;  // the current window
static int32_t head[32768], prev[MAXN];
static uint32_t cnt[32768], off[32768];
static uint16_t mem[65536];

static uint32_t hash3(uint32_t p) { return ((B[p] << 10) ^ (B[p + 1] << 5) ^ B[p + 2]) & 0x7fff; }

// direct reference: longest_match with a chain budget; returns len << 16 | dist
// (dist only when len > 2), 0 when the reference does not call it (no head)
static uint32_t ref_lm(uint32_t n, uint32_t p, uint32_t budget, uint32_t nice_cfg) {
  int32_t cur = prev[p];
  if (p + 2 >= n || cur <= 0 || p - (uint32_t)cur > MAXD) return 0;
  uint32_t look = n - p, maxc = look < 258 ? look : 258, nice = look < nice_cfg ? look : nice_cfg;
  int limit = p > MAXD ? (int)(p - MAXD) : 0;
  uint32_t bl = 2, bd = 0, st = 0;
  for (;;) {
    st++;
    uint32_t k = 0;
    while (k < maxc && buf[cur + k] == buf[p + k]) k++;
    if (k > bl) { bl = k; bd = p - cur; if (k >= nice) break; }
    if (st >= budget) break;
    int32_t nx = prev[cur];
    if (nx <= limit) break;
    cur = nx;
  }
  return (bl << 16) | (bl > 2 ? bd : 0);
}

static int a7;  // stream bytes all < 0x80: the kernel's 8-byte signature [X, b3..b9] (deflate_sweep.hip SwSig<true>)
static uint32_t x7(uint32_t p) { return ((B[p] >> 5) & 3) | ((B[p + 1] & 7) << 2) | (((B[p + 1] >> 5) & 3) << 5); }
// matched signature bytes (sigma) of a candidate
static uint32_t lcp_sig(uint32_t a, uint32_t b) {
  uint32_t k = 0;
  if (a7) {
    if (x7(a) != x7(b)) return 0;
    k = 1;
    while (k < 8 && B[a + k + 2] == B[b + k + 2]) k++;
    return k;
  }
  while (k < SIG && B[a + k] == B[b + k]) k++;
  return k;
}
static uint32_t sig_len(uint32_t sigma) { return a7 ? (sigma ? sigma + 2 : 2) : sigma; }
#define SIGN (a7 ? 8u : SIG)    // signature bytes
#define EXTB (a7 ? 10u : SIG)   // bytes known equal for a full signature match

// exact length of a long candidate (a full signature match), clamped to maxc
static uint32_t extend(uint32_t p, uint32_t q, uint32_t maxc) {
  uint32_t k = EXTB;
  while (k < maxc && B[q + k] == B[p + k]) k++;
  return k < maxc ? k : maxc;
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s FILE CHAIN NICE\n", argv[0]); return 2; }
  FILE* f = fopen(argv[1], "rb");
  const uint32_t chain = atoi(argv[2]), nice_cfg = atoi(argv[3]), chain_s = chain >> 2;
  if (!f) return 2;
  uint32_t ns = 0, sizes[4096];
  if (fread(&ns, 4, 1, f) != 1 || ns > 4096 || fread(sizes, 4, ns, f) != ns) return 2;
  long bad = 0, checked = 0, checked7 = 0, overflow = 0, longs = 0, steps = 0, windows = 0;
  for (uint32_t si = 0; si < ns; si++) {
    const uint32_t n = sizes[si];
    if (n > MAXN) return 2;
    memset(buf, 0, sizeof buf);
    if (fread(buf, 1, n, f) != n) return 2;
    B = buf;
    // reference chains (for ref_lm)
    for (int i = 0; i < 32768; i++) head[i] = -1;
    for (uint32_t p = 0; p < n; p++) {
      prev[p] = 0;
      if (p + 2 >= n) continue;
      const uint32_t h = hash3(p);
      if (head[h] > 0) prev[p] = head[h];
      head[h] = (int32_t)p;
    }
    for (uint32_t lo = 0; lo < n; lo += lo == 0 ? 65520u : 32752u) {  // capi.cpp sweep_table
      const uint32_t base = n <= 65537u || lo == 0 ? 0u : lo - 32768u;
      const uint32_t olo = lo - base, ohi = n <= 65537u ? n : lo == 0 ? 65520u : 32768u + 32752u;
      B = buf + base;
      windows++;
      const uint32_t nrel = n - base;  // the model sees the window's bytes to the stream's end
      a7 = 1;
      for (uint32_t i = 0; i < nrel && i < WIN_BYTES; i++) a7 &= B[i] < 0x80;
      // zs_k_bucket: counting sort of the inserted positions by hash (stable)
      const uint32_t m = nrel > 2 ? (nrel - 2 < ohi ? nrel - 2 : ohi) : 0;
      memset(cnt, 0, sizeof cnt);
      for (uint32_t p = 0; p < m; p++) cnt[hash3(p)]++;
      uint32_t run = 0;
      for (int h = 0; h < 32768; h++) { off[h] = run; run += cnt[h]; }
      for (uint32_t p = 0; p < m; p++) mem[off[hash3(p)]++] = (uint16_t)p;
      // zs_k_sweep, one lane per member: lock-step groups of steps, each group
      // folding its candidates' matched-bit counts into one maximum
      for (uint32_t k = 0; k < m; k++) {
        const uint32_t p = mem[k], h = hash3(p);
        if (p < olo || p >= ohi) continue;  // another window's position
        const uint32_t look = nrel - p, maxc = look < 258 ? look : 258, nice = look < nice_cfg ? look : nice_cfg;
        const int tail = maxc <= 12;
        const uint32_t limit = p > MAXD ? p - MAXD : 0;
        const uint32_t khead = (h << 16) | (limit > 1 ? limit : 1), klim = (h << 16) | limit;
        // live(t): the head needs key >= khead, the chain key > klim; monotone in t
#define LIVE(t) ((t) <= k && ((t) == 1 ? ((hash3(mem[k - 1]) << 16) | mem[k - 1]) >= khead \
                                       : ((hash3(mem[k - (t)]) << 16) | mem[k - (t)]) > klim))
        const int headok = LIVE(1);  // else no head candidate: the parse never searches here (result 0)
        const uint32_t flag = headok && (p - mem[k - 1] == MAXD) ? 0x8000u : 0u;
        const uint32_t thr0 = a7 ? 7 : 23;
        uint32_t thr = thr0, bt = 0, thr_s = thr0, bt_s = 0, nlg = 0, lg[NLONG];
        int ovf = 0;
        // groups: {1}, {2..4}, then 8 steps (4 where a block end or the chain >> 2 snapshot cuts it)
        for (uint32_t t0 = 1; headok && t0 <= chain; ) {
          uint32_t t1 = t0 == 1 ? 1 : t0 == 2 ? 4 : t0 + 7;
          const uint32_t blk_end = (t0 + 63) / 64 * 64;
          if (t1 > blk_end) t1 = blk_end;
          if (t0 <= chain_s && t1 > chain_s) t1 = chain_s;
          if (t1 > chain) t1 = chain;
          uint32_t gm = 0;
          for (uint32_t t = t0; t <= t1; t++) {
            if (!LIVE(t)) continue;
            steps++;
            const uint32_t mm = 8 * lcp_sig(p, mem[k - t]) + (lcp_sig(p, mem[k - t]) < SIGN ? (uint32_t)(rand() & 7) : 0);
            if (mm > gm) gm = mm;
          }
          if (gm > thr) { thr = gm | 7; bt = t0 | (t1 << 16); }
          if (!tail && gm >= 8 * SIGN) {
            if (nlg < NLONG) lg[nlg++] = t0 | (t1 << 16);
            else ovf = 1;
          }
          if (t1 == chain_s) { thr_s = thr; bt_s = bt; }
          t0 = t1 + 1;
        }
        if (chain_s == 0) { thr_s = thr; bt_s = bt; }
        // the first live step of group g whose signature matches exactly B bytes
        uint32_t best_t = 0, best_ts = 0;
        for (int pass = 0; pass < 2; pass++) {
          const uint32_t g = pass ? bt_s : bt, B = (pass ? thr_s : thr) >> 3;
          uint32_t found = 0;
          if (g)
            for (uint32_t t = g & 0xffff; t <= (g >> 16) && !found; t++)
              if (LIVE(t) && lcp_sig(p, mem[k - t]) == B) found = t;
          if (pass) best_ts = found; else best_t = found;
        }
        uint32_t bl = best_t ? sig_len(thr >> 3) : 2, bd = best_t ? p - mem[k - best_t] : 0;
        uint32_t bsl = best_ts ? sig_len(thr_s >> 3) : 2, bsd = best_ts ? p - mem[k - best_ts] : 0;
        if (!headok) {
          bl = bsl = 0;
        } else if (tail) {  // maxc <= 12: exact re-walk, min(lcp, maxc), first max (deflate.ts:1082-1105)
          uint32_t best = 2u << 16, best_s = best;
          for (uint32_t t = 1; t <= chain && LIVE(t); t++) {
            const uint32_t q = mem[k - t];
            uint32_t L = 0;
            while (L < 12 && B[q + L] == B[p + L]) L++;
            const uint32_t score = ((L < maxc ? L : maxc) << 16) | (0xffffu - t);
            if (score > best) best = score;
            if (t <= chain_s && score > best_s) best_s = score;
          }
          bl = best >> 16; bd = bl > 2 ? p - mem[k - (0xffffu - (best & 0xffffu))] : 0;
          bsl = best_s >> 16; bsd = bsl > 2 ? p - mem[k - (0xffffu - (best_s & 0xffffu))] : 0;
        } else if (nlg) {  // long candidates: extended in chain order with the nice cut-off
          longs += nlg;
          uint32_t lb = 0, ld = 0, lbs = 0, lds = 0;
          int stop = 0;
          for (uint32_t i = 0; i < nlg && !stop; i++) {
            const uint32_t ta = ovf ? lg[0] & 0xffff : lg[i] & 0xffff, tz = ovf ? chain : lg[i] >> 16;
            for (uint32_t t = ta; t <= tz && LIVE(t); t++) {
              const uint32_t q = mem[k - t];
              if (lcp_sig(p, q) < SIGN) continue;
              const uint32_t L = extend(p, q, maxc);
              if (L > lb) { lb = L; ld = p - q; }
              if (t <= chain_s && L > lbs) { lbs = L; lds = p - q; }
              if (L >= nice) { stop = 1; break; }
            }
            if (ovf) { overflow++; break; }
          }
          bl = lb; bd = ld;
          if (lbs) { bsl = lbs; bsd = lds; }
        }
        const uint32_t rx = headok ? (bl << 16) | (bl > 2 ? bd : 0) | flag : 0;
        const uint32_t ry = headok ? (bsl << 16) | (bsl > 2 ? bsd : 0) : 0;
        // reference
        const uint32_t gp = base + p;
        const uint32_t ex = ref_lm(n, gp, chain, nice_cfg);
        const uint32_t ey = ref_lm(n, gp, chain_s ? chain_s : 1, nice_cfg);
        const uint32_t ef = (ex && prev[gp] > 0 && gp - (uint32_t)prev[gp] == MAXD) ? 0x8000u : 0u;
        checked++;
        checked7 += a7;
        if (rx != (ex | ef) || ry != ey) {
          if (bad < 10)
            printf("stream %u pos %u: got %08x/%08x want %08x/%08x\n", si, gp, rx, ry, ex | ef, ey);
          bad++;
        }
      }
      if (n <= 65537u) break;
    }
  }
  printf("checked %ld positions (%ld in 7-bit windows) in %ld windows, mismatches %ld, sweep steps %ld, long "
         "candidates %ld, overflow lanes %ld\n", checked, checked7, windows, bad, steps, longs, overflow);
  return bad != 0;
}
