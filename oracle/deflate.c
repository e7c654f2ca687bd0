/*
 * oracle/deflate.c -- CPU restatement of the reference's deflate engine.
 *
 * TEST INFRASTRUCTURE ONLY (see zoracle.h).  Never linked into the product.
 *
 * Restates /root/reference/src/mod/deflate/{deflate,trees,utils,constants}.ts
 * for levels 1..9, strategy 0, memLevel 8, windowBits 15 -- the only
 * configuration reachable from CompressionStream (streams.ts:216-228).
 * Level 0 (deflate_stored, deflate.ts:1140-1279) is not restated here; the
 * oracle reports ZO_STREAM_ERROR for it.
 */
#include <stdlib.h>
#include <string.h>
#include "zoracle.h"

/* deflate/constants.ts:15-41 */
#define MIN_MATCH 3
#define MAX_MATCH 258
#define MIN_LOOKAHEAD (MAX_MATCH + MIN_MATCH + 1)
#define TOO_FAR 4096
#define WIN_INIT MAX_MATCH
#define LENGTH_CODES 29
#define LITERALS 256
#define L_CODES (LITERALS + 1 + LENGTH_CODES)
#define D_CODES 30
#define BL_CODES 19
#define HEAP_SIZE (2 * L_CODES + 1)
#define MAX_BITS 15
#define MAX_BL_BITS 7
#define END_BLOCK 256
#define REP_3_6 16
#define REPZ_3_10 17
#define REPZ_11_138 18
#define OS_CODE 255

#define W_BITS 15
#define W_SIZE (1u << W_BITS)
#define W_MASK (W_SIZE - 1)
#define HASH_BITS 15 /* memLevel 8 + 7, deflate.ts:312 */
#define HASH_SIZE (1u << HASH_BITS)
#define HASH_MASK (HASH_SIZE - 1)
#define HASH_SHIFT 5 /* (15+3-1)/3 truncated by `<<`, deflate.ts:315,110 */
#define LIT_BUFSIZE 16384 /* 1 << (memLevel + 6), deflate.ts:321 */
#define SYM_END (LIT_BUFSIZE - 1) /* symbols per block, deflate.ts:336 */
#define MAX_DIST (W_SIZE - MIN_LOOKAHEAD) /* deflate/utils.ts:83-85 */
#define IN_CHUNK (32 * 1024) /* streams.ts:7 */

enum { NEED_MORE, BLOCK_DONE, FINISH_STARTED, FINISH_DONE }; /* deflate/types.ts:11-16 */
enum { ST_INIT, ST_GZIP, ST_BUSY, ST_FINISH };

/* Per-level tuning, deflate.ts:86-103: good, lazy, nice, chain, slow? */
static const struct { int good, lazy, nice, chain, slow; } CONFIG[10] = {
    {0, 0, 0, 0, 0},         {4, 4, 8, 4, 0},       {4, 5, 16, 8, 0},
    {4, 6, 32, 32, 0},       {4, 4, 16, 16, 1},     {8, 16, 32, 32, 1},
    {8, 16, 128, 128, 1},    {8, 32, 128, 256, 1},  {32, 128, 258, 1024, 1},
    {32, 258, 258, 4096, 1}};

/* static tables (deflate/constants.ts:55-68, common/constants.ts:48-71) */
static const int EXTRA_LBITS[LENGTH_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                              1, 1, 2, 2, 2, 2, 3, 3, 3, 3,
                                              4, 4, 4, 4, 5, 5, 5, 5, 0};
static const int EXTRA_DBITS[D_CODES] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3,
                                         4, 4, 5, 5, 6, 6, 7, 7, 8, 8,
                                         9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const int EXTRA_BLBITS[BL_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                           0, 0, 0, 0, 0, 0, 2, 3, 7};
static const uint8_t BL_ORDER[BL_CODES] = {16, 17, 18, 0, 8,  7, 9,  6, 10, 5,
                                           11, 4,  12, 3, 13, 2, 14, 1, 15};
static const int BASE_LENGTH[LENGTH_CODES] = {
    0,  1,  2,  3,  4,  5,  6,   7,   8,   10,  12,  14,  16,  20, 24,
    28, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 0};
static const int BASE_DIST[D_CODES] = {
    0,    1,    2,    3,     4,     6,     8,    12,   16,   24,
    32,   48,   64,   96,    128,   192,   256,  384,  512,  768,
    1024, 1536, 2048, 3072,  4096,  6144,  8192, 12288, 16384, 24576};

typedef struct { uint16_t freq, code, dad, len; } node_t; /* common/types.ts:153-158 */

static node_t STATIC_LTREE[L_CODES + 2];
static node_t STATIC_DTREE[D_CODES];
static uint8_t LENGTH_CODE[MAX_MATCH - MIN_MATCH + 1];
static uint8_t DIST_CODE[512];
static int tables_ready = 0;

static unsigned bit_reverse(unsigned v, int n) { /* deflate/utils.ts:36-44 */
  unsigned r = 0;
  while (n-- > 0) { r = (r << 1) | (v & 1); v >>= 1; }
  return r;
}

/* Canonical static trees and code lookups, deflate/trees-util.ts:3-137 */
static void init_tables(void) {
  if (tables_ready) return;
  int lens[L_CODES + 2];
  int n;
  for (n = 0; n <= 143; n++) lens[n] = 8;
  for (; n <= 255; n++) lens[n] = 9;
  for (; n <= 279; n++) lens[n] = 7;
  for (; n <= 287; n++) lens[n] = 8;
  uint16_t count[MAX_BITS + 1] = {0}, next[MAX_BITS + 2];
  for (n = 0; n < L_CODES + 2; n++) count[lens[n]]++;
  unsigned code = 0;
  count[0] = 0;
  for (int b = 1; b <= MAX_BITS; b++) { code = (code + count[b - 1]) << 1; next[b] = (uint16_t)code; }
  for (n = 0; n < L_CODES + 2; n++) {
    STATIC_LTREE[n].len = (uint16_t)lens[n];
    STATIC_LTREE[n].code = (uint16_t)bit_reverse(next[lens[n]]++, lens[n]);
  }
  for (n = 0; n < D_CODES; n++) {
    STATIC_DTREE[n].len = 5;
    STATIC_DTREE[n].code = (uint16_t)bit_reverse((unsigned)n, 5);
  }
  /* LENGTH_CODE[len - MIN_MATCH] */
  for (int c = 0; c < LENGTH_CODES - 1; c++)
    for (int k = 0; k < (1 << EXTRA_LBITS[c]); k++) LENGTH_CODE[BASE_LENGTH[c] + k] = (uint8_t)c;
  LENGTH_CODE[MAX_MATCH - MIN_MATCH] = LENGTH_CODES - 1;
  /* compact DIST_CODE: index dist<256 ? dist : 256 + (dist>>7), deflate/utils.ts:87-89 */
  int dist = 0;
  for (int c = 0; c < 16; c++)
    for (int k = 0; k < (1 << EXTRA_DBITS[c]); k++) DIST_CODE[dist++] = (uint8_t)c;
  dist >>= 7;
  for (int c = 16; c < D_CODES; c++)
    for (int k = 0; k < (1 << (EXTRA_DBITS[c] - 7)); k++) DIST_CODE[256 + dist++] = (uint8_t)c;
  tables_ready = 1;
}

static int d_code(unsigned dist) { return dist < 256 ? DIST_CODE[dist] : DIST_CODE[256 + (dist >> 7)]; }

typedef struct {
  node_t *dyn;
  const node_t *stat;
  const int *extra;
  int extra_base, elems, max_length, max_code;
} desc_t;

typedef struct {
  /* z_stream view */
  const uint8_t *next_in;
  size_t avail_in, total_in;
  uint32_t adler;
  uint8_t *out;
  size_t cap, out_len;
  int overflow;
  /* engine state, common/types.ts DeflateState */
  int wrap, level, status;
  uint8_t window[2 * W_SIZE];
  uint16_t prev[W_SIZE], head[HASH_SIZE];
  unsigned ins_h;
  long block_start;
  unsigned match_length, prev_match, match_available, strstart, match_start, lookahead;
  unsigned prev_length, max_chain, max_lazy, good_match, nice_match, insert;
  unsigned long w_have;
  /* trees */
  node_t dyn_ltree[HEAP_SIZE], dyn_dtree[2 * D_CODES + 1], bl_tree[2 * BL_CODES + 1];
  desc_t l_desc, d_desc, bl_desc;
  uint16_t bl_count[MAX_BITS + 1];
  int heap[2 * L_CODES + 1], heap_len, heap_max;
  uint8_t depth[2 * L_CODES + 1];
  uint16_t sym_dist[LIT_BUFSIZE];
  uint8_t sym_lc[LIT_BUFSIZE];
  unsigned sym_next;
  unsigned long opt_len, static_len;
  /* bit writer: LSB-first; byte stream identical to trees.ts:31-88 */
  uint64_t bi_buf;
  int bi_valid;
  int blocks;
} dstate;

static __thread int g_last_blocks;
int zo_last_block_count(void) { return g_last_blocks; }

/* ---------------------------------------------------------------- output */
static void put_byte(dstate *s, unsigned c) {
  if (s->out_len < s->cap) s->out[s->out_len] = (uint8_t)c;
  else s->overflow = 1;
  s->out_len++;
}
static void put_short(dstate *s, unsigned w) { put_byte(s, w & 0xff); put_byte(s, (w >> 8) & 0xff); }
static void put_short_msb(dstate *s, unsigned w) { put_byte(s, (w >> 8) & 0xff); put_byte(s, w & 0xff); }

static void send_bits(dstate *s, unsigned value, int length) { /* trees.ts:78-88 */
  s->bi_buf |= (uint64_t)value << s->bi_valid;
  s->bi_valid += length;
  while (s->bi_valid >= 8) { put_byte(s, (unsigned)(s->bi_buf & 0xff)); s->bi_buf >>= 8; s->bi_valid -= 8; }
}
static void bi_windup(dstate *s) { /* trees.ts:43-52 */
  if (s->bi_valid > 0) put_byte(s, (unsigned)(s->bi_buf & 0xff));
  s->bi_buf = 0;
  s->bi_valid = 0;
}

/* ----------------------------------------------------------------- trees */
static void init_block(dstate *s) { /* trees.ts:90-103 */
  for (int n = 0; n < L_CODES; n++) s->dyn_ltree[n].freq = 0;
  for (int n = 0; n < D_CODES; n++) s->dyn_dtree[n].freq = 0;
  for (int n = 0; n < BL_CODES; n++) s->bl_tree[n].freq = 0;
  s->dyn_ltree[END_BLOCK].freq = 1;
  s->opt_len = s->static_len = 0;
  s->sym_next = 0;
}

static void tr_init(dstate *s) { /* trees.ts:105-152 */
  memset(s->dyn_ltree, 0, sizeof s->dyn_ltree);
  memset(s->dyn_dtree, 0, sizeof s->dyn_dtree);
  memset(s->bl_tree, 0, sizeof s->bl_tree);
  s->l_desc = (desc_t){s->dyn_ltree, STATIC_LTREE, EXTRA_LBITS, LITERALS + 1, L_CODES, MAX_BITS, 0};
  s->d_desc = (desc_t){s->dyn_dtree, STATIC_DTREE, EXTRA_DBITS, 0, D_CODES, MAX_BITS, 0};
  s->bl_desc = (desc_t){s->bl_tree, NULL, EXTRA_BLBITS, 0, BL_CODES, MAX_BL_BITS, 0};
  s->bi_buf = 0;
  s->bi_valid = 0;
  init_block(s);
}

/* heap ordering: freq, then depth (<=), trees.ts:163-165 */
static int smaller(const node_t *t, int n, int m, const uint8_t *depth) {
  return t[n].freq < t[m].freq || (t[n].freq == t[m].freq && depth[n] <= depth[m]);
}

static void pqdownheap(dstate *s, const node_t *tree, int k) { /* trees.ts:167-185 */
  int v = s->heap[k];
  int j = k << 1;
  while (j <= s->heap_len) {
    if (j < s->heap_len && smaller(tree, s->heap[j + 1], s->heap[j], s->depth)) j++;
    if (smaller(tree, v, s->heap[j], s->depth)) break;
    s->heap[k] = s->heap[j];
    k = j;
    j <<= 1;
  }
  s->heap[k] = v;
}

static void gen_bitlen(dstate *s, desc_t *desc) { /* trees.ts:187-259 */
  node_t *tree = desc->dyn;
  const int max_code = desc->max_code, base = desc->extra_base, max_length = desc->max_length;
  int h, n, m, bits, xbits, overflow = 0;
  unsigned f;
  for (bits = 0; bits <= MAX_BITS; bits++) s->bl_count[bits] = 0;
  tree[s->heap[s->heap_max]].len = 0;
  for (h = s->heap_max + 1; h < HEAP_SIZE; h++) {
    n = s->heap[h];
    bits = tree[tree[n].dad].len + 1;
    if (bits > max_length) { bits = max_length; overflow++; }
    tree[n].len = (uint16_t)bits;
    if (n > max_code) continue; /* internal node */
    s->bl_count[bits]++;
    xbits = n >= base ? desc->extra[n - base] : 0;
    f = tree[n].freq;
    s->opt_len += (unsigned long)f * (unsigned)(bits + xbits);
    if (desc->stat) s->static_len += (unsigned long)f * (unsigned)(desc->stat[n].len + xbits);
  }
  if (overflow == 0) return;
  do {
    bits = max_length - 1;
    while (s->bl_count[bits] == 0) bits--;
    s->bl_count[bits]--;
    s->bl_count[bits + 1] += 2;
    s->bl_count[max_length]--;
    overflow -= 2;
  } while (overflow > 0);
  for (bits = max_length; bits != 0; bits--) {
    n = s->bl_count[bits];
    while (n != 0) {
      m = s->heap[--h];
      if (m > max_code) continue;
      if (tree[m].len != (unsigned)bits) {
        s->opt_len += ((unsigned long)bits - tree[m].len) * tree[m].freq;
        tree[m].len = (uint16_t)bits;
      }
      n--;
    }
  }
}

static void gen_codes(node_t *tree, int max_code, const uint16_t *bl_count) { /* trees.ts:54-76 */
  uint16_t next_code[MAX_BITS + 1];
  unsigned code = 0;
  for (int bits = 1; bits <= MAX_BITS; bits++) { code = (code + bl_count[bits - 1]) << 1; next_code[bits] = (uint16_t)code; }
  for (int n = 0; n <= max_code; n++) {
    int len = tree[n].len;
    if (len == 0) continue;
    tree[n].code = (uint16_t)bit_reverse(next_code[len]++, len);
  }
}

static void build_tree(dstate *s, desc_t *desc) { /* trees.ts:261-316 */
  node_t *tree = desc->dyn;
  int elems = desc->elems, n, m, max_code = -1, node;
  s->heap_len = 0;
  s->heap_max = HEAP_SIZE;
  for (n = 0; n < elems; n++) {
    if (tree[n].freq != 0) { s->heap[++s->heap_len] = max_code = n; s->depth[n] = 0; }
    else tree[n].len = 0;
  }
  while (s->heap_len < 2) { /* force at least two codes */
    node = s->heap[++s->heap_len] = (max_code < 2 ? ++max_code : 0);
    tree[node].freq = 1;
    s->depth[node] = 0;
    s->opt_len--;
    if (desc->stat) s->static_len -= desc->stat[node].len;
  }
  desc->max_code = max_code;
  for (n = s->heap_len / 2; n >= 1; n--) pqdownheap(s, tree, n);
  node = elems;
  do {
    n = s->heap[1];
    s->heap[1] = s->heap[s->heap_len--];
    pqdownheap(s, tree, 1);
    m = s->heap[1];
    s->heap[--s->heap_max] = n;
    s->heap[--s->heap_max] = m;
    tree[node].freq = (uint16_t)(tree[n].freq + tree[m].freq);
    s->depth[node] = (uint8_t)((s->depth[n] >= s->depth[m] ? s->depth[n] : s->depth[m]) + 1);
    tree[n].dad = tree[m].dad = (uint16_t)node;
    s->heap[1] = node++;
    pqdownheap(s, tree, 1);
  } while (s->heap_len >= 2);
  s->heap[--s->heap_max] = s->heap[1];
  gen_bitlen(s, desc);
  gen_codes(tree, desc->max_code, s->bl_count);
}

/* tree run-length statistics / emission, trees.ts:318-414 */
static void scan_tree(dstate *s, node_t *tree, int max_code) {
  int prevlen = -1, curlen, nextlen = tree[0].len, count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) { max_count = 138; min_count = 3; }
  tree[max_code + 1].len = 0xffff; /* guard */
  for (int n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = tree[n + 1].len;
    if (++count < max_count && curlen == nextlen) continue;
    else if (count < min_count) s->bl_tree[curlen].freq = (uint16_t)(s->bl_tree[curlen].freq + count);
    else if (curlen != 0) {
      if (curlen != prevlen) s->bl_tree[curlen].freq++;
      s->bl_tree[REP_3_6].freq++;
    } else if (count <= 10) s->bl_tree[REPZ_3_10].freq++;
    else s->bl_tree[REPZ_11_138].freq++;
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    else if (curlen == nextlen) { max_count = 6; min_count = 3; }
    else { max_count = 7; min_count = 4; }
  }
}

static void send_code(dstate *s, int c, const node_t *tree) { send_bits(s, tree[c].code, tree[c].len); }

static void send_tree(dstate *s, node_t *tree, int max_code) {
  int prevlen = -1, curlen, nextlen = tree[0].len, count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) { max_count = 138; min_count = 3; }
  for (int n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = tree[n + 1].len;
    if (++count < max_count && curlen == nextlen) continue;
    else if (count < min_count) { do send_code(s, curlen, s->bl_tree); while (--count != 0); }
    else if (curlen != 0) {
      if (curlen != prevlen) { send_code(s, curlen, s->bl_tree); count--; }
      send_code(s, REP_3_6, s->bl_tree);
      send_bits(s, (unsigned)(count - 3), 2);
    } else if (count <= 10) { send_code(s, REPZ_3_10, s->bl_tree); send_bits(s, (unsigned)(count - 3), 3); }
    else { send_code(s, REPZ_11_138, s->bl_tree); send_bits(s, (unsigned)(count - 11), 7); }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    else if (curlen == nextlen) { max_count = 6; min_count = 3; }
    else { max_count = 7; min_count = 4; }
  }
}

static int build_bl_tree(dstate *s) { /* trees.ts:416-432 */
  scan_tree(s, s->dyn_ltree, s->l_desc.max_code);
  scan_tree(s, s->dyn_dtree, s->d_desc.max_code);
  build_tree(s, &s->bl_desc);
  int max_blindex;
  for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
    if (s->bl_tree[BL_ORDER[max_blindex]].len != 0) break;
  s->opt_len += 3 * ((unsigned long)max_blindex + 1) + 5 + 5 + 4;
  return max_blindex;
}

static void send_all_trees(dstate *s, int lcodes, int dcodes, int blcodes) { /* trees.ts:434-447 */
  send_bits(s, (unsigned)(lcodes - 257), 5);
  send_bits(s, (unsigned)(dcodes - 1), 5);
  send_bits(s, (unsigned)(blcodes - 4), 4);
  for (int rank = 0; rank < blcodes; rank++) send_bits(s, s->bl_tree[BL_ORDER[rank]].len, 3);
  send_tree(s, s->dyn_ltree, lcodes - 1);
  send_tree(s, s->dyn_dtree, dcodes - 1);
}

static void compress_block(dstate *s, const node_t *ltree, const node_t *dtree) { /* trees.ts:476-520 */
  for (unsigned i = 0; i < s->sym_next; i++) {
    unsigned dist = s->sym_dist[i];
    int lc = s->sym_lc[i];
    if (dist == 0) {
      send_code(s, lc, ltree);
    } else {
      int code = LENGTH_CODE[lc];
      send_code(s, code + LITERALS + 1, ltree);
      int extra = EXTRA_LBITS[code];
      if (extra) send_bits(s, (unsigned)(lc - BASE_LENGTH[code]), extra);
      dist--;
      code = d_code(dist);
      send_code(s, code, dtree);
      extra = EXTRA_DBITS[code];
      if (extra) send_bits(s, dist - (unsigned)BASE_DIST[code], extra);
    }
  }
  send_code(s, END_BLOCK, ltree);
}

static void tr_stored_block(dstate *s, const uint8_t *buf, unsigned stored_len, int last) { /* trees.ts:449-464 */
  send_bits(s, (0u << 1) + (unsigned)last, 3);
  bi_windup(s);
  put_short(s, stored_len);
  put_short(s, ~stored_len & 0xffff);
  for (unsigned i = 0; i < stored_len; i++) put_byte(s, buf[i]);
}

static void tr_flush_block(dstate *s, long buf_index, unsigned stored_len, int last) { /* trees.ts:544-590 */
  unsigned long opt_lenb, static_lenb;
  int max_blindex;
  build_tree(s, &s->l_desc);
  build_tree(s, &s->d_desc);
  max_blindex = build_bl_tree(s);
  opt_lenb = (s->opt_len + 3 + 7) >> 3;
  static_lenb = (s->static_len + 3 + 7) >> 3;
  if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
  s->blocks++;
  if ((unsigned long)stored_len + 4 <= opt_lenb) {
    /* The reference always passes the window (deflate.ts:1121); a negative
     * block_start would make it copy from a negative index.  Unreachable for
     * compressible or short blocks; refuse loudly rather than guess. */
    if (buf_index < 0) abort();
    tr_stored_block(s, s->window + buf_index, stored_len, last);
  } else if (static_lenb == opt_lenb) {
    send_bits(s, (1u << 1) + (unsigned)last, 3);
    compress_block(s, STATIC_LTREE, STATIC_DTREE);
  } else {
    send_bits(s, (2u << 1) + (unsigned)last, 3);
    send_all_trees(s, s->l_desc.max_code + 1, s->d_desc.max_code + 1, max_blindex + 1);
    compress_block(s, s->dyn_ltree, s->dyn_dtree);
  }
  init_block(s);
  if (last) bi_windup(s);
}

/* optional symbol trace for tests (zo_trace_symbols) */
static __thread uint32_t *g_trace;
static __thread size_t g_trace_cap, g_trace_n;
void zo_trace_symbols(uint32_t *buf, size_t cap) { g_trace = buf; g_trace_cap = cap; g_trace_n = 0; }
size_t zo_trace_count(void) { return g_trace_n; }
static void trace(uint32_t v) { if (g_trace && g_trace_n < g_trace_cap) g_trace[g_trace_n] = v; g_trace_n++; }

/* symbol tally, deflate/utils.ts:55-81; returns "block full" */
static int tally_lit(dstate *s, unsigned c) {
  trace(c);
  s->sym_dist[s->sym_next] = 0;
  s->sym_lc[s->sym_next++] = (uint8_t)c;
  s->dyn_ltree[c].freq++;
  return s->sym_next == SYM_END;
}
static int tally_dist(dstate *s, unsigned dist, unsigned len) {
  trace(0x80000000u | (len << 16) | dist);
  s->sym_dist[s->sym_next] = (uint16_t)dist;
  s->sym_lc[s->sym_next++] = (uint8_t)len;
  dist--;
  s->dyn_ltree[LENGTH_CODE[len] + LITERALS + 1].freq++;
  s->dyn_dtree[d_code(dist)].freq++;
  return s->sym_next == SYM_END;
}

/* ------------------------------------------------------------ checksums */
uint32_t zo_crc32(uint32_t crc, const uint8_t *buf, size_t len) { /* common/crc32.ts:26-58 */
  static uint32_t T[256];
  static int ready = 0;
  if (!buf) return 0;
  if (!ready) {
    for (uint32_t n = 0; n < 256; n++) {
      uint32_t c = n;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
      T[n] = c;
    }
    ready = 1;
  }
  uint32_t c = ~crc;
  for (size_t i = 0; i < len; i++) c = (c >> 8) ^ T[(c ^ buf[i]) & 0xff];
  return c ^ 0xffffffffu;
}

uint32_t zo_adler32(uint32_t adler, const uint8_t *buf, size_t len) { /* common/adler32.ts:4-25 */
  if (!buf) return 1;
  uint32_t lo = adler & 0xffff, hi = (adler >> 16) & 0xffff;
  size_t pos = 0;
  while (len > 0) {
    size_t n = len > 2000 ? 2000 : len;
    len -= n;
    while (n--) { lo += buf[pos++]; hi += lo; }
    lo %= 65521;
    hi %= 65521;
  }
  return (hi << 16) | lo;
}

/* --------------------------------------------------------- match engine */
#define UPDATE_HASH(h, c) ((((h) << HASH_SHIFT) ^ (c)) & HASH_MASK) /* deflate.ts:109-111 */

static unsigned insert_string(dstate *s, unsigned str) { /* deflate.ts:113-118 */
  s->ins_h = UPDATE_HASH(s->ins_h, s->window[str + (MIN_MATCH - 1)]);
  unsigned head = s->prev[str & W_MASK] = s->head[s->ins_h];
  s->head[s->ins_h] = (uint16_t)str;
  return head;
}

static void slide_hash(dstate *s) { /* deflate.ts:125-141 */
  for (unsigned n = 0; n < HASH_SIZE; n++) { unsigned m = s->head[n]; s->head[n] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0); }
  for (unsigned n = 0; n < W_SIZE; n++) { unsigned m = s->prev[n]; s->prev[n] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0); }
}

static unsigned read_buf(dstate *s, uint8_t *buf, unsigned size) { /* deflate.ts:143-164 */
  unsigned len = s->avail_in > size ? size : (unsigned)s->avail_in;
  if (len == 0) return 0;
  s->avail_in -= len;
  memcpy(buf, s->next_in, len);
  if (s->wrap == 1) s->adler = zo_adler32(s->adler, buf, len);
  else if (s->wrap == 2) s->adler = zo_crc32(s->adler, buf, len);
  s->next_in += len;
  s->total_in += len;
  return len;
}

static void fill_window(dstate *s) { /* deflate.ts:166-236 */
  const unsigned window_size = 2 * W_SIZE;
  long more;
  do {
    more = (long)window_size - (long)s->lookahead - (long)s->strstart;
    if (more == 0 && s->strstart == 0 && s->lookahead == 0) more = W_SIZE;
    else if (more == -1) more--;
    if (s->strstart >= W_SIZE + MAX_DIST) {
      memmove(s->window, s->window + W_SIZE, (size_t)(W_SIZE - more));
      s->match_start -= W_SIZE;
      s->strstart -= W_SIZE;
      s->block_start -= W_SIZE;
      if (s->insert > s->strstart) s->insert = s->strstart;
      slide_hash(s);
      more += W_SIZE;
    }
    if (s->avail_in == 0) break;
    unsigned n = read_buf(s, s->window + s->strstart + s->lookahead, (unsigned)more);
    s->lookahead += n;
    if (s->lookahead + s->insert >= MIN_MATCH) {
      unsigned str = s->strstart - s->insert;
      s->ins_h = s->window[str];
      s->ins_h = UPDATE_HASH(s->ins_h, s->window[str + 1]);
      while (s->insert) {
        s->ins_h = UPDATE_HASH(s->ins_h, s->window[str + MIN_MATCH - 1]);
        s->prev[str & W_MASK] = s->head[s->ins_h];
        s->head[s->ins_h] = (uint16_t)str;
        str++;
        s->insert--;
        if (s->lookahead + s->insert < MIN_MATCH) break;
      }
    }
  } while (s->lookahead < MIN_LOOKAHEAD && s->avail_in != 0);
  if (s->w_have < window_size) {
    unsigned long curr = s->strstart + s->lookahead, init;
    if (s->w_have < curr) {
      init = window_size - curr;
      if (init > WIN_INIT) init = WIN_INIT;
      memset(s->window + curr, 0, init);
      s->w_have = curr + init;
    } else if (s->w_have < curr + WIN_INIT) {
      init = curr + WIN_INIT - s->w_have;
      if (init > window_size - s->w_have) init = window_size - s->w_have;
      memset(s->window + s->w_have, 0, init);
      s->w_have += init;
    }
  }
}

/* longest_match as the reference states it, with the loop-invariant
 * maxCompare = min(MAX_MATCH, lookahead), deflate.ts:1053-1115 */
static unsigned longest_match(dstate *s, unsigned cur_match) {
  unsigned chain_length = s->max_chain;
  const unsigned scan = s->strstart;
  unsigned best_len = s->prev_length;
  unsigned nice_match = s->nice_match;
  const unsigned limit = s->strstart > MAX_DIST ? s->strstart - MAX_DIST : 0;
  const uint8_t *win = s->window;
  const unsigned lookahead = s->lookahead;
  const unsigned max_compare = MAX_MATCH < lookahead ? MAX_MATCH : lookahead;
  uint8_t scan_end1 = win[scan + best_len - 1];
  uint8_t scan_end = win[scan + best_len];
  if (best_len >= s->good_match) chain_length >>= 2;
  if (nice_match > lookahead) nice_match = lookahead;
  do {
    const unsigned m = cur_match;
    if (win[m + best_len] != scan_end || win[m + best_len - 1] != scan_end1 || win[m] != win[scan] ||
        win[m + 1] != win[scan + 1])
      continue;
    unsigned k = 2;
    while (k < max_compare && win[scan + k] == win[m + k]) k++;
    if (k > best_len) {
      s->match_start = cur_match;
      best_len = k;
      if (k >= nice_match) break;
      scan_end1 = win[scan + best_len - 1];
      scan_end = win[scan + best_len];
    }
  } while ((cur_match = s->prev[cur_match & W_MASK]) > limit && --chain_length != 0);
  return best_len <= lookahead ? best_len : lookahead;
}

static void flush_block_only(dstate *s, int last) { /* deflate.ts:1120-1124 */
  tr_flush_block(s, s->block_start, (unsigned)((long)s->strstart - s->block_start), last);
  s->block_start = s->strstart;
}

static int deflate_fast(dstate *s, int finish) { /* deflate.ts:1281-1350 */
  unsigned hash_head;
  int bflush;
  for (;;) {
    if (s->lookahead < MIN_LOOKAHEAD) {
      fill_window(s);
      if (s->lookahead < MIN_LOOKAHEAD && !finish) return NEED_MORE;
      if (s->lookahead == 0) break;
    }
    hash_head = 0;
    if (s->lookahead >= MIN_MATCH) hash_head = insert_string(s, s->strstart);
    if (hash_head != 0 && s->strstart - hash_head <= MAX_DIST) s->match_length = longest_match(s, hash_head);
    if (s->match_length >= MIN_MATCH) {
      bflush = tally_dist(s, s->strstart - s->match_start, s->match_length - MIN_MATCH);
      s->lookahead -= s->match_length;
      if (s->match_length <= s->max_lazy && s->lookahead >= MIN_MATCH) {
        s->match_length--;
        do { s->strstart++; insert_string(s, s->strstart); } while (--s->match_length != 0);
        s->strstart++;
      } else {
        s->strstart += s->match_length;
        s->match_length = 0;
        s->ins_h = s->window[s->strstart];
        s->ins_h = UPDATE_HASH(s->ins_h, s->window[s->strstart + 1]);
      }
    } else {
      bflush = tally_lit(s, s->window[s->strstart]);
      s->lookahead--;
      s->strstart++;
    }
    if (bflush) flush_block_only(s, 0);
  }
  s->insert = s->strstart < MIN_MATCH - 1 ? s->strstart : MIN_MATCH - 1;
  flush_block_only(s, 1); /* finish is the only way out of the loop */
  return FINISH_DONE;
}

static int deflate_slow(dstate *s, int finish) { /* deflate.ts:1352-1448 */
  unsigned hash_head;
  int bflush;
  for (;;) {
    if (s->lookahead < MIN_LOOKAHEAD) {
      fill_window(s);
      if (s->lookahead < MIN_LOOKAHEAD && !finish) return NEED_MORE;
      if (s->lookahead == 0) break;
    }
    hash_head = 0;
    if (s->lookahead >= MIN_MATCH) hash_head = insert_string(s, s->strstart);
    s->prev_length = s->match_length;
    s->prev_match = s->match_start;
    s->match_length = MIN_MATCH - 1;
    if (hash_head != 0 && s->prev_length < s->max_lazy && s->strstart - hash_head <= MAX_DIST) {
      s->match_length = longest_match(s, hash_head);
      if (s->match_length <= 5 && s->match_length == MIN_MATCH && s->strstart - s->match_start > TOO_FAR)
        s->match_length = MIN_MATCH - 1;
    }
    if (s->prev_length >= MIN_MATCH && s->match_length <= s->prev_length) {
      unsigned max_insert = s->strstart + s->lookahead - MIN_MATCH;
      bflush = tally_dist(s, s->strstart - 1 - s->prev_match, s->prev_length - MIN_MATCH);
      s->lookahead -= s->prev_length - 1;
      s->prev_length -= 2;
      do {
        if (++s->strstart <= max_insert) insert_string(s, s->strstart);
      } while (--s->prev_length != 0);
      s->match_available = 0;
      s->match_length = MIN_MATCH - 1;
      s->strstart++;
      if (bflush) flush_block_only(s, 0);
    } else if (s->match_available) {
      bflush = tally_lit(s, s->window[s->strstart - 1]);
      if (bflush) flush_block_only(s, 0);
      s->strstart++;
      s->lookahead--;
    } else {
      s->match_available = 1;
      s->strstart++;
      s->lookahead--;
    }
  }
  if (s->match_available) { tally_lit(s, s->window[s->strstart - 1]); s->match_available = 0; }
  s->insert = s->strstart < MIN_MATCH - 1 ? s->strstart : MIN_MATCH - 1;
  flush_block_only(s, 1);
  return FINISH_DONE;
}

/* deflate() restricted to the calls streams.ts makes (Z_NO_FLUSH, Z_FINISH)
 * with an output buffer that never fills, deflate.ts:716-989. */
static void deflate_call(dstate *s, int finish) {
  if (s->status == ST_INIT && s->wrap == 0) s->status = ST_BUSY;
  if (s->status == ST_INIT) { /* zlib header, deflate.ts:753-786 */
    unsigned header = (8u + ((W_BITS - 8u) << 4)) << 8, level_flags;
    if (s->level < 2) level_flags = 0;
    else if (s->level < 6) level_flags = 1;
    else if (s->level == 6) level_flags = 2;
    else level_flags = 3;
    header |= level_flags << 6;
    header += 31 - (header % 31);
    put_short_msb(s, header);
    s->adler = 1;
    s->status = ST_BUSY;
  }
  if (s->status == ST_GZIP) { /* gzip header without gzhead, deflate.ts:787-806 */
    s->adler = 0;
    put_byte(s, 31); put_byte(s, 139); put_byte(s, 8);
    for (int i = 0; i < 5; i++) put_byte(s, 0);
    put_byte(s, s->level == 9 ? 2 : (s->level < 2 ? 4 : 0));
    put_byte(s, OS_CODE);
    s->status = ST_BUSY;
  }
  if (s->avail_in != 0 || s->lookahead != 0 || (finish && s->status != ST_FINISH)) {
    int bstate = CONFIG[s->level].slow ? deflate_slow(s, finish) : deflate_fast(s, finish);
    if (bstate == FINISH_DONE) s->status = ST_FINISH;
  }
  if (!finish || s->wrap <= 0) return;
  if (s->wrap == 2) { /* deflate.ts:971-979 */
    for (int i = 0; i < 4; i++) put_byte(s, (s->adler >> (8 * i)) & 0xff);
    for (int i = 0; i < 4; i++) put_byte(s, (unsigned)((s->total_in >> (8 * i)) & 0xff));
  } else {
    put_short_msb(s, (s->adler >> 16) & 0xffff);
    put_short_msb(s, s->adler & 0xffff);
  }
  s->wrap = -s->wrap;
}

size_t zo_deflate_bound(size_t n, int wbits) { /* deflate.ts:615-674, memLevel 8 / wbits 15 branch */
  size_t wraplen = wbits < 0 ? 0 : (wbits > 15 ? 18 : 6);
  return n + (n >> 12) + (n >> 14) + (n >> 25) + 13 - 6 + wraplen;
}

int zo_compress(const uint8_t *in, size_t n, int level, int wbits, uint8_t *out, size_t cap, size_t *out_len,
                int *phase) {
  *out_len = 0;
  *phase = ZO_PHASE_NONE;
  if (level == -1) level = 6; /* Z_DEFAULT_COMPRESSION, deflate.ts:268-270 */
  int wrap = 1;
  if (wbits < 0) { wrap = 0; if (wbits < -15) { *phase = ZO_PHASE_INIT; return ZO_STREAM_ERROR; } wbits = -wbits; }
  else if (wbits > 15) { wrap = 2; wbits -= 16; }
  if (wbits < 8 || wbits > 15 || level < 0 || level > 9 || (wbits == 8 && wrap != 1)) {
    *phase = ZO_PHASE_INIT; /* deflate.ts:281-294 */
    return ZO_STREAM_ERROR;
  }
  if (wbits != 15 || level == 0) { *phase = ZO_PHASE_INIT; return ZO_STREAM_ERROR; } /* not restated */
  init_tables();
  dstate *s = (dstate *)calloc(1, sizeof(dstate));
  if (!s) return ZO_MEM_ERROR;
  s->out = out;
  s->cap = cap;
  s->wrap = wrap;
  s->level = level;
  s->status = wrap == 2 ? ST_GZIP : ST_INIT;
  s->adler = wrap == 2 ? 0 : 1; /* deflate.ts:462 */
  tr_init(s);
  /* lm_init, deflate.ts:470-487 */
  s->max_lazy = (unsigned)CONFIG[level].lazy;
  s->good_match = (unsigned)CONFIG[level].good;
  s->nice_match = (unsigned)CONFIG[level].nice;
  s->max_chain = (unsigned)CONFIG[level].chain;
  s->match_length = s->prev_length = MIN_MATCH - 1;
  /* transform(): <=32 KiB sub-chunks, deflate(Z_NO_FLUSH) while input remains */
  for (size_t off = 0; off < n; off += IN_CHUNK) {
    size_t len = n - off < IN_CHUNK ? n - off : IN_CHUNK;
    s->next_in = in + off;
    s->avail_in = len;
    while (s->avail_in > 0) deflate_call(s, 0);
  }
  /* flush(): deflate(Z_FINISH) */
  deflate_call(s, 1);
  *out_len = s->out_len;
  g_last_blocks = s->blocks;
  int overflow = s->overflow;
  free(s);
  return overflow ? ZO_BUF_ERROR : ZO_STREAM_END;
}
