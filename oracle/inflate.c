/*
 * oracle/inflate.c -- CPU restatement of the reference's inflate engine.
 *
 * TEST INFRASTRUCTURE ONLY (see zoracle.h).  Never linked into the product.
 *
 * Restates /root/reference/src/mod/inflate/{inflate,inffast,inftrees,
 * constants,utils}.ts including the deflate64 mode (windowBits -16), driven
 * exactly as streams.ts drives it for one write()+close(): 32 KiB input
 * sub-chunks with Z_NO_FLUSH, each call given a fresh 64 KiB output buffer
 * (streams.ts:6-7,78-93), then Z_FINISH calls (streams.ts:132-166).
 * Modelling the buffer sizes matters for the sliding window, for when
 * inflate_fast is entered, and for which stream-layer call reports an error.
 */
#include <stdlib.h>
#include <string.h>
#include "zoracle.h"

#define OUT_BUF (64 * 1024) /* streams.ts:6 */
#define IN_CHUNK (32 * 1024) /* streams.ts:7 */
#define MAXBITS 15
#define ENOUGH_LENS 852 /* inflate/constants.ts:4-6 */
#define ENOUGH_DISTS 592
#define ENOUGH_DISTS_9 594

/* packed table entry: op << 24 | bits << 16 | val (inflate/utils.ts:51-72) */
typedef uint32_t code_t;
#define C_OP(c) ((c) >> 24)
#define C_BITS(c) (((c) >> 16) & 0xff)
#define C_VAL(c) ((c) & 0xffff)
/* When set, reproduce the reference's inflate_fast window-wrap defect
 * (inffast.ts:139-147) under the synchronous stream model in which every
 * inflate() call gets the same recycled 64 KiB output buffer. */
static __thread int g_ref_bugs = 1;
void zo_set_reference_bugs(int on) { g_ref_bugs = on; }

static code_t pack(unsigned op, unsigned bits, unsigned val) { return (op << 24) | (bits << 16) | val; }

/* InflateMode, common/types.ts:165-198 */
enum { HEAD = 0, FLAGS, TIME, OS, EXLEN, EXTRA, NAME, COMMENT, HCRC, DICTID, DICT, TYPE, TYPEDO, STORED, COPY_, COPY,
       TABLE, LENLENS, CODELENS, LEN_, LEN, LENEXT, DIST, DISTEXT, MATCH, LIT, CHECK, LENGTH, DONE, BAD, MEM, SYNC };
enum { CODES = 0, LENS, DISTS };

static const uint8_t BL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

/* length/distance base and op tables, inflate/constants.ts:8-45.
 * ops: deflate mode = 16 + extra (flag 16), deflate64 = 128 + extra. */
static uint16_t LBASE[31], LEXT[31], DBASE[32], DEXT[32];
static uint16_t LBASE9[31], LEXT9[31], DBASE9[32], DEXT9[32];
static int tables_ready = 0;

static void init_tables(void) {
  if (tables_ready) return;
  static const int lbits[28] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5};
  static const int dbits[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  int base = 3;
  for (int i = 0; i < 28; i++) {
    LBASE[i] = LBASE9[i] = (uint16_t)base;
    LEXT[i] = (uint16_t)(16 + lbits[i]);
    LEXT9[i] = (uint16_t)(128 + lbits[i]);
    base += 1 << lbits[i];
  }
  LBASE[28] = 258; LEXT[28] = 16;            /* code 285: 258, no extra */
  LBASE9[28] = 3; LEXT9[28] = 128 + 16;      /* deflate64: 3 + 16 extra bits */
  LBASE[29] = LBASE[30] = LBASE9[29] = LBASE9[30] = 0;
  LEXT[29] = 73; LEXT[30] = 200;             /* invalid markers */
  LEXT9[29] = 72; LEXT9[30] = 78;
  base = 1;
  for (int i = 0; i < 30; i++) {
    DBASE[i] = DBASE9[i] = (uint16_t)base;
    DEXT[i] = (uint16_t)(16 + dbits[i]);
    DEXT9[i] = (uint16_t)(128 + dbits[i]);
    base += 1 << dbits[i];
  }
  DBASE[30] = DBASE[31] = 0; DEXT[30] = DEXT[31] = 64;
  DBASE9[30] = 32769; DBASE9[31] = 49153; DEXT9[30] = DEXT9[31] = 128 + 14;
  tables_ready = 1;
}

/* inflate_table with the two parameter sets, inftrees.ts:34-279 */
static int inflate_table(int type, const uint16_t *lens, unsigned codes, code_t *table, unsigned *bits_io,
                         uint16_t *work, int d64, unsigned *used_out) {
  unsigned len, sym, min, max, root, curr, drop, used, huff, incr, fill, low, mask;
  int left;
  code_t here;
  unsigned next = 0; /* index into table */
  const uint16_t *base = NULL, *extra = NULL;
  int match;
  uint16_t count[MAXBITS + 1], offs[MAXBITS + 1];
  const unsigned enough_d = d64 ? ENOUGH_DISTS_9 : ENOUGH_DISTS;

  for (len = 0; len <= MAXBITS; len++) count[len] = 0;
  for (sym = 0; sym < codes; sym++) count[lens[sym]]++;
  root = *bits_io;
  for (max = MAXBITS; max >= 1; max--) if (count[max] != 0) break;
  if (root > max) root = max;
  if (max == 0) {
    if (!d64) { /* _createTableWhenNoCodes */
      here = pack(64, 1, 0);
      table[0] = here;
      table[1] = here;
      *bits_io = 1;
      *used_out = 0; /* the reference does not advance the index here */
      return 0;
    }
    return -1;
  }
  for (min = 1; min < max; min++) if (count[min] != 0) break;
  if (root < min) root = min;
  left = 1;
  for (len = 1; len <= MAXBITS; len++) {
    left <<= 1;
    left -= count[len];
    if (left < 0) return -1;
  }
  if (left > 0 && (type == CODES || max != 1)) return -1;
  offs[1] = 0;
  for (len = 1; len < MAXBITS; len++) offs[len + 1] = (uint16_t)(offs[len] + count[len]);
  for (sym = 0; sym < codes; sym++) if (lens[sym] != 0) work[offs[lens[sym]]++] = (uint16_t)sym;
  switch (type) {
    case CODES: base = extra = work; match = d64 ? 19 : 20; break;
    case LENS: base = d64 ? LBASE9 : LBASE; extra = d64 ? LEXT9 : LEXT; match = d64 ? 256 : 257; break;
    default: base = d64 ? DBASE9 : DBASE; extra = d64 ? DEXT9 : DEXT; match = d64 ? -1 : 0;
  }
  huff = 0;
  sym = 0;
  len = min;
  curr = root;
  drop = 0;
  low = (unsigned)-1;
  used = 1u << root;
  mask = used - 1;
#define OVER(u) ((type == LENS && (d64 ? (u) >= ENOUGH_LENS : (u) > ENOUGH_LENS)) || \
                 (type == DISTS && (d64 ? (u) >= enough_d : (u) > enough_d)))
  if (OVER(used)) return 1;
  for (;;) {
    /* createTableEntry, inftrees.ts:281-307 */
    int w = work[sym];
    if (d64 ? w < match : w + 1 < match) here = pack(0, len - drop, (unsigned)w);
    else if (d64 ? w > match : w >= match) {
      int idx = (d64 && type == LENS) ? w - 257 : (d64 ? w : w - match);
      here = pack(extra[idx], len - drop, base[idx]);
    } else here = pack(32 + 64, len - drop, 0);
    incr = 1u << (len - drop);
    fill = 1u << curr;
    min = fill;
    do { fill -= incr; table[next + (huff >> drop) + fill] = here; } while (fill != 0);
    incr = 1u << (len - 1);
    while (huff & incr) incr >>= 1;
    if (incr != 0) { huff &= incr - 1; huff += incr; } else huff = 0;
    sym++;
    if (--count[len] == 0) {
      if (len == max) break;
      len = lens[work[sym]];
    }
    if (len > root && (huff & mask) != low) {
      if (drop == 0) drop = root;
      next += 1u << curr;
      curr = len - drop;
      left = 1 << curr;
      while (curr + drop < max) {
        left -= count[curr + drop];
        if (left <= 0) break;
        curr++;
        left <<= 1;
      }
      used += 1u << curr;
      if (OVER(used)) return 1;
      low = huff & mask;
      table[low] = pack(curr, root, next);
    }
  }
  if (huff != 0) {
    here = pack(64, len - drop, 0);
    while (huff != 0) {
      if (drop != 0 && (huff & mask) != low) {
        drop = 0;
        len = root;
        next = 0;
        curr = root;
        here = pack(64, len, 0);
      }
      table[next + (huff >> drop)] = here;
      incr = 1u << (len - 1);
      while (huff & incr) incr >>= 1;
      if (incr != 0) { huff &= incr - 1; huff += incr; } else huff = 0;
    }
  }
#undef OVER
  *used_out = used;
  *bits_io = root;
  return 0;
}

typedef struct {
  /* z_stream view */
  const uint8_t *next_in;
  unsigned avail_in;
  size_t total_in, total_out;
  uint8_t *next_out;
  unsigned avail_out;
  const char *msg;
  /* InflateState, inflate/utils.ts:11-49 */
  int mode, last, wrap, havedict, flags, d64, sane, back;
  uint32_t check, total;
  unsigned w_bits, w_size, w_have, w_next;
  uint8_t *window;
  uint32_t hold;
  unsigned bits, length, offset, extra, was;
  const code_t *lencode, *distcode;
  unsigned lenbits, distbits, ncode, nlen, ndist, have;
  uint16_t lens[320], work[288];
  code_t codes[ENOUGH_LENS + ENOUGH_DISTS_9];
  code_t fixed[544];
} istate;

static void fixedtables(istate *st) { /* inflate.ts:218-280 (cached per mode there; rebuilt here) */
  unsigned sym, bits, used;
  for (sym = 0; sym < 144; sym++) st->lens[sym] = 8;
  for (; sym < 256; sym++) st->lens[sym] = 9;
  for (; sym < 280; sym++) st->lens[sym] = 7;
  for (; sym < 288; sym++) st->lens[sym] = 8;
  memset(st->fixed, 0, sizeof st->fixed);
  bits = 9;
  inflate_table(LENS, st->lens, 288, st->fixed, &bits, st->work, st->d64, &used);
  unsigned dist_at = used;
  for (sym = 0; sym < 32; sym++) st->lens[sym] = 5;
  bits = 5;
  inflate_table(DISTS, st->lens, 32, st->fixed + dist_at, &bits, st->work, st->d64, &used);
  st->lencode = st->fixed;
  st->lenbits = 9;
  st->distcode = st->fixed + dist_at;
  st->distbits = 5;
}

static int updatewindow(istate *st, const uint8_t *end, unsigned copy) { /* inflate.ts:282-324 */
  if (!st->window) {
    st->window = (uint8_t *)calloc(1u << st->w_bits, 1);
    if (!st->window) return 1;
  }
  if (st->w_size == 0) { st->w_size = 1u << st->w_bits; st->w_next = 0; st->w_have = 0; }
  if (copy >= st->w_size) {
    memcpy(st->window, end - st->w_size, st->w_size);
    st->w_next = 0;
    st->w_have = st->w_size;
  } else {
    unsigned dist = st->w_size - st->w_next;
    if (dist > copy) dist = copy;
    memcpy(st->window + st->w_next, end - copy, dist);
    copy -= dist;
    if (copy) {
      memcpy(st->window, end - copy, copy);
      st->w_next = copy;
      st->w_have = st->w_size;
    } else {
      st->w_next += dist;
      if (st->w_next == st->w_size) st->w_next = 0;
      if (st->w_have < st->w_size) st->w_have += dist;
    }
  }
  return 0;
}

/* inflate_fast, inffast.ts:5-228.  Entered only when have >= 6, left >= 258. */
static void inflate_fast(istate *st, unsigned start) {
  const uint8_t *in = st->next_in;
  const uint8_t *last = in + (st->avail_in - 5);
  uint8_t *out = st->next_out;
  uint8_t *beg = out - (start - st->avail_out);
  uint8_t *end = out + (st->avail_out - 257);
  const unsigned wsize = st->w_size, whave = st->w_have, wnext = st->w_next;
  const uint8_t *window = st->window;
  uint32_t hold = st->hold;
  unsigned bits = st->bits;
  const code_t *lcode = st->lencode, *dcode = st->distcode;
  const unsigned lmask = (1u << st->lenbits) - 1, dmask = (1u << st->distbits) - 1;
  code_t here;
  unsigned op, len, dist;
  const uint8_t *from;
  do {
    if (bits < 15) { hold += (uint32_t)(*in++) << bits; bits += 8; hold += (uint32_t)(*in++) << bits; bits += 8; }
    here = lcode[hold & lmask];
  dolen:
    op = C_BITS(here); hold >>= op; bits -= op;
    op = C_OP(here);
    if (op == 0) {
      *out++ = (uint8_t)C_VAL(here);
    } else if (op & 16) {
      len = C_VAL(here);
      op &= 15;
      if (op) {
        if (bits < op) { hold += (uint32_t)(*in++) << bits; bits += 8; }
        len += hold & ((1u << op) - 1);
        hold >>= op; bits -= op;
      }
      if (bits < 15) { hold += (uint32_t)(*in++) << bits; bits += 8; hold += (uint32_t)(*in++) << bits; bits += 8; }
      here = dcode[hold & dmask];
    dodist:
      op = C_BITS(here); hold >>= op; bits -= op;
      op = C_OP(here);
      if (op & 16) {
        dist = C_VAL(here);
        op &= 15;
        if (bits < op) {
          hold += (uint32_t)(*in++) << bits; bits += 8;
          if (bits < op) { hold += (uint32_t)(*in++) << bits; bits += 8; }
        }
        dist += hold & ((1u << op) - 1);
        hold >>= op; bits -= op;
        op = (unsigned)(out - beg);
        if (dist > op) { /* copy from window */
          op = dist - op;
          if (op > whave && st->sane) { st->msg = "invalid distance too far back"; st->mode = BAD; break; }
          from = window;
          if (wnext == 0) {
            from += wsize - op;
            if (op < len) { len -= op; do *out++ = *from++; while (--op); from = out - dist; }
          } else if (wnext < op) {
            from += wsize + wnext - op;
            op -= wnext;
            if (op < len) {
              len -= op;
              do *out++ = *from++; while (--op);
              from = window;
              if (wnext < len) { op = wnext; len -= op; do *out++ = *from++; while (--op); from = out - dist; }
              else if (g_ref_bugs) from = beg; /* inffast.ts:139-147: the reference keeps reading `output` from index 0 */
            }
          } else {
            from += wnext - op;
            if (op < len) { len -= op; do *out++ = *from++; while (--op); from = out - dist; }
          }
          while (len > 0) { *out++ = *from++; len--; }
        } else {
          from = out - dist;
          while (len > 0) { *out++ = *from++; len--; }
        }
      } else if ((op & 64) == 0) {
        here = dcode[C_VAL(here) + (hold & ((1u << op) - 1))];
        goto dodist;
      } else {
        st->msg = "invalid distance code"; st->mode = BAD; break;
      }
    } else if ((op & 64) == 0) {
      here = lcode[C_VAL(here) + (hold & ((1u << op) - 1))];
      goto dolen;
    } else if (op & 32) {
      st->mode = TYPE; break;
    } else {
      st->msg = "invalid literal/length code"; st->mode = BAD; break;
    }
  } while (in < last && out < end);
  len = bits >> 3;
  in -= len;
  bits -= len << 3;
  hold &= (1u << bits) - 1;
  st->avail_in = (unsigned)(in < last ? 5 + (last - in) : 5 - (in - last));
  st->avail_out = (unsigned)(out < end ? 257 + (end - out) : 257 - (out - end));
  st->next_in = in;
  st->next_out = out;
  st->hold = hold;
  st->bits = bits;
}

static int inflate_reset2(istate *st, int wbits) { /* inflate.ts:138-172 */
  int wrap;
  if (wbits < 0) {
    if (wbits < -16) return ZO_STREAM_ERROR;
    wrap = 0;
    st->d64 = wbits == -16;
    wbits = -wbits;
  } else {
    wrap = (wbits >> 4) + 5;
    st->d64 = 0;
    if (wbits < 48) wbits &= 15;
  }
  if (wbits && (wbits < 8 || wbits > (st->d64 ? 16 : 15))) return ZO_STREAM_ERROR;
  st->wrap = wrap;
  st->w_bits = (unsigned)wbits;
  st->w_size = st->w_have = st->w_next = 0;
  st->total = 0;
  st->msg = "";
  if (st->wrap) st->check = (uint32_t)(st->wrap & 1); /* strm._adler */
  st->mode = st->d64 ? TYPE : HEAD;
  st->last = 0;
  st->havedict = 0;
  st->flags = -1;
  st->hold = 0;
  st->bits = 0;
  st->lencode = st->distcode = st->codes;
  st->sane = 1;
  st->back = -1;
  return ZO_OK;
}

/* one inflate() call, inflate.ts:332-1185 */
static int inflate_call(istate *st, int finish) {
  const uint8_t *next;
  uint8_t *put;
  unsigned have, left, in, out, copy, len;
  uint32_t hold;
  unsigned bits;
  code_t here, last;
  int ret = ZO_OK;
  const uint8_t *out_start = st->next_out;
  if (st->mode == TYPE) st->mode = TYPEDO;
#define LOAD() do { put = st->next_out; left = st->avail_out; next = st->next_in; have = st->avail_in; hold = st->hold; bits = st->bits; } while (0)
#define RESTORE() do { st->next_out = put; st->avail_out = left; st->next_in = next; st->avail_in = have; st->hold = hold; st->bits = bits; } while (0)
#define INITBITS() do { hold = 0; bits = 0; } while (0)
#define PULLBYTE() do { if (have == 0) goto inf_leave; have--; hold += (uint32_t)(*next++) << bits; bits += 8; } while (0)
#define NEEDBITS(n) do { while (bits < (unsigned)(n)) PULLBYTE(); } while (0)
#define BITS(n) ((unsigned)hold & ((1u << (n)) - 1))
#define DROPBITS(n) do { hold >>= (n); bits -= (unsigned)(n); } while (0)
#define BYTEBITS() do { hold >>= bits & 7; bits -= bits & 7; } while (0)
  LOAD();
  in = have;
  out = left;
  for (;;) {
    switch (st->mode) {
      case HEAD:
        if (st->wrap == 0) { st->mode = TYPEDO; break; }
        NEEDBITS(16);
        if ((st->wrap & 2) && hold == 0x8b1f) {
          if (st->w_bits == 0) st->w_bits = 15;
          uint8_t hb[2] = {(uint8_t)(hold & 0xff), (uint8_t)((hold >> 8) & 0xff)};
          st->check = zo_crc32(zo_crc32(0, NULL, 0), hb, 2);
          INITBITS();
          st->mode = FLAGS;
          break;
        }
        if (!(st->wrap & 1) || ((BITS(8) << 8) + (hold >> 8)) % 31) { st->msg = "incorrect header check"; st->mode = BAD; break; }
        if (BITS(4) != 8) { st->msg = "unknown compression method"; st->mode = BAD; break; }
        DROPBITS(4);
        len = BITS(4) + 8;
        if (st->w_bits == 0) st->w_bits = len;
        if (len > 15 || len > st->w_bits) { st->msg = "invalid window size"; st->mode = BAD; break; }
        st->flags = 0;
        st->check = zo_adler32(0, NULL, 0);
        st->mode = (hold & 0x200) ? DICTID : TYPE;
        INITBITS();
        break;
      case FLAGS:
        NEEDBITS(16);
        st->flags = (int)hold;
        if ((st->flags & 0xff) != 8) { st->msg = "unknown compression method"; st->mode = BAD; break; }
        if (st->flags & 0xe000) { st->msg = "unknown header flags set"; st->mode = BAD; break; }
        if ((st->flags & 0x0200) && (st->wrap & 4)) {
          uint8_t hb[2] = {(uint8_t)(hold & 0xff), (uint8_t)((hold >> 8) & 0xff)};
          st->check = zo_crc32(st->check, hb, 2);
        }
        INITBITS();
        st->mode = TIME;
        /* fallthrough */
      case TIME:
        NEEDBITS(32);
        if ((st->flags & 0x0200) && (st->wrap & 4)) {
          uint8_t hb[4] = {(uint8_t)hold, (uint8_t)(hold >> 8), (uint8_t)(hold >> 16), (uint8_t)(hold >> 24)};
          st->check = zo_crc32(st->check, hb, 4);
        }
        INITBITS();
        st->mode = OS;
        /* fallthrough */
      case OS:
        NEEDBITS(16);
        if ((st->flags & 0x0200) && (st->wrap & 4)) {
          uint8_t hb[2] = {(uint8_t)(hold & 0xff), (uint8_t)((hold >> 8) & 0xff)};
          st->check = zo_crc32(st->check, hb, 2);
        }
        INITBITS();
        st->mode = EXLEN;
        /* fallthrough */
      case EXLEN:
        if (st->flags & 0x0400) {
          NEEDBITS(16);
          st->length = hold;
          if ((st->flags & 0x0200) && (st->wrap & 4)) {
            uint8_t hb[2] = {(uint8_t)(hold & 0xff), (uint8_t)((hold >> 8) & 0xff)};
            st->check = zo_crc32(st->check, hb, 2);
          }
          INITBITS();
        }
        st->mode = EXTRA;
        /* fallthrough */
      case EXTRA:
        if (st->flags & 0x0400) {
          copy = st->length;
          if (copy > have) copy = have;
          if (copy) {
            if ((st->flags & 0x0200) && (st->wrap & 4)) st->check = zo_crc32(st->check, next, copy);
            have -= copy;
            next += copy;
            st->length -= copy;
          }
          if (st->length) goto inf_leave;
        }
        st->length = 0;
        st->mode = NAME;
        /* fallthrough */
      case NAME:
        if (st->flags & 0x0800) {
          if (have == 0) goto inf_leave;
          copy = 0;
          do len = next[copy++]; while (len && copy < have);
          if ((st->flags & 0x0200) && (st->wrap & 4)) st->check = zo_crc32(st->check, next, copy);
          have -= copy;
          next += copy;
          if (len) goto inf_leave;
        }
        st->length = 0;
        st->mode = COMMENT;
        /* fallthrough */
      case COMMENT:
        if (st->flags & 0x1000) {
          if (have == 0) goto inf_leave;
          copy = 0;
          do len = next[copy++]; while (len && copy < have);
          if ((st->flags & 0x0200) && (st->wrap & 4)) st->check = zo_crc32(st->check, next, copy);
          have -= copy;
          next += copy;
          if (len) goto inf_leave;
        }
        st->mode = HCRC;
        /* fallthrough */
      case HCRC:
        if (st->flags & 0x0200) {
          NEEDBITS(16);
          if ((st->wrap & 4) && hold != (st->check & 0xffff)) { st->msg = "header crc mismatch"; st->mode = BAD; break; }
          INITBITS();
        }
        st->check = zo_crc32(0, NULL, 0);
        st->mode = TYPE;
        break;
      case DICTID:
        NEEDBITS(32);
        st->check = ((hold & 0xff) << 24) | (((hold >> 8) & 0xff) << 16) | (((hold >> 16) & 0xff) << 8) | ((hold >> 24) & 0xff);
        INITBITS();
        st->mode = DICT;
        /* fallthrough */
      case DICT:
        if (!st->havedict) { RESTORE(); return ZO_NEED_DICT; }
        st->check = 1;
        st->mode = TYPE;
        /* fallthrough */
      case TYPE:
        /* Z_BLOCK / Z_TREES are never passed by the stream layer */
        /* fallthrough */
      case TYPEDO:
        if (st->last) { BYTEBITS(); st->mode = CHECK; break; }
        NEEDBITS(3);
        st->last = (int)BITS(1);
        DROPBITS(1);
        switch (BITS(2)) {
          case 0: st->mode = STORED; break;
          case 1: fixedtables(st); st->mode = LEN_; break;
          case 2: st->mode = TABLE; break;
          case 3: st->msg = "invalid block type"; st->mode = BAD;
        }
        DROPBITS(2);
        break;
      case STORED:
        BYTEBITS();
        NEEDBITS(32);
        if ((hold & 0xffff) != ((hold >> 16) ^ 0xffff)) { st->msg = "invalid stored block lengths"; st->mode = BAD; break; }
        st->length = hold & 0xffff;
        INITBITS();
        st->mode = COPY_;
        /* fallthrough */
      case COPY_:
        st->mode = COPY;
        /* fallthrough */
      case COPY:
        copy = st->length;
        if (copy) {
          if (copy > have) copy = have;
          if (copy > left) copy = left;
          if (copy == 0) goto inf_leave;
          memcpy(put, next, copy);
          have -= copy;
          next += copy;
          left -= copy;
          put += copy;
          st->length -= copy;
          break;
        }
        st->mode = TYPE;
        break;
      case TABLE:
        NEEDBITS(14);
        st->nlen = BITS(5) + 257;
        DROPBITS(5);
        st->ndist = BITS(5) + 1;
        DROPBITS(5);
        st->ncode = BITS(4) + 4;
        DROPBITS(4);
        if (st->nlen > 286 || (!st->d64 && st->ndist > 30)) {
          st->msg = st->d64 ? "too many length" : "too many length or distance symbols";
          st->mode = BAD;
          break;
        }
        st->have = 0;
        st->mode = LENLENS;
        /* fallthrough */
      case LENLENS: {
        while (st->have < st->ncode) { NEEDBITS(3); st->lens[BL_ORDER[st->have++]] = (uint16_t)BITS(3); DROPBITS(3); }
        while (st->have < 19) st->lens[BL_ORDER[st->have++]] = 0;
        st->lencode = st->distcode = st->codes;
        st->lenbits = 7;
        unsigned used;
        int r = inflate_table(CODES, st->lens, 19, st->codes, &st->lenbits, st->work, st->d64, &used);
        if (r) { st->msg = "invalid code lengths set"; st->mode = BAD; break; }
        st->have = 0;
        st->mode = CODELENS;
      }
        /* fallthrough */
      case CODELENS: {
        while (st->have < st->nlen + st->ndist) {
          for (;;) {
            here = st->lencode[BITS(st->lenbits)];
            if (C_BITS(here) <= bits) break;
            PULLBYTE();
          }
          if (C_VAL(here) < 16) {
            DROPBITS(C_BITS(here));
            st->lens[st->have++] = (uint16_t)C_VAL(here);
          } else {
            if (C_VAL(here) == 16) {
              NEEDBITS(C_BITS(here) + 2);
              DROPBITS(C_BITS(here));
              if (st->have == 0) { st->msg = "invalid bit length repeat"; st->mode = BAD; break; }
              len = st->lens[st->have - 1];
              copy = 3 + BITS(2);
              DROPBITS(2);
            } else if (C_VAL(here) == 17) {
              NEEDBITS(C_BITS(here) + 3);
              DROPBITS(C_BITS(here));
              len = 0;
              copy = 3 + BITS(3);
              DROPBITS(3);
            } else {
              NEEDBITS(C_BITS(here) + 7);
              DROPBITS(C_BITS(here));
              len = 0;
              copy = 11 + BITS(7);
              DROPBITS(7);
            }
            if (st->have + copy > st->nlen + st->ndist) { st->msg = "invalid bit length repeat"; st->mode = BAD; break; }
            while (copy--) st->lens[st->have++] = (uint16_t)len;
          }
        }
        if (st->mode == BAD) break;
        if (st->lens[256] == 0) { st->msg = "invalid code -- missing end-of-block"; st->mode = BAD; break; }
        unsigned lused, dused;
        st->lenbits = 9;
        int r = inflate_table(LENS, st->lens, st->nlen, st->codes, &st->lenbits, st->work, st->d64, &lused);
        st->lencode = st->codes;
        if (r) { st->msg = "invalid literal/lengths set"; st->mode = BAD; break; }
        st->distbits = 6;
        r = inflate_table(DISTS, st->lens + st->nlen, st->ndist, st->codes + lused, &st->distbits, st->work, st->d64, &dused);
        st->distcode = st->codes + lused;
        if (r) { st->msg = "invalid distances set"; st->mode = BAD; break; }
        st->mode = LEN_;
      }
        /* fallthrough */
      case LEN_:
        st->mode = LEN;
        /* fallthrough */
      case LEN:
        if (!st->d64 && have >= 6 && left >= 258) {
          RESTORE();
          inflate_fast(st, out);
          LOAD();
          if (st->mode == TYPE) st->back = -1;
          break;
        }
        st->back = 0;
        for (;;) {
          here = st->lencode[BITS(st->lenbits)];
          if (C_BITS(here) <= bits) break;
          PULLBYTE();
        }
        if (C_OP(here) && (C_OP(here) & 0xf0) == 0) {
          last = here;
          for (;;) {
            here = st->lencode[C_VAL(last) + (BITS(C_BITS(last) + C_OP(last)) >> C_BITS(last))];
            if (C_BITS(last) + C_BITS(here) <= bits) break;
            PULLBYTE();
          }
          DROPBITS(C_BITS(last));
          st->back += (int)C_BITS(last);
        }
        DROPBITS(C_BITS(here));
        st->back += (int)C_BITS(here);
        st->length = C_VAL(here);
        if (C_OP(here) == 0) { st->mode = LIT; break; }
        if (C_OP(here) & 32) { st->back = -1; st->mode = TYPE; break; }
        if (C_OP(here) & 64) { st->msg = "invalid literal/length code"; st->mode = BAD; break; }
        st->extra = C_OP(here) & (st->d64 ? 31u : 15u);
        st->mode = LENEXT;
        /* fallthrough */
      case LENEXT:
        if (st->extra) {
          NEEDBITS(st->extra);
          st->length += BITS(st->extra);
          DROPBITS(st->extra);
          st->back += (int)st->extra;
        }
        st->was = st->length;
        st->mode = DIST;
        /* fallthrough */
      case DIST:
        for (;;) {
          here = st->distcode[BITS(st->distbits)];
          if (C_BITS(here) <= bits) break;
          PULLBYTE();
        }
        if ((C_OP(here) & 0xf0) == 0) {
          last = here;
          for (;;) {
            here = st->distcode[C_VAL(last) + (BITS(C_BITS(last) + C_OP(last)) >> C_BITS(last))];
            if (C_BITS(last) + C_BITS(here) <= bits) break;
            PULLBYTE();
          }
          DROPBITS(C_BITS(last));
          st->back += (int)C_BITS(last);
        }
        DROPBITS(C_BITS(here));
        st->back += (int)C_BITS(here);
        if (C_OP(here) & 64) { st->msg = "invalid distance code"; st->mode = BAD; break; }
        st->offset = C_VAL(here);
        st->extra = C_OP(here) & 15;
        st->mode = DISTEXT;
        /* fallthrough */
      case DISTEXT:
        if (st->extra) {
          NEEDBITS(st->extra);
          st->offset += BITS(st->extra);
          DROPBITS(st->extra);
          st->back += (int)st->extra;
        }
        st->mode = MATCH;
        /* fallthrough */
      case MATCH:
        if (left == 0) goto inf_leave;
        copy = out - left;
        if (st->offset > copy) {
          copy = st->offset - copy;
          if (copy > st->w_have && st->sane) { st->msg = "invalid distance too far back"; st->mode = BAD; break; }
          const uint8_t *from;
          if (copy > st->w_next) { copy -= st->w_next; from = st->window + (st->w_size - copy); }
          else from = st->window + (st->w_next - copy);
          if (copy > st->length) copy = st->length;
          if (copy > left) copy = left;
          for (unsigned i = 0; i < copy; i++) *put++ = *from++;
        } else {
          const uint8_t *from = put - st->offset;
          copy = st->length;
          if (copy > left) copy = left;
          for (unsigned i = 0; i < copy; i++) *put++ = *from++;
        }
        left -= copy;
        st->length -= copy;
        if (st->length == 0) st->mode = LEN;
        break;
      case LIT:
        if (left == 0) goto inf_leave;
        *put++ = (uint8_t)st->length;
        left--;
        st->mode = LEN;
        break;
      case CHECK:
        if (st->wrap) {
          NEEDBITS(32);
          out -= left;
          st->total_out += out;
          st->total += out;
          if ((st->wrap & 4) && out)
            st->check = st->flags ? zo_crc32(st->check, put - out, out) : zo_adler32(st->check, put - out, out);
          out = left;
          uint32_t want = st->flags ? hold
                                    : (((hold & 0xff) << 24) | (((hold >> 8) & 0xff) << 16) |
                                       (((hold >> 16) & 0xff) << 8) | ((hold >> 24) & 0xff));
          if ((st->wrap & 4) && want != st->check) { st->msg = "incorrect data check"; st->mode = BAD; break; }
          INITBITS();
        }
        st->mode = LENGTH;
        /* fallthrough */
      case LENGTH:
        if (st->wrap && st->flags) {
          NEEDBITS(32);
          if ((st->wrap & 4) && hold != st->total) { st->msg = "incorrect length check"; st->mode = BAD; break; }
          INITBITS();
        }
        st->mode = DONE;
        /* fallthrough */
      case DONE:
        ret = ZO_STREAM_END;
        goto inf_leave;
      case BAD:
        ret = ZO_DATA_ERROR;
        goto inf_leave;
      case MEM:
        return ZO_MEM_ERROR;
      default:
        return ZO_STREAM_ERROR;
    }
  }
inf_leave: /* inflate.ts:1059-1100 */
  RESTORE();
  if (st->w_size ||
      (out != st->avail_out && st->mode < BAD && (st->d64 ? st->mode < DONE : st->mode < CHECK)) || !finish) {
    unsigned written = out - st->avail_out;
    if (updatewindow(st, st->next_out, written)) { st->mode = MEM; return ZO_MEM_ERROR; }
  }
  in -= st->avail_in;
  out -= st->avail_out;
  st->total_in += in;
  st->total_out += out;
  st->total += out;
  if ((st->wrap & 4) && out)
    st->check = st->flags ? zo_crc32(st->check, st->next_out - out, out) : zo_adler32(st->check, st->next_out - out, out);
  if ((in == 0 && out == 0 && ret == ZO_OK) || (finish && ret == ZO_OK)) ret = ZO_BUF_ERROR;
  (void)out_start;
  return ret;
#undef LOAD
#undef RESTORE
#undef INITBITS
#undef PULLBYTE
#undef NEEDBITS
#undef BITS
#undef DROPBITS
#undef BYTEBITS
}

int zo_decompress(const uint8_t *in, size_t n, int wbits, uint8_t *out, size_t cap, size_t *out_len, size_t *consumed,
                  int *phase, const char **msg) {
  *out_len = 0;
  *consumed = 0;
  *phase = ZO_PHASE_NONE;
  *msg = "";
  init_tables();
  istate *st = (istate *)calloc(1, sizeof(istate));
  if (!st) return ZO_MEM_ERROR;
  int ret = inflate_reset2(st, wbits);
  if (ret != ZO_OK) { free(st); *phase = ZO_PHASE_INIT; return ret; }
  uint8_t *obuf = (uint8_t *)malloc(OUT_BUF);
  size_t total = 0;
  int ended = 0, result = ZO_STREAM_END, ovf = 0;
  /* transform(): streams.ts:68-131 */
  for (size_t off = 0; off < n && !ended && result == ZO_STREAM_END; off += IN_CHUNK) {
    size_t len = n - off < IN_CHUNK ? n - off : IN_CHUNK;
    st->next_in = in + off;
    st->avail_in = (unsigned)len;
    while (st->avail_in > 0) {
      st->next_out = obuf;
      st->avail_out = OUT_BUF;
      int r = inflate_call(st, 0);
      size_t produced = OUT_BUF - st->avail_out;
      if (total + produced > cap) ovf = 1; else memcpy(out + total, obuf, produced);
      total += produced;
      if (r == ZO_STREAM_END) { ended = 1; break; }
      if (r != ZO_OK) { result = r; *phase = ZO_PHASE_PROCESS; *msg = st->msg; break; }
    }
  }
  /* flush(): streams.ts:132-166 */
  if (!ended && result == ZO_STREAM_END) {
    for (;;) {
      st->next_out = obuf;
      st->avail_out = OUT_BUF;
      int r = inflate_call(st, 1);
      size_t produced = OUT_BUF - st->avail_out;
      if (total + produced > cap) ovf = 1; else memcpy(out + total, obuf, produced);
      total += produced;
      if (r == ZO_STREAM_END) break;
      if (r != ZO_OK) { result = r; *phase = ZO_PHASE_FINISH; *msg = st->msg; break; }
    }
  }
  *out_len = total;
  *consumed = st->total_in;
  free(obuf);
  free(st->window);
  free(st);
  if (ovf) { *phase = ZO_PHASE_NONE; return ZO_MEM_ERROR; }
  return result;
}
