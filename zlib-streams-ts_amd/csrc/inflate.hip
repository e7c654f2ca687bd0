// inflate.hip -- batched DecompressionStream(format) on gfx950.
//
// One wave per stream.  Decoding is serial in bit position, so the 64 lanes
// run the reference's inflate state machine in lock-step on identical values
// (uniform control flow, broadcast LDS/L1 reads) and split only the byte-moving
// work: match copies (up to 64 bytes per step, or `dist` bytes when the copy
// overlaps itself), stored-block copies, and flushing the LDS history ring to
// HBM with the running Adler-32 / CRC-32 folded in wave-parallel.
//
// The state machine is the reference's inflate() (inflate.ts:332-1185) with
// inflate_fast (inffast.ts:5-228) and inflate_table (inftrees.ts:62-307),
// including the deflate64 mode (windowBits -16: 64 KiB window, length code 285
// = 3 + 16 extra bits, distance codes 30/31, never inflate_fast).  It is driven
// exactly as streams.ts drives it for one write() + close(): the input is cut
// into 32 KiB sub-chunks, each inflate(Z_NO_FLUSH) call gets a fresh 64 KiB
// output buffer, then inflate(Z_FINISH) calls (streams.ts:68-182).  Emulating
// those call boundaries reproduces when inflate_fast runs, the window bookkeeping
// (w_have) and which stream-layer call reports an error ("process error: N"
// vs "finalization error: N").
//
// The reference's window-wrap defect is reproduced (flag ZS_INF_REF_WRAP, the
// default): when an inflate_fast copy sourced from the window wraps the ring
// (w_next < op2) and the rest fits in w_next, inffast.ts:133-147 sets
// from_index = 0 and copies the rest from the caller's OUTPUT buffer at index
// 0 -- i.e. from where this inflate() call began writing -- instead of from
// window[0].  The engine tracks the reference's w_next (updatewindow,
// inflate.ts:282-324, under inf_leave's own call condition,
// inflate.ts:1059-1072) and copies from the call's first output byte, which
// is always already written when read (tests/golden/inffast_wrap_defect.json,
// made by the reference itself).  Without the flag it copies the true history
// (zlib semantics).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"
#include "zs_inflate.h"

#define IN_CHUNK 32768u   // streams.ts:7
#define OUT_BUF 65536u    // streams.ts:6
#define ENOUGH_LENS 852u  // inflate/constants.ts:4-6
#define ENOUGH_DISTS_9 594u
#define FLUSH_AT 4096u    // ring bytes flushed to HBM per step

typedef uint32_t zcode;  // op << 24 | bits << 16 | val (inflate/utils.ts:51-72)
#define C_OP(c) ((c) >> 24)
#define C_BITS(c) (((c) >> 16) & 0xffu)
#define C_VAL(c) ((c) & 0xffffu)

enum { HEAD = 0, FLAGS, TIME, OS, EXLEN, EXTRA, NAME, COMMENT, HCRC, DICTID, DICT, TYPE, TYPEDO, STORED, COPY_, COPY,
       TABLE, LENLENS, CODELENS, LEN_, LEN, LENEXT, DIST, DISTEXT, MATCH, LIT, CHECK, LENGTH, DONE, BAD };
enum { CODES = 0, LENS, DISTS };

static __device__ __forceinline__ zcode zpack(uint32_t op, uint32_t bits, uint32_t val) {
  return (op << 24) | (bits << 16) | val;
}

// length/distance tables, inflate/constants.ts:8-45 (ops: 16 + extra, deflate64: 128 + extra)
static __device__ __forceinline__ void zs_lbase(uint32_t i, bool d64, uint32_t& base, uint32_t& op) {
  static constexpr uint16_t lb[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
  static constexpr uint8_t le[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
  if (i < 28) { base = lb[i]; op = (d64 ? 128u : 16u) + le[i]; }
  else if (i == 28) { base = d64 ? 3u : 258u; op = d64 ? 144u : 16u; }
  else { base = 0; op = d64 ? (i == 29 ? 72u : 78u) : (i == 29 ? 73u : 200u); }
}
static __device__ __forceinline__ void zs_dbase(uint32_t i, bool d64, uint32_t& base, uint32_t& op) {
  static constexpr uint16_t db[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                      193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
  static constexpr uint8_t de[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  if (i < 30) { base = db[i]; op = (d64 ? 128u : 16u) + de[i]; }
  else if (d64) { base = i == 30 ? 32769u : 49153u; op = 128u + 14u; }
  else { base = 0; op = 64u; }
}

// inflate_table (inftrees.ts:62-279).  Returns 0 ok, -1 bad code set, 1 over ENOUGH.
// All lanes execute it on identical values (writes are duplicated, benign).
static __device__ int zs_inflate_table(int type, const uint16_t* lens, uint32_t codes, zcode* table, uint32_t* bits_io,
                                       uint16_t* work, bool d64, uint32_t* used_out) {
  uint32_t len, sym, min, max, root, curr, drop, used, huff, incr, fill, low, mask;
  int left;
  zcode here;
  uint32_t next = 0;
  uint16_t count[16], offs[16];
  const uint32_t enough_d = d64 ? ENOUGH_DISTS_9 : 592u;
  for (len = 0; len <= 15; len++) count[len] = 0;
  for (sym = 0; sym < codes; sym++) count[lens[sym]]++;
  root = *bits_io;
  for (max = 15; max >= 1; max--) if (count[max] != 0) break;
  if (root > max) root = max;
  if (max == 0) {
    if (!d64) {  // _createTableWhenNoCodes
      table[0] = zpack(64, 1, 0);
      table[1] = zpack(64, 1, 0);
      *bits_io = 1;
      *used_out = 0;
      return 0;
    }
    return -1;
  }
  for (min = 1; min < max; min++) if (count[min] != 0) break;
  if (root < min) root = min;
  left = 1;
  for (len = 1; len <= 15; len++) {
    left <<= 1;
    left -= count[len];
    if (left < 0) return -1;
  }
  if (left > 0 && (type == CODES || max != 1)) return -1;
  offs[1] = 0;
  for (len = 1; len < 15; len++) offs[len + 1] = (uint16_t)(offs[len] + count[len]);
  for (sym = 0; sym < codes; sym++) if (lens[sym] != 0) work[offs[lens[sym]]++] = (uint16_t)sym;
  const int match = type == CODES ? (d64 ? 19 : 20) : type == LENS ? (d64 ? 256 : 257) : (d64 ? -1 : 0);
  huff = 0;
  sym = 0;
  len = min;
  curr = root;
  drop = 0;
  low = 0xffffffffu;
  used = 1u << root;
  mask = used - 1;
#define ZS_OVER(u) ((type == LENS && (d64 ? (u) >= ENOUGH_LENS : (u) > ENOUGH_LENS)) || \
                    (type == DISTS && (d64 ? (u) >= enough_d : (u) > enough_d)))
  if (ZS_OVER(used)) return 1;
  for (;;) {
    const int w = work[sym];
    if (d64 ? w < match : w + 1 < match) {
      here = zpack(0, len - drop, (uint32_t)w);
    } else if (d64 ? w > match : w >= match) {
      uint32_t b, op;
      if (type == CODES) { b = (uint32_t)work[w - match]; op = b; }  // unreachable for valid CODES tables
      else if (type == LENS) zs_lbase((uint32_t)(w - 257), d64, b, op);
      else zs_dbase((uint32_t)(d64 ? w : w - match), d64, b, op);
      here = zpack(op, len - drop, b);
    } else {
      here = zpack(32 + 64, len - drop, 0);
    }
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
      if (ZS_OVER(used)) return 1;
      low = huff & mask;
      table[low] = zpack(curr, root, next);
    }
  }
  if (huff != 0) {
    here = zpack(64, len - drop, 0);
    while (huff != 0) {
      if (drop != 0 && (huff & mask) != low) {
        drop = 0;
        len = root;
        next = 0;
        curr = root;
        here = zpack(64, len, 0);
      }
      table[next + (huff >> drop)] = here;
      incr = 1u << (len - 1);
      while (huff & incr) incr >>= 1;
      if (incr != 0) { huff &= incr - 1; huff += incr; } else huff = 0;
    }
  }
#undef ZS_OVER
  *used_out = used;
  *bits_io = root;
  return 0;
}

// ---------------------------------------------------------- checksums (wave)
static __device__ uint32_t zs_crc_mul(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0xedb88320u : b >> 1;
  }
  return p;
}
static __device__ uint32_t zs_crc_x8n(uint32_t len) {
  uint32_t p = 1u << 31, sq = 1u << 23;
  while (len) {
    if (len & 1) p = zs_crc_mul(sq, p);
    sq = zs_crc_mul(sq, sq);
    len >>= 1;
  }
  return p;
}

#define ZS_IBUF 4096u

struct zs_lds {
  uint8_t ibuf[ZS_IBUF + 16];  // staged input bytes [ib0, ib0 + ZS_IBUF)
  uint32_t crct[256];
  uint32_t red[64];
  uint16_t lens[320];
  uint16_t work[288];
  zcode codes[ENOUGH_LENS + ENOUGH_DISTS_9];
  zcode fixed[544];
};

// State of one stream (all lanes hold identical copies).
struct zs_ist {
  const uint8_t* src;
  uint32_t n;         // input length
  uint8_t* dst;
  uint32_t cap;       // output capacity
  uint8_t* ring;      // LDS history ring
  uint32_t rmask;
  uint64_t total;     // bytes output so far (absolute)
  uint64_t flushed;   // bytes already copied from ring to dst (and checksummed)
  int mode, last, wrap, havedict, flags, d64, back;
  uint32_t check, w_bits, w_size, w_have, w_next;
  int ref_wrap;  // reproduce inffast.ts:133-147 (see the top of this file)
  uint64_t hold;
  uint32_t bits, length, offset, extra, was;
  uint32_t lenbits, distbits, ncode, nlen, ndist, have_;
  uint32_t lencode_off, distcode_off;  // into codes[] or fixed[] (bit 31: fixed)
  int msg;
  int overflow;
  uint32_t total_in;
  uint32_t ib0;  // input index of ibuf[0]
};

// input byte at absolute index i (i < n), staged 4 KiB at a time through LDS
static __device__ __forceinline__ uint32_t zs_in(zs_lds& L, zs_ist& S, uint32_t i) {
  if (i - S.ib0 >= ZS_IBUF) {
    __builtin_amdgcn_wave_barrier();
    for (uint32_t k = threadIdx.x; k < ZS_IBUF; k += 64) L.ibuf[k] = i + k < S.n ? S.src[i + k] : 0;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    S.ib0 = i;
  }
  return L.ibuf[i - S.ib0];
}

static __device__ __forceinline__ zcode zs_lcode(const zs_lds& L, const zs_ist& S, uint32_t i) {
  return (S.lencode_off & 0x80000000u) ? L.fixed[(S.lencode_off & 0x7fffffffu) + i] : L.codes[S.lencode_off + i];
}
static __device__ __forceinline__ zcode zs_dcode(const zs_lds& L, const zs_ist& S, uint32_t i) {
  return (S.distcode_off & 0x80000000u) ? L.fixed[(S.distcode_off & 0x7fffffffu) + i] : L.codes[S.distcode_off + i];
}

// Copy ring bytes [flushed, upto) to HBM, folding them into the running check.
static __device__ void zs_flush(zs_lds& L, zs_ist& S, uint64_t upto) {
  const uint32_t lane = threadIdx.x;
  // running check: crc32 for gzip (flags > 0), adler32 for zlib (flags == 0), none for raw
  const int chk = (S.wrap & 4) ? (S.flags > 0 ? 2 : (S.flags == 0 ? 1 : 0)) : 0;
  while (S.flushed < upto) {
    const uint64_t f0 = S.flushed;
    const uint32_t cnt = (uint32_t)min<uint64_t>(upto - f0, FLUSH_AT);
    if (f0 + cnt <= S.cap) {
      for (uint32_t i = lane; i < cnt; i += 64) S.dst[f0 + i] = S.ring[(f0 + i) & S.rmask];
    }
    if (chk) {
      const uint32_t per = (cnt + 63) / 64;
      const uint32_t b0 = min(cnt, lane * per), b1 = min(cnt, b0 + per);
      if (chk == 2) {
        uint32_t c = 0xffffffffu;
        for (uint32_t i = b0; i < b1; i++) c = (c >> 8) ^ L.crct[(c ^ S.ring[(f0 + i) & S.rmask]) & 0xff];
        L.red[lane] = c ^ 0xffffffffu;
        __syncthreads();
        uint32_t crc = S.check;  // crc32(crc, chunk): fold segments in order
        const uint32_t xp = zs_crc_x8n(per);
        for (uint32_t i = 0; i < 64; i++) {
          const uint32_t lo = min(cnt, i * per), hi = min(cnt, lo + per);
          if (hi == lo) break;
          crc = zs_crc_mul(hi - lo == per ? xp : zs_crc_x8n(hi - lo), crc) ^ L.red[i];
        }
        __syncthreads();
        S.check = crc;
      } else {
        // adler32(check, chunk): A' = A + sum x, B' = B + cnt*A + sum (cnt - j) x_j  (mod 65521)
        uint32_t a = 0, w = 0;
        for (uint32_t i = b0; i < b1; i++) {
          const uint32_t x = S.ring[(f0 + i) & S.rmask];
          a += x;
          w += (cnt - i) * x;
          w %= 65521u;
        }
        a %= 65521u;
        uint32_t a64 = a, w64 = w;  // 64 x 65520 < 2^32
        for (int d = 32; d >= 1; d >>= 1) {
          a64 += __shfl_xor(a64, d, 64);
          w64 += __shfl_xor(w64, d, 64);
        }
        const uint64_t A = S.check & 0xffffu, B = S.check >> 16;
        const uint64_t nA = (A + a64) % 65521u;
        const uint64_t nB = (B + (uint64_t)cnt % 65521u * A + (uint64_t)w64) % 65521u;
        S.check = (uint32_t)((nB << 16) | nA);
      }
    }
    S.flushed = f0 + cnt;
  }
}

static __device__ __forceinline__ void zs_put(zs_ist& S, uint32_t c) {
  if (threadIdx.x == 0) S.ring[S.total & S.rmask] = (uint8_t)c;
  S.total++;
}

// match copy of len bytes from dist back (all lanes)
static __device__ __forceinline__ void zs_copy(zs_ist& S, uint32_t dist, uint32_t len) {
  const uint32_t step = dist < 64 ? dist : 64;
  for (uint32_t o = 0; o < len; o += step) {
    const uint32_t k = min(step, len - o);
    if (threadIdx.x < k) {
      const uint64_t at = S.total + o + threadIdx.x;
      S.ring[at & S.rmask] = S.ring[(at - dist) & S.rmask];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  S.total += len;
}

static __device__ void zs_fixedtables(zs_lds& L, zs_ist& S) {  // inflate.ts:218-280
  uint32_t sym, bits, used;
  for (sym = 0; sym < 144; sym++) L.lens[sym] = 8;
  for (; sym < 256; sym++) L.lens[sym] = 9;
  for (; sym < 280; sym++) L.lens[sym] = 7;
  for (; sym < 288; sym++) L.lens[sym] = 8;
  bits = 9;
  zs_inflate_table(LENS, L.lens, 288, L.fixed, &bits, L.work, S.d64, &used);
  const uint32_t dist_at = used;
  for (sym = 0; sym < 32; sym++) L.lens[sym] = 5;
  bits = 5;
  zs_inflate_table(DISTS, L.lens, 32, L.fixed + dist_at, &bits, L.work, S.d64, &used);
  S.lencode_off = 0x80000000u;
  S.lenbits = 9;
  S.distcode_off = 0x80000000u | dist_at;
  S.distbits = 5;
}

// One inflate() call (inflate.ts:332-1185).  The call's input is src[in0, in0 + avail)
// and its output buffer holds `avail_out` bytes.  Returns the Z_* code; advances
// *in_pos by the bytes the call consumed and *out_used by the bytes it produced.
static __device__ int zs_inflate_call(zs_lds& L, zs_ist& S, uint32_t in0, uint32_t avail, uint32_t avail_out,
                                      bool finish, uint32_t* consumed, uint32_t* produced) {
  uint32_t next = in0;          // absolute input index
  uint32_t have = avail;        // bytes available to this call
  uint32_t left = avail_out;    // output space of this call
  uint64_t hold = S.hold;
  uint32_t bits = S.bits;
  const uint32_t in_start = have, out_start = left;
  uint32_t out = left;          // `out` of the reference (reset at CHECK)
  int ret = ZS_Z_OK;
  zcode here, last;
  uint32_t len, copy;
#define PULLBYTE() do { if (have == 0) goto inf_leave; have--; hold += (uint64_t)zs_in(L, S, next++) << bits; bits += 8; } while (0)
#define NEEDBITS(k) do { while (bits < (uint32_t)(k)) PULLBYTE(); } while (0)
#define BITS(k) ((uint32_t)hold & ((1u << (k)) - 1))
#define DROPBITS(k) do { hold >>= (k); bits -= (uint32_t)(k); } while (0)
#define INITBITS() do { hold = 0; bits = 0; } while (0)
#define BYTEBITS() do { hold >>= bits & 7; bits -= bits & 7; } while (0)
  if (S.mode == TYPE) S.mode = TYPEDO;
  for (;;) {
    // keep the ring from overrunning unflushed bytes
    if (S.total - S.flushed >= FLUSH_AT) zs_flush(L, S, S.total - (S.total & (FLUSH_AT - 1)));
    if (S.total > S.cap) { S.overflow = 1; goto inf_leave; }
    switch (S.mode) {
      case HEAD:
        if (S.wrap == 0) { S.mode = TYPEDO; break; }
        NEEDBITS(16);
        if ((S.wrap & 2) && hold == 0x8b1f) {
          if (S.w_bits == 0) S.w_bits = 15;
          uint32_t c = 0xffffffffu;
          c = (c >> 8) ^ L.crct[(c ^ (uint32_t)(hold & 0xff)) & 0xff];
          c = (c >> 8) ^ L.crct[(c ^ (uint32_t)((hold >> 8) & 0xff)) & 0xff];
          S.check = c ^ 0xffffffffu;
          INITBITS();
          S.mode = FLAGS;
          break;
        }
        if (!(S.wrap & 1) || ((BITS(8) << 8) + (uint32_t)(hold >> 8)) % 31) { S.msg = ZS_MSG_HEADER_CHECK; S.mode = BAD; break; }
        if (BITS(4) != 8) { S.msg = ZS_MSG_METHOD; S.mode = BAD; break; }
        DROPBITS(4);
        len = BITS(4) + 8;
        if (S.w_bits == 0) S.w_bits = len;
        if (len > 15 || len > S.w_bits) { S.msg = ZS_MSG_WINDOW; S.mode = BAD; break; }
        S.flags = 0;
        S.check = 1;
        S.mode = (hold & 0x200) ? DICTID : TYPE;
        INITBITS();
        break;
      case FLAGS:
        NEEDBITS(16);
        S.flags = (int)hold;
        if ((S.flags & 0xff) != 8) { S.msg = ZS_MSG_METHOD; S.mode = BAD; break; }
        if (S.flags & 0xe000) { S.msg = ZS_MSG_FLAGS; S.mode = BAD; break; }
        S.mode = TIME;
        if ((S.flags & 0x0200) && (S.wrap & 4)) {
          uint32_t c = ~S.check;
          for (int k = 0; k < 2; k++) c = (c >> 8) ^ L.crct[(c ^ (uint32_t)(hold >> (8 * k))) & 0xff];
          S.check = ~c;
        }
        INITBITS();
        [[fallthrough]];
      case TIME:
        NEEDBITS(32);
        if ((S.flags & 0x0200) && (S.wrap & 4)) {
          uint32_t c = ~S.check;
          for (int k = 0; k < 4; k++) c = (c >> 8) ^ L.crct[(c ^ (uint32_t)(hold >> (8 * k))) & 0xff];
          S.check = ~c;
        }
        INITBITS();
        S.mode = OS;
        [[fallthrough]];
      case OS:
        NEEDBITS(16);
        if ((S.flags & 0x0200) && (S.wrap & 4)) {
          uint32_t c = ~S.check;
          for (int k = 0; k < 2; k++) c = (c >> 8) ^ L.crct[(c ^ (uint32_t)(hold >> (8 * k))) & 0xff];
          S.check = ~c;
        }
        INITBITS();
        S.mode = EXLEN;
        [[fallthrough]];
      case EXLEN:
        if (S.flags & 0x0400) {
          NEEDBITS(16);
          S.length = (uint32_t)hold;
          if ((S.flags & 0x0200) && (S.wrap & 4)) {
            uint32_t c = ~S.check;
            for (int k = 0; k < 2; k++) c = (c >> 8) ^ L.crct[(c ^ (uint32_t)(hold >> (8 * k))) & 0xff];
            S.check = ~c;
          }
          INITBITS();
        }
        S.mode = EXTRA;
        [[fallthrough]];
      case EXTRA:
        if (S.flags & 0x0400) {
          copy = S.length;
          if (copy > have) copy = have;
          if (copy) {
            if ((S.flags & 0x0200) && (S.wrap & 4)) {
              uint32_t c = ~S.check;
              for (uint32_t k = 0; k < copy; k++) c = (c >> 8) ^ L.crct[(c ^ zs_in(L, S, next + k)) & 0xff];
              S.check = ~c;
            }
            have -= copy;
            next += copy;
            S.length -= copy;
          }
          if (S.length) goto inf_leave;
        }
        S.length = 0;
        S.mode = NAME;
        [[fallthrough]];
      case NAME:
      case COMMENT: {
        const int flag = S.mode == NAME ? 0x0800 : 0x1000;
        if (S.flags & flag) {
          if (have == 0) goto inf_leave;
          copy = 0;
          do len = zs_in(L, S, next + copy++); while (len && copy < have);
          if ((S.flags & 0x0200) && (S.wrap & 4)) {
            uint32_t c = ~S.check;
            for (uint32_t k = 0; k < copy; k++) c = (c >> 8) ^ L.crct[(c ^ zs_in(L, S, next + k)) & 0xff];
            S.check = ~c;
          }
          have -= copy;
          next += copy;
          if (len) goto inf_leave;
        }
        if (S.mode == NAME) { S.length = 0; S.mode = COMMENT; break; }
        S.mode = HCRC;
        break;
      }
      case HCRC:
        if (S.flags & 0x0200) {
          NEEDBITS(16);
          if ((S.wrap & 4) && (uint32_t)hold != (S.check & 0xffff)) { S.msg = ZS_MSG_HEADER_CRC; S.mode = BAD; break; }
          INITBITS();
        }
        S.check = 0;
        S.mode = TYPE;
        break;
      case DICTID:
        NEEDBITS(32);
        S.check = __builtin_bswap32((uint32_t)hold);
        INITBITS();
        S.mode = DICT;
        [[fallthrough]];
      case DICT:
        // no dictionary API through the stream layer: Z_NEED_DICT (inflate.ts:594-597)
        S.hold = hold;
        S.bits = bits;
        *consumed = in_start - have;
        *produced = out_start - left;
        S.total_in += in_start - have;
        return ZS_Z_NEED_DICT;
      case TYPE:
      case TYPEDO:
        if (S.last) { BYTEBITS(); S.mode = CHECK; break; }
        NEEDBITS(3);
        S.last = (int)BITS(1);
        DROPBITS(1);
        switch (BITS(2)) {
          case 0: S.mode = STORED; break;
          case 1: zs_fixedtables(L, S); S.mode = LEN_; break;
          case 2: S.mode = TABLE; break;
          default: S.msg = ZS_MSG_BLOCK_TYPE; S.mode = BAD;
        }
        DROPBITS(2);
        break;
      case STORED:
        BYTEBITS();
        NEEDBITS(32);
        if ((hold & 0xffff) != (((hold >> 16) & 0xffff) ^ 0xffff)) { S.msg = ZS_MSG_STORED_LEN; S.mode = BAD; break; }
        S.length = (uint32_t)(hold & 0xffff);
        INITBITS();
        S.mode = COPY_;
        [[fallthrough]];
      case COPY_:
        S.mode = COPY;
        [[fallthrough]];
      case COPY:
        copy = S.length;
        if (copy) {
          if (copy > have) copy = have;
          if (copy > left) copy = left;
          if (copy > FLUSH_AT) copy = FLUSH_AT;  // bounded by the ring headroom
          if (copy == 0) goto inf_leave;
          for (uint32_t k = threadIdx.x; k < copy; k += 64) S.ring[(S.total + k) & S.rmask] = S.src[next + k];
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
          S.total += copy;
          have -= copy;
          next += copy;
          left -= copy;
          S.length -= copy;
          break;
        }
        S.mode = TYPE;
        break;
      case TABLE:
        NEEDBITS(14);
        S.nlen = BITS(5) + 257;
        DROPBITS(5);
        S.ndist = BITS(5) + 1;
        DROPBITS(5);
        S.ncode = BITS(4) + 4;
        DROPBITS(4);
        if (S.nlen > 286 || (!S.d64 && S.ndist > 30)) {
          S.msg = S.d64 ? ZS_MSG_TOO_MANY_D64 : ZS_MSG_TOO_MANY;
          S.mode = BAD;
          break;
        }
        S.have_ = 0;
        S.mode = LENLENS;
        [[fallthrough]];
      case LENLENS: {
        while (S.have_ < S.ncode) {
          NEEDBITS(3);
          L.lens[ZS_BL_ORDER[S.have_++]] = (uint16_t)BITS(3);
          DROPBITS(3);
        }
        while (S.have_ < 19) L.lens[ZS_BL_ORDER[S.have_++]] = 0;
        S.lencode_off = S.distcode_off = 0;
        S.lenbits = 7;
        uint32_t used;
        const int r = zs_inflate_table(CODES, L.lens, 19, L.codes, &S.lenbits, L.work, S.d64, &used);
        if (r) { S.msg = ZS_MSG_CODE_LENGTHS; S.mode = BAD; break; }
        S.have_ = 0;
        S.mode = CODELENS;
      }
        [[fallthrough]];
      case CODELENS: {
        while (S.have_ < S.nlen + S.ndist) {
          for (;;) {
            here = zs_lcode(L, S, BITS(S.lenbits));
            if (C_BITS(here) <= bits) break;
            PULLBYTE();
          }
          if (C_VAL(here) < 16) {
            DROPBITS(C_BITS(here));
            L.lens[S.have_++] = (uint16_t)C_VAL(here);
          } else {
            if (C_VAL(here) == 16) {
              NEEDBITS(C_BITS(here) + 2);
              DROPBITS(C_BITS(here));
              if (S.have_ == 0) { S.msg = ZS_MSG_REPEAT; S.mode = BAD; break; }
              len = L.lens[S.have_ - 1];
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
            if (S.have_ + copy > S.nlen + S.ndist) { S.msg = ZS_MSG_REPEAT; S.mode = BAD; break; }
            while (copy--) L.lens[S.have_++] = (uint16_t)len;
          }
        }
        if (S.mode == BAD) break;
        if (L.lens[256] == 0) { S.msg = ZS_MSG_MISSING_EOB; S.mode = BAD; break; }
        uint32_t lused, dused;
        S.lenbits = 9;
        int r = zs_inflate_table(LENS, L.lens, S.nlen, L.codes, &S.lenbits, L.work, S.d64, &lused);
        S.lencode_off = 0;
        if (r) { S.msg = ZS_MSG_LITLEN_SET; S.mode = BAD; break; }
        S.distbits = 6;
        r = zs_inflate_table(DISTS, L.lens + S.nlen, S.ndist, L.codes + lused, &S.distbits, L.work, S.d64, &dused);
        S.distcode_off = lused;
        if (r) { S.msg = ZS_MSG_DIST_SET; S.mode = BAD; break; }
        S.mode = LEN_;
      }
        [[fallthrough]];
      case LEN_:
        S.mode = LEN;
        [[fallthrough]];
      case LEN:
        if (!S.d64 && have >= 6 && left >= 258) {
          // ---------------- inflate_fast (inffast.ts:5-228) ----------------
          const uint32_t last_in = next + (have - 5);
          const uint64_t beg = S.total - (out_start - left);  // output index where this call began
          const uint64_t endo = S.total + (left - 257);
          const uint32_t lmask = (1u << S.lenbits) - 1, dmask = (1u << S.distbits) - 1;
          const uint32_t whave = S.w_have;
          uint32_t op, dist;
          do {
            if (S.total - S.flushed >= FLUSH_AT) zs_flush(L, S, S.total - (S.total & (FLUSH_AT - 1)));
            while (bits < 15) { hold += (uint64_t)zs_in(L, S, next++) << bits; bits += 8; }
            here = zs_lcode(L, S, (uint32_t)hold & lmask);
            for (;;) {  // dolen
              op = C_BITS(here);
              hold >>= op;
              bits -= op;
              op = C_OP(here);
              if (op == 0) {
                zs_put(S, C_VAL(here));
                break;
              } else if (op & 16) {
                len = C_VAL(here);
                op &= 15;
                if (op) {
                  while (bits < op) { hold += (uint64_t)zs_in(L, S, next++) << bits; bits += 8; }
                  len += (uint32_t)hold & ((1u << op) - 1);
                  hold >>= op;
                  bits -= op;
                }
                while (bits < 15) { hold += (uint64_t)zs_in(L, S, next++) << bits; bits += 8; }
                here = zs_dcode(L, S, (uint32_t)hold & dmask);
                for (;;) {  // dodist
                  op = C_BITS(here);
                  hold >>= op;
                  bits -= op;
                  op = C_OP(here);
                  if (op & 16) {
                    dist = C_VAL(here);
                    op &= 15;
                    while (bits < op) { hold += (uint64_t)zs_in(L, S, next++) << bits; bits += 8; }
                    dist += (uint32_t)hold & ((1u << op) - 1);
                    hold >>= op;
                    bits -= op;
                    const uint64_t outmax = S.total - beg;
                    if (dist > outmax && dist - outmax > whave) {  // inffast.ts:103-112
                      S.msg = ZS_MSG_TOO_FAR;
                      S.mode = BAD;
                      goto fast_done;
                    }
                    if (S.ref_wrap && dist > outmax) {
                      // window-sourced copy: the wrap case of inffast.ts:126-147
                      const uint32_t op2 = (uint32_t)(dist - outmax), wn = S.w_next;
                      if (wn != 0 && wn < op2 && op2 - wn < len && wn >= len - (op2 - wn)) {
                        const uint32_t op3 = op2 - wn;
                        zs_copy(S, dist, op3);                            // window tail (true history)
                        zs_copy(S, (uint32_t)(S.total - beg), len - op3);  // output[0..]: from this call's start
                        break;
                      }
                    }
                    zs_copy(S, dist, len);
                    break;
                  } else if ((op & 64) == 0) {
                    here = zs_dcode(L, S, C_VAL(here) + ((uint32_t)hold & ((1u << op) - 1)));
                  } else {
                    S.msg = ZS_MSG_DIST_CODE;
                    S.mode = BAD;
                    goto fast_done;
                  }
                }
                break;
              } else if ((op & 64) == 0) {
                here = zs_lcode(L, S, C_VAL(here) + ((uint32_t)hold & ((1u << op) - 1)));
              } else if (op & 32) {
                S.mode = TYPE;
                goto fast_done;
              } else {
                S.msg = ZS_MSG_LITLEN_CODE;
                S.mode = BAD;
                goto fast_done;
              }
            }
          } while (next < last_in && S.total < endo);
        fast_done: {
          const uint32_t used = bits >> 3;  // return unused whole bytes
          next -= used;
          bits -= used << 3;
          hold &= (1ull << bits) - 1;
          const uint64_t out_now = S.total - beg;
          left = out_start - (uint32_t)out_now;
          have = in0 + avail - next;
        }
          if (S.mode == TYPE) S.back = -1;
          break;
        }
        S.back = 0;
        for (;;) {
          here = zs_lcode(L, S, BITS(S.lenbits));
          if (C_BITS(here) <= bits) break;
          PULLBYTE();
        }
        if (C_OP(here) && (C_OP(here) & 0xf0) == 0) {
          last = here;
          for (;;) {
            here = zs_lcode(L, S, C_VAL(last) + (BITS(C_BITS(last) + C_OP(last)) >> C_BITS(last)));
            if (C_BITS(last) + C_BITS(here) <= bits) break;
            PULLBYTE();
          }
          DROPBITS(C_BITS(last));
        }
        DROPBITS(C_BITS(here));
        S.length = C_VAL(here);
        if (C_OP(here) == 0) { S.mode = LIT; break; }
        if (C_OP(here) & 32) { S.back = -1; S.mode = TYPE; break; }
        if (C_OP(here) & 64) { S.msg = ZS_MSG_LITLEN_CODE; S.mode = BAD; break; }
        S.extra = C_OP(here) & (S.d64 ? 31u : 15u);
        S.mode = LENEXT;
        [[fallthrough]];
      case LENEXT:
        if (S.extra) {
          NEEDBITS(S.extra);
          S.length += BITS(S.extra);
          DROPBITS(S.extra);
        }
        S.was = S.length;
        S.mode = DIST;
        [[fallthrough]];
      case DIST:
        for (;;) {
          here = zs_dcode(L, S, BITS(S.distbits));
          if (C_BITS(here) <= bits) break;
          PULLBYTE();
        }
        if ((C_OP(here) & 0xf0) == 0) {
          last = here;
          for (;;) {
            here = zs_dcode(L, S, C_VAL(last) + (BITS(C_BITS(last) + C_OP(last)) >> C_BITS(last)));
            if (C_BITS(last) + C_BITS(here) <= bits) break;
            PULLBYTE();
          }
          DROPBITS(C_BITS(last));
        }
        DROPBITS(C_BITS(here));
        if (C_OP(here) & 64) { S.msg = ZS_MSG_DIST_CODE; S.mode = BAD; break; }
        S.offset = C_VAL(here);
        S.extra = C_OP(here) & 15;
        S.mode = DISTEXT;
        [[fallthrough]];
      case DISTEXT:
        if (S.extra) {
          NEEDBITS(S.extra);
          S.offset += BITS(S.extra);
          DROPBITS(S.extra);
        }
        S.mode = MATCH;
        [[fallthrough]];
      case MATCH: {
        if (left == 0) goto inf_leave;
        const uint32_t in_call = out - left;
        if (S.offset > in_call && S.offset - in_call > S.w_have) { S.msg = ZS_MSG_TOO_FAR; S.mode = BAD; break; }
        copy = S.length;
        if (copy > left) copy = left;
        if (copy > FLUSH_AT) copy = FLUSH_AT;  // deflate64 lengths reach 65538: bound by ring headroom
        zs_copy(S, S.offset, copy);
        left -= copy;
        S.length -= copy;
        if (S.length == 0) S.mode = LEN;
        break;
      }
      case LIT:
        if (left == 0) goto inf_leave;
        zs_put(S, S.length);
        left--;
        S.mode = LEN;
        break;
      case CHECK:
        if (S.wrap) {
          NEEDBITS(32);
          out -= left;
          // the running check covers everything output so far (inflate.ts:1010-1015)
          zs_flush(L, S, S.total);
          out = left;
          const uint32_t want = S.flags ? (uint32_t)hold : __builtin_bswap32((uint32_t)hold);
          if ((S.wrap & 4) && want != S.check) { S.msg = ZS_MSG_DATA_CHECK; S.mode = BAD; break; }
          INITBITS();
        }
        S.mode = LENGTH;
        [[fallthrough]];
      case LENGTH:
        if (S.wrap && S.flags) {
          NEEDBITS(32);
          if ((S.wrap & 4) && (uint32_t)hold != (uint32_t)S.total) { S.msg = ZS_MSG_LENGTH_CHECK; S.mode = BAD; break; }
          INITBITS();
        }
        S.mode = DONE;
        [[fallthrough]];
      case DONE:
        ret = ZS_Z_STREAM_END;
        goto inf_leave;
      case BAD:
        ret = ZS_Z_DATA_ERROR;
        goto inf_leave;
      default:
        ret = ZS_Z_STREAM_ERROR;
        goto inf_leave;
    }
  }
inf_leave:
  S.hold = hold;
  S.bits = bits;
  {
    const uint32_t in_used = in_start - have;
    const uint32_t out_used = out_start - left;
    // updatewindow bookkeeping (inflate.ts:282-324) under inf_leave's call
    // condition (inflate.ts:1060-1067; note `|| flush != Z_FINISH` at top level)
    const uint32_t written = out - left;
    if (S.w_size || (written && S.mode < BAD && (S.d64 ? S.mode < DONE : S.mode < CHECK)) || !finish) {
      if (S.w_size == 0) { S.w_size = 1u << S.w_bits; S.w_next = 0; S.w_have = 0; }
      if (written >= S.w_size) {
        S.w_next = 0;
        S.w_have = S.w_size;
      } else {
        const uint32_t d = min(S.w_size - S.w_next, written);
        if (written > d) {
          S.w_next = written - d;
          S.w_have = S.w_size;
        } else {
          S.w_next += d;
          if (S.w_next == S.w_size) S.w_next = 0;
          S.w_have = min(S.w_size, S.w_have + d);
        }
      }
    }
    *consumed = in_used;
    *produced = out_used;
    S.total_in += in_used;
    if ((in_used == 0 && out_used == 0 && ret == ZS_Z_OK) || (finish && ret == ZS_Z_OK)) ret = ZS_Z_BUF_ERROR;
  }
  return ret;
#undef PULLBYTE
#undef NEEDBITS
#undef BITS
#undef DROPBITS
#undef INITBITS
#undef BYTEBITS
}

extern __shared__ __attribute__((aligned(16))) uint8_t zs_inflate_smem[];

__global__ __launch_bounds__(64) void zs_k_inflate(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                   const uint64_t* __restrict__ out_off,
                                                   const uint32_t* __restrict__ out_cap, int wbits,
                                                   zs_inflate_result* __restrict__ res,
                                                   const zs_lane_res* __restrict__ only, int flags) {
  zs_lds& L = *reinterpret_cast<zs_lds*>(zs_inflate_smem);
  const int s = blockIdx.x;
  if (only && only[s].bail == 0) return;  // decoded cleanly by the lane path
  zs_ist S;
  S.src = in + in_off[s];
  S.n = in_len[s];
  S.dst = out + out_off[s];
  S.cap = out_cap[s];
  // inflateReset2 (inflate.ts:138-172)
  int w = wbits;
  if (w < 0) { S.wrap = 0; S.d64 = (w == -16); w = -w; }
  else { S.wrap = (w >> 4) + 5; S.d64 = 0; if (w < 48) w &= 15; }
  S.w_bits = (uint32_t)w;
  S.ring = zs_inflate_smem + sizeof(zs_lds);
  S.rmask = (S.d64 ? 65536u : 32768u) + (S.d64 ? 65536u : 32768u) - 1;  // ring = 2 x window
  S.total = S.flushed = 0;
  S.mode = S.d64 ? TYPE : HEAD;
  S.last = 0; S.havedict = 0; S.flags = -1; S.back = -1;
  S.check = S.wrap ? (uint32_t)(S.wrap & 1) : 0;
  S.w_size = 0; S.w_have = 0; S.w_next = 0;
  S.ref_wrap = (flags & ZS_INF_REF_WRAP) != 0;
  S.hold = 0; S.bits = 0;
  S.length = S.offset = S.extra = S.was = 0;
  S.lenbits = S.distbits = S.ncode = S.nlen = S.ndist = S.have_ = 0;
  S.lencode_off = S.distcode_off = 0;
  S.msg = ZS_MSG_NONE;
  S.overflow = 0;
  S.total_in = 0;
  S.ib0 = 0xf0000000u;
  for (uint32_t i = threadIdx.x; i < 256; i += 64) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
    L.crct[i] = c;
  }
  __syncthreads();

  int status = ZS_Z_STREAM_END, phase = ZS_PHASE_NONE_;
  bool ended = false;
  // transform(): 32 KiB sub-chunks, inflate(Z_NO_FLUSH) while input remains (streams.ts:68-131)
  for (uint32_t off = 0; off < S.n && !ended && phase == ZS_PHASE_NONE_; off += IN_CHUNK) {
    uint32_t pos = off;
    const uint32_t end = min(S.n, off + IN_CHUNK);
    while (pos < end) {
      uint32_t used, produced;
      const int r = zs_inflate_call(L, S, pos, end - pos, OUT_BUF, false, &used, &produced);
      pos += used;
      if (S.overflow) break;
      if (r == ZS_Z_STREAM_END) { ended = true; break; }
      if (r != ZS_Z_OK) { status = r; phase = ZS_PHASE_PROCESS_; break; }
    }
    if (S.overflow) break;
  }
  // flush(): inflate(Z_FINISH) until Z_STREAM_END (streams.ts:132-166)
  if (!ended && phase == ZS_PHASE_NONE_ && !S.overflow) {
    for (;;) {
      uint32_t used, produced;
      const int r = zs_inflate_call(L, S, S.n, 0, OUT_BUF, true, &used, &produced);
      if (S.overflow) break;
      if (r == ZS_Z_STREAM_END) break;
      if (r != ZS_Z_OK) { status = r; phase = ZS_PHASE_FINISH_; break; }
    }
  }
  if (!S.overflow) zs_flush(L, S, S.total);
  if (threadIdx.x == 0) {
    zs_inflate_result R;
    if (S.overflow || S.total > S.cap) {
      R.status = ZS_Z_BUF_ERROR;
      R.phase = ZS_PHASE_NONE_;
      R.msg = ZS_MSG_CAPACITY;
      R.out_len = 0;
    } else {
      R.status = status;
      R.phase = phase;
      R.msg = status == ZS_Z_DATA_ERROR ? S.msg : ZS_MSG_NONE;
      R.out_len = (uint32_t)S.total;
    }
    R.consumed = S.total_in;
    res[s] = R;
  }
}

size_t zs_inflate_smem_bytes(int wbits) {
  const size_t ring = wbits == -16 ? 2 * 65536 : 2 * 32768;
  return sizeof(zs_lds) + ring;
}

// ===================================================================== fast path
// One LANE per member.  The exact kernel above spends a whole wave on one
// stream because it re-enacts the stream layer's call boundaries; a member
// whose decoding those boundaries cannot change decodes straight through in one
// lane instead: a deflate64 member (the reference decodes it with the slow state
// machine only, whose window copies are exact), or a deflate / zlib / gzip member
// that one inflate() call of the reference decodes whole (see ZS_INF_REF_WRAP
// below).  zlib's own tables (inflate_table above, so invalid codes are
// recognised exactly as the reference does), a 64-bit bit buffer, output written
// to HBM and match history read back from it.  A member takes the exact path
// instead (zs_k_inflate over the bailed members) on ANY condition that is not a
// clean end of stream -- a data error, truncated input, a dictionary request,
// gzip header fields, a checksum or length mismatch, or output capacity -- so
// statuses, phases and messages always come from the exact state machine.
struct zs_lane_tabs {
  zcode codes[ENOUGH_LENS + ENOUGH_DISTS_9];
  uint16_t lens[320];
  uint16_t work[288];
};

struct zs_lane_reader {
  const uint8_t* src;
  uint32_t n, pos;  // bytes moved into hold so far
  uint64_t hold;
  uint32_t bits;
  uint32_t pf;      // input bytes [pos, pos + 4), loaded one refill ahead (zero past the end)
};

static __device__ __forceinline__ uint32_t zs_lr_load4(const zs_lane_reader& R, uint32_t at) {
  uint32_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++)
    if (at + k < R.n) v |= (uint32_t)R.src[at + k] << (8 * k);
  return v;
}
// bits < 32 -> bits >= 32: the prefetched word enters hold and the next one is
// requested, so its latency overlaps the decoding of the bits just added
static __device__ __forceinline__ void zs_lr_fill(zs_lane_reader& R) {
  R.hold |= (uint64_t)R.pf << R.bits;
  R.bits += 32;
  R.pos += 4;
  R.pf = zs_lr_load4(R, R.pos);
}
// bits consumed so far
static __device__ __forceinline__ uint64_t zs_lr_bitpos(const zs_lane_reader& R) {
  return (uint64_t)R.pos * 8u - R.bits;
}
// consumed bits beyond the input: a truncated stream (the exact path reports it)
static __device__ __forceinline__ bool zs_lr_over(const zs_lane_reader& R) {
  return zs_lr_bitpos(R) > (uint64_t)R.n * 8u;
}
static __device__ __forceinline__ uint32_t zs_lr_take(zs_lane_reader& R, uint32_t k) {  // k <= 32
  if (R.bits < k) zs_lr_fill(R);
  const uint32_t v = (uint32_t)R.hold & (k == 32 ? 0xffffffffu : ((1u << k) - 1));
  R.hold >>= k;
  R.bits -= k;
  return v;
}
static __device__ __forceinline__ void zs_lr_align(zs_lane_reader& R) {
  const uint32_t d = R.bits & 7u;
  R.hold >>= d;
  R.bits -= d;
}

// decode one Huffman symbol with a zlib table (root `rbits`); returns the final entry
static __device__ __forceinline__ zcode zs_lane_decode(zs_lane_reader& R, const zcode* t, uint32_t rbits) {
  if (R.bits < 32) zs_lr_fill(R);
  zcode here = t[(uint32_t)R.hold & ((1u << rbits) - 1)];
  if (C_OP(here) && (C_OP(here) & 0xf0) == 0) {  // second-level table
    const uint32_t rb = C_BITS(here);
    const zcode last = here;
    here = t[C_VAL(last) + (((uint32_t)R.hold & ((1u << (rb + C_OP(last))) - 1)) >> rb)];
    R.hold >>= rb;
    R.bits -= rb;
  }
  R.hold >>= C_BITS(here);
  R.bits -= C_BITS(here);
  return here;
}

// LDS root tables of one lane: 8-bit lit/len and 6-bit distance roots, u16
// entries (code length << 12 | symbol), 0 = code longer than the root (the lane
// then decodes with its zlib table in HBM).  640 B per lane: four 64-lane
// workgroups fill a CU's 160 KB.
#define ZS_LROOT 8u
#define ZS_DROOT 6u
struct zs_lane_lds {
  uint16_t lit[1u << ZS_LROOT];
  uint16_t dist[1u << ZS_DROOT];
};

static __device__ void zs_lane_root(uint16_t* tab, uint32_t rbits, const uint16_t* lens, uint32_t n) {
  uint32_t count[16], next[16];
  for (uint32_t l = 0; l < 16; l++) count[l] = 0;
  for (uint32_t i = 0; i < n; i++) count[lens[i]]++;
  count[0] = 0;
  uint32_t code = 0;
  for (uint32_t l = 1; l < 16; l++) {  // canonical first codes (RFC 1951 3.2.2)
    code = (code + count[l - 1]) << 1;
    next[l] = code;
  }
  for (uint32_t k = 0; k < (1u << rbits); k++) tab[k] = 0;
  for (uint32_t sym = 0; sym < n; sym++) {
    const uint32_t l = lens[sym];
    if (l == 0) continue;
    const uint32_t c = next[l]++;
    if (l > rbits) continue;
    const uint32_t r = __builtin_bitreverse32(c) >> (32 - l);  // the stream sends codes MSB first
    for (uint32_t k = r; k < (1u << rbits); k += 1u << l) tab[k] = (uint16_t)((l << 12) | sym);
  }
}

// a root-table symbol as the zlib table entry the decoder consumes (zs_lbase /
// zs_dbase's ops: 16 + extra bits, deflate64 128 + extra bits)
static __device__ __forceinline__ zcode zs_lit_entry(uint32_t sym, bool d64) {
  if (sym < 256) return zpack(0, 0, sym);
  if (sym == 256) return zpack(32 + 64, 0, 0);
  const uint32_t c = sym - 257;  // length codes: base / extra bits (inflate/constants.ts:8-23)
  const uint32_t f = d64 ? 128u : 16u;
  if (c < 8) return zpack(f, 0, c + 3);
  if (c == 28) return d64 ? zpack(128 + 16, 0, 3) : zpack(16, 0, 258);  // deflate64: 3 + 16 extra bits
  const uint32_t x = (c >> 2) - 1;
  return zpack(f + x, 0, ((4u | (c & 3u)) << x) + 3u);
}
static __device__ __forceinline__ zcode zs_dist_entry(uint32_t d, bool d64) {
  const uint32_t f = d64 ? 128u : 16u;
  if (d < 4) return zpack(f, 0, d + 1);
  const uint32_t x = (d >> 1) - 1;  // codes 30/31 (deflate64 only): 32769 / 49153 + 14 extra bits
  return zpack(f + x, 0, ((2u | (d & 1u)) << x) + 1u);
}

__global__ __launch_bounds__(64) void zs_k_inflate_lane(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint32_t* __restrict__ out_cap, int wbits, uint32_t n_members,
                                                        zs_lane_tabs* __restrict__ tabs, zs_lane_res* __restrict__ res,
                                                        uint32_t* __restrict__ lens_out, int flags) {
  extern __shared__ zs_lane_lds LL[];  // blockDim.x entries
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_members) return;
  zs_lane_tabs& T = tabs[s];
  zs_lane_lds& F = LL[threadIdx.x];
  zs_lane_reader R;
  R.src = in + in_off[s];
  R.n = in_len[s];
  R.pos = 0;
  R.hold = 0;
  R.bits = 0;
  R.pf = zs_lr_load4(R, 0);
  uint8_t* dst = out + out_off[s];
  // This path decodes a member in one go, without the stream layer's call
  // boundaries.  A member whose input fits one 32 KiB sub-chunk and whose
  // output fits one 64 KiB output buffer is decoded by ONE inflate() call of
  // the reference (streams.ts:6-7,78-93) that never copies from the window, so
  // the window-wrap behaviour (ZS_INF_REF_WRAP) cannot arise; any other member
  // takes the exact path, which emulates the calls.
  // deflate64 members never reach inflate_fast in the reference (inflate.ts:841),
  // so they carry no call-boundary behaviour and decode here at any size.
  const bool d64 = wbits == -16;
  const bool ref_wrap = (flags & ZS_INF_REF_WRAP) != 0 && !d64;
  const uint32_t cap = ref_wrap ? min(out_cap[s], 65536u) : out_cap[s];
  const uint32_t lmask = d64 ? 31u : 15u;  // length extra-bit mask (inflate.ts:891)
  uint32_t total = 0;
  zs_lane_res r = {1u, 0u, 0u, 0u};
  const int wrap = wbits < 0 ? 0 : (wbits >> 4) + 5;  // inflate.ts:152-160
  bool bail = ref_wrap && R.n > 32768u;  // several sub-chunks: exact path
  // ---- wrapper header (inflate.ts:377-580): plain zlib / gzip headers only
  if (!bail && wrap) {
    const uint32_t b0 = zs_lr_take(R, 8), b1 = zs_lr_take(R, 8);
    if ((wrap & 2) && b0 == 0x1f && b1 == 0x8b) {
      const uint32_t cm = zs_lr_take(R, 8), flg = zs_lr_take(R, 8);
      zs_lr_take(R, 32);  // MTIME
      zs_lr_take(R, 16);  // XFL, OS
      if (cm != 8 || flg != 0) bail = true;  // FEXTRA / FNAME / FCOMMENT / FHCRC / reserved: exact path
    } else if (wrap & 1) {
      if (((b0 << 8) | b1) % 31 || (b0 & 15) != 8 || (b0 >> 4) + 8 > 15 || (b1 & 0x20)) bail = true;
    } else {
      bail = true;  // "incorrect header check"
    }
  }
  // ---- blocks
  bool last = false;
  while (!bail && !last) {
    last = zs_lr_take(R, 1) != 0;
    const uint32_t type = zs_lr_take(R, 2);
    const zcode* lt;
    const zcode* dt;
    uint32_t lbits, dbits;
    if (type == 0) {  // stored (inflate.ts:615-660)
      zs_lr_align(R);
      const uint32_t len = zs_lr_take(R, 16), nlen = zs_lr_take(R, 16);
      if (len != (nlen ^ 0xffffu) || zs_lr_over(R) || total + len > cap) { bail = true; break; }
      for (uint32_t i = 0; i < len; i++) dst[total + i] = (uint8_t)zs_lr_take(R, 8);
      total += len;
      if (zs_lr_over(R)) { bail = true; break; }
      continue;
    }
    if (type == 1) {  // fixed tables (inflate.ts:218-280)
      uint32_t sym, used;
      for (sym = 0; sym < 144; sym++) T.lens[sym] = 8;
      for (; sym < 256; sym++) T.lens[sym] = 9;
      for (; sym < 280; sym++) T.lens[sym] = 7;
      for (; sym < 288; sym++) T.lens[sym] = 8;
      lbits = 9;
      zs_inflate_table(LENS, T.lens, 288, T.codes, &lbits, T.work, d64, &used);
      for (sym = 0; sym < 32; sym++) T.lens[sym] = 5;
      dbits = 5;
      zs_inflate_table(DISTS, T.lens, 32, T.codes + used, &dbits, T.work, d64, &sym);
      lt = T.codes;
      dt = T.codes + used;
      for (sym = 0; sym < 288; sym++) T.lens[sym] = sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8;
      zs_lane_root(F.lit, ZS_LROOT, T.lens, 286);  // 286/287 stay out of the root: invalid codes decode via T
      for (sym = 0; sym < 30; sym++) T.lens[sym] = 5;
      zs_lane_root(F.dist, ZS_DROOT, T.lens, d64 ? 32 : 30);  // deflate: 30/31 likewise
    } else if (type == 2) {  // dynamic (inflate.ts:662-836)
      const uint32_t nlen = zs_lr_take(R, 5) + 257, ndist = zs_lr_take(R, 5) + 1, ncode = zs_lr_take(R, 4) + 4;
      if (nlen > 286 || (!d64 && ndist > 30)) { bail = true; break; }
      uint32_t i;
      for (i = 0; i < ncode; i++) T.lens[ZS_BL_ORDER[i]] = (uint16_t)zs_lr_take(R, 3);
      for (; i < 19; i++) T.lens[ZS_BL_ORDER[i]] = 0;
      uint32_t cbits = 7, used;
      if (zs_inflate_table(CODES, T.lens, 19, T.codes, &cbits, T.work, d64, &used)) { bail = true; break; }
      i = 0;
      while (i < nlen + ndist) {
        const zcode here = zs_lane_decode(R, T.codes, cbits);
        const uint32_t v = C_VAL(here);
        if (v < 16) { T.lens[i++] = (uint16_t)v; continue; }
        uint32_t rep, val = 0;
        if (v == 16) {
          if (i == 0) { bail = true; break; }
          val = T.lens[i - 1];
          rep = 3 + zs_lr_take(R, 2);
        } else if (v == 17) {
          rep = 3 + zs_lr_take(R, 3);
        } else {
          rep = 11 + zs_lr_take(R, 7);
        }
        if (i + rep > nlen + ndist) { bail = true; break; }
        while (rep--) T.lens[i++] = (uint16_t)val;
      }
      if (bail || zs_lr_over(R) || T.lens[256] == 0) { bail = true; break; }
      lbits = 9;
      uint32_t lused, dused;
      if (zs_inflate_table(LENS, T.lens, nlen, T.codes, &lbits, T.work, d64, &lused)) { bail = true; break; }
      dbits = 6;
      if (zs_inflate_table(DISTS, T.lens + nlen, ndist, T.codes + lused, &dbits, T.work, d64, &dused)) {
        bail = true;
        break;
      }
      lt = T.codes;
      dt = T.codes + lused;
      zs_lane_root(F.lit, ZS_LROOT, T.lens, nlen);
      zs_lane_root(F.dist, ZS_DROOT, T.lens + nlen, ndist);
    } else {
      bail = true;  // "invalid block type"
      break;
    }
    // symbols (inffast.ts:5-228 semantics, without the call boundaries)
    for (;;) {
      if (R.bits < 32) zs_lr_fill(R);
      zcode here;
      const uint32_t fe = F.lit[(uint32_t)R.hold & ((1u << ZS_LROOT) - 1)];
      if (fe >> 12) {
        R.hold >>= fe >> 12;
        R.bits -= fe >> 12;
        here = zs_lit_entry(fe & 0x1ffu, d64);
      } else {
        here = zs_lane_decode(R, lt, lbits);
      }
      uint32_t op = C_OP(here);
      if (op == 0) {
        if (total >= cap) { bail = true; break; }
        dst[total++] = (uint8_t)C_VAL(here);
        continue;
      }
      if (op & 32) break;                   // end of block
      if (op & 64) { bail = true; break; }  // "invalid literal/length code"
      uint32_t len = C_VAL(here) + zs_lr_take(R, op & lmask);
      if (R.bits < 32) zs_lr_fill(R);
      const uint32_t de = F.dist[(uint32_t)R.hold & ((1u << ZS_DROOT) - 1)];
      if (de >> 12) {
        R.hold >>= de >> 12;
        R.bits -= de >> 12;
        here = zs_dist_entry(de & 0x1fu, d64);
      } else {
        here = zs_lane_decode(R, dt, dbits);
      }
      op = C_OP(here);
      if (op & 64) { bail = true; break; }  // "invalid distance code"
      const uint32_t dist = C_VAL(here) + zs_lr_take(R, op & 15u);
      if (dist > total || total + len > cap) { bail = true; break; }  // too far back / capacity
      const uint8_t* from = dst + total - dist;
      uint8_t* to = dst + total;
      if (dist >= 8) {  // 8 independent loads, then 8 stores: one memory round trip per 8 bytes
        for (uint32_t i = 0; i < len; i += 8) {
          uint8_t b[8];
#pragma unroll
          for (int k = 0; k < 8; k++) b[k] = i + k < len ? from[i + k] : 0;
#pragma unroll
          for (int k = 0; k < 8; k++)
            if (i + k < len) to[i + k] = b[k];
        }
      } else {  // overlapping copy: the source is being written
        for (uint32_t i = 0; i < len; i++) to[i] = from[i];
      }
      total += len;
    }
    if (zs_lr_over(R)) bail = true;
  }
  // ---- trailer (inflate.ts:1006-1036)
  if (!bail && wrap) {
    zs_lr_align(R);
    const uint32_t a = zs_lr_take(R, 32);
    if (wrap & 2 && !(wrap & 1)) {  // gzip: crc32 LE, then ISIZE LE
      r.want = a;
      const uint32_t isize = zs_lr_take(R, 32);
      if (isize != total) bail = true;
    } else {
      r.want = __builtin_bswap32(a);  // zlib: adler32 big-endian
    }
    if (zs_lr_over(R)) bail = true;
  }
  if (!bail) {
    r.bail = 0;
    r.out_len = total;
    r.consumed = (uint32_t)((zs_lr_bitpos(R) + 7u) >> 3);
  }
  res[s] = r;
  lens_out[s] = r.out_len;  // for the checksum pass over the decoded bytes
}

size_t zs_inflate_lane_scratch_bytes() { return sizeof(zs_lane_tabs); }
size_t zs_inflate_lane_lds_bytes() { return sizeof(zs_lane_lds); }

// checksum of the decoded output against the trailer: a mismatch sends the member to the exact path
__global__ void zs_k_inflate_lane_verify(zs_lane_res* __restrict__ res, const uint32_t* __restrict__ check,
                                         uint32_t n) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n && res[s].bail == 0 && res[s].want != check[s]) res[s].bail = 1;
}
