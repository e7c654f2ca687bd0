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
#include "zs_inftab.h"

#define IN_CHUNK 32768u   // streams.ts:7
#define OUT_BUF 65536u    // streams.ts:6
#define FLUSH_AT 4096u    // ring bytes flushed to HBM per step

enum { HEAD = 0, FLAGS, TIME, OS, EXLEN, EXTRA, NAME, COMMENT, HCRC, DICTID, DICT, TYPE, TYPEDO, STORED, COPY_, COPY,
       TABLE, LENLENS, CODELENS, LEN_, LEN, LENEXT, DIST, DISTEXT, MATCH, LIT, CHECK, LENGTH, DONE, BAD };
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

// The lane-per-member fast path lives in inflate_lane.hip.

// checksum of the decoded output against the trailer: a mismatch sends the member to the exact path
__global__ void zs_k_inflate_lane_verify(zs_lane_res* __restrict__ res, const uint32_t* __restrict__ check,
                                         uint32_t n) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n && res[s].bail == 0 && res[s].want != check[s]) res[s].bail = 1;
}
