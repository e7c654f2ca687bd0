// zs_refcalls.h -- the bookkeeping of the reference's inflate() calls for a
// deflate / zlib / gzip member decoded straight through: the wave kernel
// (inflate_wave.hip) keeps it in scalars, the lane kernel (inflate_lane.hip,
// large members) per lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// The reference's inflate() calls, for a deflate / zlib / gzip member decoded
// straight through here (bookkeeping only, no data).  The stream layer
// (streams.ts:78-93) gives each call the input left in one 32 KiB sub-chunk and
// a fresh 64 KiB output buffer; a call ends when the sub-chunk runs out (the
// symbol whose bits cross its end is finished by the next call's slow path) or
// the buffer is full.  inf_leave's updatewindow (inflate.ts:282-322,1059-1073)
// then appends the call's output to the 32 KiB window (w_next, w_have).
// inflate_fast runs a symbol iff the LEN state found >= 6 unread input bytes and
// >= 258 bytes of buffer left (inflate.ts LEN), or the fast loop went on after
// the previous symbol (inffast.ts:24, inIndex < last && outIndex < end, its
// byte refills simulated bit-exactly).  Only inflate_fast has the window-wrap
// copy (inffast.ts:127-147): when the window part of a copy wraps past
// window[w_next] and the rest (at most w_next bytes) would come from
// window[0..], the reference copies output[0..] -- the CURRENT call's buffer,
// i.e. the call's first bytes -- instead.  wrap() says whether a copy does that.
// PT: the type of bit positions (uint64_t; uint32_t for members under 512 MB)
template <typename PT>
struct zs_refcalls_t {
  uint32_t B;       // output position where the current call began
  uint32_t wn, wh;  // w_next, w_have when it began
  uint32_t cend;    // input byte where the current sub-chunk ends
  uint32_t fast;    // inside inflate_fast
  // symbols starting below both are far from the call's ends (see symbol())
  PT sfar;        // 8 cend - 96
  uint32_t ofar;  // B + 65536 - 516
  __device__ __forceinline__ void init() {
    B = 0;
    wn = 0;
    wh = 0;
    cend = 32768u;
    fast = 0;
    sfar = (PT)8u * cend - 96u;
    ofar = 65536u - 516u;
  }
  __device__ __forceinline__ void next_chunk() {
    cend += 32768u;
    sfar = (PT)8u * cend - 96u;
  }
  __device__ __forceinline__ void end_call(uint32_t at) {
    const uint32_t produced = at - B;
    if (produced >= 32768u) {
      wn = 0;
      wh = 32768u;
    } else if (produced) {
      const uint32_t d = min(32768u - wn, produced), rest = produced - d;
      if (rest) {
        wn = rest;
        wh = 32768u;
      } else {
        wn += d;
        if (wn == 32768u) wn = 0;
        wh = min(wh + d, 32768u);
      }
    }
    B = at;
    ofar = at + 65536u - 516u;
    fast = 0;
  }
  // a symbol with bits [sb, sb + l1 + e1 + l2 + e2) writing len bytes at o;
  // true iff inflate_fast runs it whole
  __device__ __forceinline__ bool symbol(PT sb, uint32_t o, uint32_t len, uint32_t l1, uint32_t e1, uint32_t l2,
                                         uint32_t e2, bool eob) {
    // Far from both ends of the call (sb + 96 bits below the sub-chunk's end, o
    // + 516 below the buffer's): the LEN state's test passes (>= 12 bytes and
    // >= 516 bytes left) and so does the fast loop's after the symbol (its
    // pulls reach at most sb + 48 bits, below 8 (cend - 5) - 7; o + len <= o +
    // 258 < B + 65279), so inflate_fast runs it and goes on unless it is the
    // end of block -- nothing else to track.
    if (__builtin_expect(sb < sfar && o < ofar, 1)) {
      fast = !eob;
      return true;
    }
    if (o < B + 65536u && sb + l1 + e1 + l2 + e2 <= (PT)8u * cend) return in_call(sb, o, len, l1, e1, l2, e2, eob);
    if (o > B + 65536u) end_call(B + 65536u);  // the copy before filled the buffer
    while (sb >= (PT)8u * cend) {  // sub-chunks that ended before the symbol
      end_call(o);
      next_chunk();
    }
    if (sb + l1 + e1 + l2 + e2 > (PT)8u * cend) {  // crosses the sub-chunk's end: the next call's slow path
      end_call(o);
      next_chunk();
      return false;
    }
    if (o >= B + 65536u) {  // the buffer is full: the next call's slow path writes it
      end_call(B + 65536u);
      return false;
    }
    return in_call(sb, o, len, l1, e1, l2, e2, eob);
  }
  __device__ __forceinline__ bool in_call(PT sb, uint32_t o, uint32_t len, uint32_t l1, uint32_t e1, uint32_t l2,
                                          uint32_t e2, bool eob) {
    if (!fast) {  // the LEN state (inflate.ts): have >= 6 && left >= 258
      const uint32_t pulled = (uint32_t)((sb + 7u) >> 3);
      if (!(cend - pulled >= 6u && B + 65536u - o >= 258u)) return false;
      fast = 1;
    }
    if (eob) {
      fast = 0;
      return true;
    }
    // inflate_fast pulls whole bytes until it holds the bits a step needs: 15 at
    // the code (sb), then for a length / distance pair e1 at sb + l1, 15 at
    // sb + l1 + e1 and e2 at sb + l1 + e1 + l2 -- the largest requirement is one
    // of the last two.  Its pulled count fin = max(fin, ceil(req / 8)) only
    // grows and passed the loop's test fin < cend - 5 at the previous step (or
    // is the LEN state's, below it), so after this step the test is this
    // step's own: ceil(req / 8) < cend - 5, i.e. req + 7 < 8 (cend - 5).
    const PT d = sb + l1 + e1;
    const PT req = (len > 1u || l2) ? max(d + 15u, d + l2 + e2) : sb + 15u;
    if (!(req + 7u < (PT)8u * (cend - 5u) && o + len < B + 65536u - 257u)) fast = 0;  // the fast loop's condition
    return true;
  }
  // a stored block's len bytes at input byte in, output o (the COPY state: the slow path)
  __device__ __forceinline__ void stored(uint32_t in, uint32_t o, uint32_t len) {
    if (o > B + 65536u) end_call(B + 65536u);
    while (len) {
      while (in >= cend) {
        end_call(o);
        next_chunk();
      }
      if (o >= B + 65536u) end_call(B + 65536u);
      const uint32_t take = min(len, min(cend - in, B + 65536u - o));
      in += take;
      o += take;
      len -= take;
    }
  }
  // the window-wrap copy (inffast.ts:127-147) for a copy inflate_fast runs: the
  // number of bytes (at the copy's end) that come from the call's first output
  // bytes instead of the window, 0 if none
  __device__ __forceinline__ uint32_t wrap(uint32_t o, uint32_t len, uint32_t dist) const {
    if (dist <= o - B || wn == 0) return 0;
    const uint32_t op2 = dist - (o - B);
    if (wn >= op2) return 0;
    const uint32_t op3 = op2 - wn;
    return (op3 < len && wn >= len - op3) ? len - op3 : 0u;
  }
};
using zs_refcalls = zs_refcalls_t<uint64_t>;
