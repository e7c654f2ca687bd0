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
  uint32_t fin;  // inflate_fast's pulled bytes (member offset); its bit count is 8 fin - the bits consumed
  __device__ __forceinline__ void init() {
    B = 0;
    wn = 0;
    wh = 0;
    cend = 32768u;
    fast = 0;
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
    fast = 0;
  }
  // inflate_fast pulls whole bytes until it holds `need` bits past bit position pos: with its bit count
  // 8 fin - pos, that is fin = max(fin, ceil((pos + need) / 8))
  __device__ __forceinline__ void pull_to(PT pos_plus_need) {
    fin = max(fin, (uint32_t)((pos_plus_need + 7u) >> 3));
  }
  // a symbol with bits [sb, sb + l1 + e1 + l2 + e2) writing len bytes at o;
  // true iff inflate_fast runs it whole
  // (the common case -- inside the current call's sub-chunk and buffer --
  // skips the boundary logic)
  __device__ __forceinline__ bool symbol(PT sb, uint32_t o, uint32_t len, uint32_t l1, uint32_t e1, uint32_t l2,
                                         uint32_t e2, bool eob) {
    if (__builtin_expect(o < B + 65536u && sb + l1 + e1 + l2 + e2 <= (PT)8u * cend, 1))
      return in_call(sb, o, len, l1, e1, l2, e2, eob);
    if (o > B + 65536u) end_call(B + 65536u);  // the copy before filled the buffer
    while (sb >= (PT)8u * cend) {  // sub-chunks that ended before the symbol
      end_call(o);
      cend += 32768u;
    }
    if (sb + l1 + e1 + l2 + e2 > (PT)8u * cend) {  // crosses the sub-chunk's end: the next call's slow path
      end_call(o);
      cend += 32768u;
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
      if (cend - pulled >= 6u && B + 65536u - o >= 258u) {
        fast = 1;
        fin = pulled;
      } else {
        return false;
      }
    }
    // pulls: 15 bits at the code (sb), then for a length / distance pair e1 at
    // sb + l1, 15 at sb + l1 + e1 and e2 at sb + l1 + e1 + l2 -- whose largest
    // requirement is one of the last two
    if (eob) {
      pull_to(sb + 15u);
      fast = 0;
      return true;
    }
    if (len > 1u || l2) {
      const PT d = sb + l1 + e1;
      pull_to(max(d + 15u, d + l2 + e2));
    } else {
      pull_to(sb + 15u);
    }
    if (!(fin < cend - 5u && o + len < B + 65536u - 257u)) fast = 0;  // the fast loop's condition
    return true;
  }
  // a stored block's len bytes at input byte in, output o (the COPY state: the slow path)
  __device__ __forceinline__ void stored(uint32_t in, uint32_t o, uint32_t len) {
    if (o > B + 65536u) end_call(B + 65536u);
    while (len) {
      while (in >= cend) {
        end_call(o);
        cend += 32768u;
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
