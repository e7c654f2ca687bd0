"""CPU model of the segmented decode's call-state plan (inflate_seg.hip).

The reference decodes a DecompressionStream in inflate() calls (32 KiB input
sub-chunks, 64 KiB output buffers, streams.ts:78-93) and its inflate_fast
copies some bytes from the call's first output bytes instead of the window
(inffast.ts:127-147).  The GPU decodes a member in PIECES (block starts and
mid-block sync points) that run in parallel, so each piece needs the call state
at its start.  This model checks the plan that gives it:

  * the call state evolves only at sub-chunk crossing events (the first symbol
    whose bits end past 262144 k) and buffer fills (the first symbol whose
    output position reaches B + 65536); both are known from each piece's
    (output count, events, last symbol length) alone;
  * a piece that does not start within 144 bits before a sub-chunk end may
    start with any `fast` value: the flag only matters in the near zones, and
    in the output zone (> B + 65020) no copy can reach before the call start;
  * a stored block is one piece: the reference's COPY state (inflate.ts:645-660)
    ends calls inside it at sub-chunk ends and buffer fills, which the plan
    replays from its input offset and length alone (zs_refcalls_t::stored).

It decodes members serially (symbols with their bit fields), replays the
reference's bookkeeping (a transcription of zs_refcalls.h) over the whole
member, then per piece from the planned state, and compares every copy's
window-wrap decision; the serial expansion is also compared with the oracle
(reference_bugs = 1), i.e. the reference's own semantics.

  python3 tools/emu/emu_seg.py [n_members]
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import corpus  # noqa: E402
import oracle  # noqa: E402

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
BLO = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self, data):
        self.d = bytes(data) + bytes(8)

    def get(self, pos, k):
        b = pos >> 3
        v = int.from_bytes(self.d[b:b + (((pos & 7) + k + 7) >> 3)], "little")
        return (v >> (pos & 7)) & ((1 << k) - 1)


def table(lens):
    bl = [0] * 16
    for x in lens:
        if x:
            bl[x] += 1
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, x in enumerate(lens):
        if x:
            c = nxt[x]
            nxt[x] += 1
            t[(x, int(format(c, "0%db" % x)[::-1], 2))] = s
    return t, max(lens)


def dec(br, pos, t):
    tab, m = t
    for x in range(1, m + 1):
        s = tab.get((x, br.get(pos, x)))
        if s is not None:
            return s, x
    raise ValueError("bad code")


def decode(data):
    """Serial decode of a raw deflate member: symbols as dicts (sb, o, len, dist,
    l1, e1, l2, e2, eob, blk; a stored block is one symbol with its bytes in raw)
    and the block starts (bit of the block header)."""
    br = Bits(data)
    pos, o, syms, blocks = 0, 0, [], []
    while True:
        blocks.append((pos, len(syms)))
        last = br.get(pos, 1)
        typ = br.get(pos + 1, 2)
        pos += 3
        if typ == 0:
            pos = (pos + 7) & ~7
            n = br.get(pos, 16)
            assert n == br.get(pos + 16, 16) ^ 0xFFFF
            pos += 32
            raw = data[pos >> 3:(pos >> 3) + n]
            syms.append(dict(sb=pos, o=o, len=n, dist=0, l1=0, e1=0, l2=0, e2=0, eob=False, blk=len(blocks) - 1,
                             stored=True, raw=raw))
            o += n
            pos += 8 * n
            if last:
                return syms, blocks, pos
            continue
        if typ == 1:
            lens = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
            lt, dt = table(lens), table([5] * 30)
        else:
            hlit, hdist, hc = br.get(pos, 5) + 257, br.get(pos + 5, 5) + 1, br.get(pos + 10, 4) + 4
            pos += 14
            cl = [0] * 19
            for i in range(hc):
                cl[BLO[i]] = br.get(pos, 3)
                pos += 3
            ct = table(cl)
            lens = []
            while len(lens) < hlit + hdist:
                s, x = dec(br, pos, ct)
                pos += x
                if s < 16:
                    lens.append(s)
                elif s == 16:
                    r = 3 + br.get(pos, 2); pos += 2; lens += [lens[-1]] * r
                elif s == 17:
                    r = 3 + br.get(pos, 3); pos += 3; lens += [0] * r
                else:
                    r = 11 + br.get(pos, 7); pos += 7; lens += [0] * r
            lt, dt = table(lens[:hlit]), table(lens[hlit:])
        while True:
            sb = pos
            s, l1 = dec(br, pos, lt)
            pos += l1
            if s < 256:
                syms.append(dict(sb=sb, o=o, len=1, dist=0, l1=l1, e1=0, l2=0, e2=0, eob=False, blk=len(blocks) - 1))
                o += 1
                continue
            if s == 256:
                syms.append(dict(sb=sb, o=o, len=0, dist=0, l1=l1, e1=0, l2=0, e2=0, eob=True, blk=len(blocks) - 1))
                break
            c = s - 257
            e1 = LEXT[c]
            n = LBASE[c] + br.get(pos, e1)
            pos += e1
            d, l2 = dec(br, pos, dt)
            pos += l2
            e2 = DEXT[d]
            dist = DBASE[d] + br.get(pos, e2)
            pos += e2
            syms.append(dict(sb=sb, o=o, len=n, dist=dist, l1=l1, e1=e1, l2=l2, e2=e2, eob=False,
                             blk=len(blocks) - 1))
            o += n
        if last:
            return syms, blocks, pos


class Calls:
    """zs_refcalls_t (zs_refcalls.h), transcribed."""

    def __init__(self, B=0, wn=0, wh=0, cend=32768, fast=0):
        self.B, self.wn, self.wh, self.cend, self.fast = B, wn, wh, cend, fast

    def state(self):
        return (self.B, self.wn, self.wh, self.cend)

    def next_chunk(self):
        self.cend += 32768

    def end_call(self, at):
        produced = at - self.B
        if produced >= 32768:
            self.wn, self.wh = 0, 32768
        elif produced:
            d = min(32768 - self.wn, produced)
            rest = produced - d
            if rest:
                self.wn, self.wh = rest, 32768
            else:
                self.wn += d
                if self.wn == 32768:
                    self.wn = 0
                self.wh = min(self.wh + d, 32768)
        self.B = at
        self.fast = 0

    def symbol(self, sb, o, n, l1, e1, l2, e2, eob):
        sfar, ofar = 8 * self.cend - 96, self.B + 65536 - 516
        if sb < sfar and o < ofar:
            self.fast = 0 if eob else 1
            return True
        end = sb + l1 + e1 + l2 + e2
        if o < self.B + 65536 and end <= 8 * self.cend:
            return self.in_call(sb, o, n, l1, e1, l2, e2, eob)
        if o > self.B + 65536:
            self.end_call(self.B + 65536)
        while sb >= 8 * self.cend:
            self.end_call(o)
            self.next_chunk()
        if end > 8 * self.cend:
            self.end_call(o)
            self.next_chunk()
            return False
        if o >= self.B + 65536:
            self.end_call(self.B + 65536)
            return False
        return self.in_call(sb, o, n, l1, e1, l2, e2, eob)

    def in_call(self, sb, o, n, l1, e1, l2, e2, eob):
        if not self.fast:
            pulled = (sb + 7) >> 3
            if not (self.cend - pulled >= 6 and self.B + 65536 - o >= 258):
                return False
            self.fast = 1
        if eob:
            self.fast = 0
            return True
        d = sb + l1 + e1
        req = max(d + 15, d + l2 + e2) if (n > 1 or l2) else sb + 15
        if not (req + 7 < 8 * (self.cend - 5) and o + n < self.B + 65536 - 257):
            self.fast = 0
        return True

    def wrap(self, o, n, dist):
        if dist <= o - self.B or self.wn == 0:
            return 0
        op2 = dist - (o - self.B)
        if self.wn >= op2:
            return 0
        op3 = op2 - self.wn
        return n - op3 if (op3 < n and self.wn >= n - op3) else 0

    def stored(self, at, o, n):
        if o > self.B + 65536:
            self.end_call(self.B + 65536)
        while n == 0 and self.cend < at:  # (the plan's form: an empty block takes its header's crossings)
            self.end_call(o)
            self.next_chunk()
        while n:
            while at >= self.cend:
                self.end_call(o)
                self.next_chunk()
            if o >= self.B + 65536:
                self.end_call(self.B + 65536)
            take = min(n, self.cend - at, self.B + 65536 - o)
            at, o, n = at + take, o + take, n - take


def replay(syms, C, lo, hi):
    """wrap tails of symbols lo..hi-1 from state C"""
    tails = {}
    for i in range(lo, hi):
        s = syms[i]
        if s.get("stored"):
            C.stored(s["sb"] >> 3, s["o"], s["len"])
            continue
        run = C.symbol(s["sb"], s["o"], s["len"], s["l1"], s["e1"], s["l2"], s["e2"], s["eob"])
        if run and s["dist"]:
            t = C.wrap(s["o"], s["len"], s["dist"])
            if t:
                tails[i] = (t, C.B)
    return tails


def expand(syms, tails):
    out = bytearray()
    for i, s in enumerate(syms):
        if s["eob"]:
            continue
        if s.get("stored"):
            out += s["raw"]
            continue
        if not s["dist"]:
            out.append(s["lit"])
            continue
        t, B = tails.get(i, (0, 0))
        for k in range(s["len"] - t):
            out.append(out[-s["dist"]])
        for k in range(t):
            out.append(out[B + k])
    return bytes(out)


def events(syms):
    """crossing event k: the first symbol whose end bit is past 262144 k (blocks
    are contiguous in bits except for their headers: a symbol starting past the
    boundary after a header is the event too); a stored block takes the
    boundaries before its end itself (Calls.stored), no events"""
    ev, k = [], 1
    for i, s in enumerate(syms):
        end = s["sb"] + (8 * s["len"] if s.get("stored") else s["l1"] + s["e1"] + s["l2"] + s["e2"])
        while end > 262144 * k:
            if not s.get("stored"):
                ev.append((k, i))
            k += 1
    return ev


def plan(syms, blocks, starts):
    """Phase B: the call state at each piece start (symbol indices `starts`, the
    first one 0), from the pieces' events, output offsets and last lengths;
    unclean starts (within 144 bits before a sub-chunk end) merge into the piece
    before.  Returns [(start index, state, fast)]."""
    # the events and the stored blocks, in symbol order
    acts = sorted([(i, k) for k, i in events(syms)] + [(i, 0) for i, s in enumerate(syms) if s.get("stored")])
    blkstart = {b[1] for b in blocks}
    C = Calls()
    out = [(0, (0, 0, 0, 32768), 0)]
    ei = 0
    for j in range(1, len(starts)):
        a = starts[j]
        s = syms[a]
        O = s["o"]
        # events of symbols before the piece, each with the fills before it, and stored blocks
        while ei < len(acts) and acts[ei][0] < a:
            i = acts[ei][0]
            if acts[ei][1] == 0:
                C.stored(syms[i]["sb"] >> 3, syms[i]["o"], syms[i]["len"])
            else:
                o_e = syms[i]["o"]
                while o_e >= C.B + 65536:
                    C.end_call(C.B + 65536)
                C.end_call(o_e)
                C.next_chunk()
            ei += 1
        prev = syms[a - 1]
        o_prev = O if prev.get("stored") else prev["o"]  # = O - last_len (0 after an end of block or stored block)
        while o_prev >= C.B + 65536:
            C.end_call(C.B + 65536)
        if a not in blkstart and s["sb"] + 144 > 8 * C.cend:
            continue  # unclean: the piece before decodes this one too
        out.append((a, C.state(), 0 if a in blkstart else 1))
    return out


def check(data, ref, piece_syms, rng):
    syms, blocks, end = decode(data)
    # the literal values (for expand)
    br = Bits(data)
    # re-decode literal values cheaply: expand needs them
    full = oracle.decompress(data, "deflate-raw", cap=1 << 24, reference_bugs=False)[1]
    for s in syms:
        if not s["eob"] and not s["dist"]:
            s["lit"] = full[s["o"]]
    serial = replay(syms, Calls(), 0, len(syms))
    got = expand(syms, serial)
    assert got == ref, "serial replay != reference"
    # pieces: block starts + random mid-block starts
    starts = sorted({b[1] for b in blocks} | {i for i in range(1, len(syms)) if rng.random() < 1.0 / piece_syms
                                                and not syms[i - 1]["eob"]})
    P = plan(syms, blocks, starts)
    tails = {}
    nmerge = len(starts) - len(P)
    for j, (a, st, fast) in enumerate(P):
        b = P[j + 1][0] if j + 1 < len(P) else len(syms)
        for f in (fast, 1 - fast):  # any fast value at a clean start
            C = Calls(*st, fast=f)
            t = replay(syms, C, a, b)
            if f == fast:
                tails.update(t)
            else:
                assert t == {k: v for k, v in serial.items() if a <= k < b}, ("fast-dependent", j, a)
    assert tails == serial, "piecewise wrap decisions differ"
    return len(serial), len(P), nmerge


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    rng = random.Random(7)
    tot = [0, 0, 0]
    cases = []
    for i in range(n):
        # M-corpus members at L6 / L9 hit the window-wrap copy (short calls in
        # output: the incompressible kilobytes), T-corpus ones rarely
        kind = ["mixed", "text"][i % 2]
        size = rng.choice([262144, 200000, 500000, 70000])
        cases.append((kind, size, corpus.stream_seed(rng.randrange(4096)), rng.choice([1, 6, 9, 6])))
    for kind, size, seed, lv in cases:
        src = corpus.make({"kind": kind, "n": size, "seed": seed})
        c = oracle.compress(src, lv, "deflate-raw")[1]
        ref = oracle.decompress(c, "deflate-raw", cap=size, reference_bugs=True)[1]
        for ps in (40, 300, 2000):
            w, npieces, nm = check(c, ref, ps, rng)
            tot[0] += w
            tot[1] += npieces
            tot[2] += nm
        print(kind, size, "L%d" % lv, "wraps", w, "ref!=src", ref != src, flush=True)
    print("ok: wrap copies %d, pieces %d, merged starts %d" % tuple(tot))


if __name__ == "__main__":
    main()
