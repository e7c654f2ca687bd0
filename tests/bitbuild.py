"""Hand-built deflate / deflate64 streams (fixed-Huffman blocks, RFC 1951
3.2.6) for edge cases no encoder here produces: deflate64 length code 285
with its 16 extra bits (inflate/constants.ts:12,28: base 3, up to 65,538
bytes) and the 32,769 / 49,153 distance codes 30/31 (constants.ts:34).

A symbol list is [("lit", byte) | ("copy", length, distance) | ...]; expand()
is the plain LZ77 meaning of the list (the expected output), build() the bits."""


class _Bits:
    def __init__(self):
        self.acc, self.n, self.out = 0, 0, bytearray()

    def put(self, v, k):  # k bits of v, LSB first (RFC 1951 3.1.1)
        self.acc |= (v & ((1 << k) - 1)) << self.n
        self.n += k
        while self.n >= 8:
            self.out.append(self.acc & 0xff)
            self.acc >>= 8
            self.n -= 8

    def code(self, c, k):  # a Huffman code: most significant bit first
        self.put(int(format(c, "0%db" % k)[::-1], 2), k)

    def bytes(self):
        return bytes(self.out) + (bytes([self.acc]) if self.n else b"")


def _fixed_lit(b, sym):
    if sym < 144:
        b.code(0x30 + sym, 8)
    elif sym < 256:
        b.code(0x190 + sym - 144, 9)
    elif sym < 280:
        b.code(sym - 256, 7)
    else:
        b.code(0xc0 + sym - 280, 8)


# (base, extra bits) per length code 257.. and distance code 0..; deflate64
# differs in length code 285 (3 + 16 extra bits) and adds distance codes 30/31
_LEN = [(3, 0), (4, 0), (5, 0), (6, 0), (7, 0), (8, 0), (9, 0), (10, 0), (11, 1), (13, 1), (15, 1), (17, 1),
        (19, 2), (23, 2), (27, 2), (31, 2), (35, 3), (43, 3), (51, 3), (59, 3), (67, 4), (83, 4), (99, 4),
        (115, 4), (131, 5), (163, 5), (195, 5), (227, 5), (258, 0)]
_DIST = [(1, 0), (2, 0), (3, 0), (4, 0), (5, 1), (7, 1), (9, 2), (13, 2), (17, 3), (25, 3), (33, 4), (49, 4),
         (65, 5), (97, 5), (129, 6), (193, 6), (257, 7), (385, 7), (513, 8), (769, 8), (1025, 9), (1537, 9),
         (2049, 10), (3073, 10), (4097, 11), (6145, 11), (8193, 12), (12289, 12), (16385, 13), (24577, 13),
         (32769, 14), (49153, 14)]


def _len_code(n, d64):
    if d64 and n > 257:  # only code 285 reaches past 257 in deflate64
        return 28, n - 3, 16
    if not d64 and n == 258:
        return 28, 0, 0
    for i in range(27, -1, -1):
        base, x = _LEN[i]
        if base <= n < base + (1 << x):
            return i, n - base, x
    raise ValueError(n)


def _dist_code(d):
    for i in range(len(_DIST) - 1, -1, -1):
        base, x = _DIST[i]
        if base <= d < base + (1 << x):
            return i, d - base, x
    raise ValueError(d)


def build(symbols, d64=True):
    """One final fixed-Huffman block holding the symbols."""
    b = _Bits()
    b.put(1, 1)  # BFINAL
    b.put(1, 2)  # BTYPE = 01 (fixed)
    for s in symbols:
        if s[0] == "lit":
            _fixed_lit(b, s[1])
        else:
            _, n, d = s
            i, ev, ex = _len_code(n, d64)
            _fixed_lit(b, 257 + i)
            b.put(ev, ex)
            j, dv, dx = _dist_code(d)
            b.code(j, 5)
            b.put(dv, dx)
    _fixed_lit(b, 256)
    return b.bytes()


def expand(symbols):
    out = bytearray()
    for s in symbols:
        if s[0] == "lit":
            out.append(s[1])
        else:
            _, n, d = s
            for _ in range(n):
                out.append(out[-d])
    return bytes(out)


def long_copies():
    """deflate64 members with copies longer than the 64 KiB window: lengths
    65,537 / 65,538 at distances that do not divide 65,536, and a 49,153+
    distance behind them."""
    cases = []
    lits = [("lit", c) for c in b"abc"]
    cases.append(lits + [("copy", 65538, 3)])
    seed = [("lit", (i * 37 + 11) & 0xff) for i in range(300)]
    cases.append(seed + [("copy", 65537, 299), ("copy", 1000, 50000)])
    cases.append([("lit", c) for c in b"xy"] + [("copy", 65538, 2), ("copy", 65538, 65536), ("copy", 300, 7)])
    return [(build(s, True), expand(s)) for s in cases]
