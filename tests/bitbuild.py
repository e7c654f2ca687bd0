"""Hand-built deflate / deflate64 streams (fixed-Huffman blocks, RFC 1951
3.2.6) for edge cases no encoder here produces: deflate64 length code 285
with its 16 extra bits (inflate/constants.ts:12,28: base 3, up to 65,538
bytes) and the 32,769 / 49,153 distance codes 30/31 (constants.ts:34).

A symbol list is [("lit", byte) | ("copy", length, distance) | ...]; expand()
is the plain LZ77 meaning of the list (the expected output), build() the bits.
blocks() strings stored blocks (RFC 1951 3.2.4) and fixed ones into one member."""


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


def _fixed_block(b, symbols, final, d64):
    b.put(1 if final else 0, 1)  # BFINAL
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


def build(symbols, d64=True):
    """One final fixed-Huffman block holding the symbols."""
    b = _Bits()
    _fixed_block(b, symbols, True, d64)
    return b.bytes()


def blocks(parts, d64=False):
    """A member of blocks in order, the last one final: ("stored", bytes) -- BTYPE 00, the bits to the byte
    boundary, LEN, NLEN, the bytes (at most 65,535) -- ("fixed", symbols), or ("bits", block, nbits, expansion):
    one block taken verbatim from an encoder's member (its first nbits, BFINAL rewritten).  Returns (member,
    expansion)."""
    b, out = _Bits(), bytearray()
    for k, part in enumerate(parts):
        final = k + 1 == len(parts)
        if part[0] == "bits":
            _, data, nbits, exp = part
            b.put(1 if final else 0, 1)
            for i in range(1, nbits):
                b.put((data[i >> 3] >> (i & 7)) & 1, 1)
            out += exp
        elif part[0] == "stored":
            data = part[1]
            assert len(data) <= 65535
            b.put(1 if final else 0, 1)
            b.put(0, 2)
            b.put(0, (8 - b.n) & 7)
            b.put(len(data), 16)
            b.put(len(data) ^ 0xFFFF, 16)
            for x in data:
                b.put(x, 8)
            out += data
        else:
            _fixed_block(b, part[1], final, d64)
            for s in part[1]:
                if s[0] == "lit":
                    out.append(s[1])
                else:
                    for _ in range(s[1]):
                        out.append(out[-s[2]])
    return b.bytes(), bytes(out)


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


def stored_mix(rng, n, src, level0=False):
    """A member of about n output bytes: stored blocks (0 .. 65,535 bytes of src, sizes not multiples of 4) and,
    unless level0, fixed blocks between them whose copies reach back up to 32 KiB -- into the stored bytes too.
    Returns (member, expansion)."""
    parts, made, at = [], 0, 0
    while made < n:
        if level0 or rng.random() < 0.5:
            k = min(rng.choice([0, 1, 7, 999, 5003, 20001, 65535]), n - made + 1)
            parts.append(("stored", src[at % len(src):at % len(src) + k]))
            at += k
            made += len(parts[-1][1])
        else:
            syms = []
            for _ in range(rng.choice([10, 300, 4000])):
                if made < 1 or rng.random() < 0.6:
                    syms.append(("lit", src[at % len(src)]))
                    at += 1
                    made += 1
                else:  # (short copies: under 8 output bytes per input byte, as the segmented decode takes)
                    ln = rng.choice([3, 4, 9, 17, 40])
                    syms.append(("copy", ln, rng.randint(1, min(made, 32768))))
                    made += ln
            parts.append(("fixed", syms))
    return blocks(parts)
