# Share of symbol steps of C3's members (M-corpus 64 KiB, L6) whose copy reaches further back than a per-lane
# history of a given size, and the chance that some lane of a 64-lane wave takes such a copy in a step
# (profiles/r06/c3/far_copy_model.txt).  CPU only: python's zlib 1.2.11 gives the reference's bytes at L6.
import sys, zlib
sys.path.insert(0, "zlib-streams-ts_amd")
import zsamd

LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LE = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DB = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
      6145, 8193, 12289, 16385, 24577]
DE = [0, 0, 0, 0] + [k // 2 for k in range(2, 28)]


def build(lens):
    bl = [0] * 16
    for l in lens:
        if l:
            bl[l] += 1
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, l in enumerate(lens):
        if l:
            t[(l, nxt[l])] = s
            nxt[l] += 1
    return t


class BR:
    def __init__(self, d):
        self.d, self.p = d, 0

    def bits(self, n):
        v = 0
        for i in range(n):
            v |= ((self.d[self.p >> 3] >> (self.p & 7)) & 1) << i
            self.p += 1
        return v


def dec(br, t):
    c = l = 0
    while True:
        c = (c << 1) | br.bits(1)
        l += 1
        if (l, c) in t:
            return t[(l, c)]


def dists_of(data):
    br, out = BR(data), []
    while True:
        last, typ = br.bits(1), br.bits(2)
        if typ == 0:
            br.p = (br.p + 7) & ~7
            ln = br.bits(16)
            br.bits(16)
            br.p += 8 * ln
            if last:
                return out
            continue
        if typ == 1:
            ll, dl = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8, [5] * 30
        else:
            hl, hd, hc = br.bits(5) + 257, br.bits(5) + 1, br.bits(4) + 4
            order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
            cl = [0] * 19
            for i in range(hc):
                cl[order[i]] = br.bits(3)
            ct, lens = build(cl), []
            while len(lens) < hl + hd:
                v = dec(br, ct)
                if v < 16:
                    lens.append(v)
                elif v == 16:
                    lens += [lens[-1]] * (3 + br.bits(2))
                elif v == 17:
                    lens += [0] * (3 + br.bits(3))
                else:
                    lens += [0] * (11 + br.bits(7))
            ll, dl = lens[:hl], lens[hl:]
        lt, dt = build(ll), build(dl)
        while True:
            s = dec(br, lt)
            if s < 256:
                out.append(0)
            elif s == 256:
                break
            else:
                i = s - 257
                br.bits(LE[i])
                d = dec(br, dt)
                out.append(DB[d] + br.bits(DE[d]))
        if last:
            return out


n_members = int(sys.argv[1]) if len(sys.argv) > 1 else 16
buf = bytes(zsamd.corpus("mixed", 0, n_members, 65536))
dists = []
for m in range(n_members):
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    dists += dists_of(c.compress(buf[m * 65536:(m + 1) * 65536]) + c.flush())
n = len(dists)
for th in (124, 252, 508, 1020, 2044):
    p = sum(1 for d in dists if d > th) / n
    print("dist > %5d: %.3f of symbol steps; P(some of 64 lanes) = %.4f" % (th, p, 1 - (1 - p) ** 64))
print("symbols", n, "copies", sum(1 for d in dists if d))
