"""Statistics of the segmented decode's records (zs_debug_fetch 17/18/19/21)
after decoding n members: spans per member, chain length per span, piece bits,
merged pieces, the plan's pieces.  python3 tools/dbg/seg_stats.py [kind] [n] [size] [level] [fmt]"""
import ctypes
import os
import struct
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus  # noqa: E402
import oracle  # noqa: E402

BLK = 64  # sizeof(zs_seg_blk)
LS = 4 * 19


def fetch(eng, what, nbytes):
    buf = ctypes.create_string_buffer(nbytes)
    got = eng._L.zs_debug_fetch(eng._ctx, what, 0, buf, nbytes)
    return buf.raw[:got]


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "text"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 262144
    lv = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    fmt = sys.argv[5] if len(sys.argv) > 5 else "deflate-raw"
    import torch
    torch.cuda.init()
    import zsamd
    eng = zsamd.Engine(0)
    for kv in sys.argv[6:]:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    srcs = [corpus.make({"kind": kind, "n": size, "seed": corpus.stream_seed(i)}) for i in range(n)]
    comps = [oracle.compress(s, lv, fmt)[1] for s in srcs]
    got = eng.decompress_batch_raw(comps, fmt, [size] * n)
    print("seg count", eng.last_seg_count(), "ok", sum(g[3] == s for g, s in zip(got, srcs)), "of", n,
          "comp bytes", [len(c) for c in comps[:4]])
    B = fetch(eng, 17, BLK * 4096)
    nb = len(B) // BLK
    spans = []
    for b in range(nb):
        v = struct.unpack_from("<16I", B, BLK * b)
        if v[0] != 0xffffffff and v[0] < n:
            spans.append((b,) + v)
    Lr = fetch(eng, 18, LS * 64 * (max(s[0] for s in spans) + 1))
    per_m = Counter(s[1] for s in spans)
    print("spans per member", sorted(per_m.values())[:8], "...", "total", len(spans))
    chain = Counter()
    bits = []
    merged = 0
    for s in spans:
        b = s[0]
        flags, nl, S = s[6], s[11], s[12]
        np_ = 0
        for l in range(64):
            v = struct.unpack_from("<19I", Lr, LS * (64 * b + l))
            if v[0] != 0xffffffff:
                np_ += 1
                bits.append(v[1] - v[0])
                if not (v[18] & 1):
                    merged += 1
        chain[(np_, nl, flags)] += 1
    print("(pieces, nl, flags) per span:", chain.most_common(12))
    bits.sort()
    print("piece bits: n %d median %d p90 %d max %d; not decoded (merged / unplaced) %d" % (
        len(bits), bits[len(bits) // 2], bits[len(bits) * 9 // 10], bits[-1], merged))
    M = fetch(eng, 19, 32 * n)
    print("members (bad, total, consumed, want, npieces, nalloc):", [struct.unpack_from("<6I", M, 32 * m) for m in range(min(n, 4))])


if __name__ == "__main__":
    main()
