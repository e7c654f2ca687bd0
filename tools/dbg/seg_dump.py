"""Dumps the segmented decode's records (zs_debug_fetch 16..20) after decoding a
few members: per member the outcome, per block its header / lanes / end, per
lane its piece.  python3 tools/dbg/seg_dump.py [kind] [n] [level] [fmt]"""
import ctypes
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus  # noqa: E402
import oracle  # noqa: E402


def fetch(eng, what, nbytes):
    buf = ctypes.create_string_buffer(nbytes)
    got = eng._L.zs_debug_fetch(eng._ctx, what, 0, buf, nbytes)
    return buf.raw[:got]


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "text"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    lv = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    fmt = sys.argv[4] if len(sys.argv) > 4 else "deflate-raw"
    import torch
    torch.cuda.init()
    import zsamd
    eng = zsamd.Engine(0)
    srcs = [corpus.make({"kind": kind, "n": 262144, "seed": corpus.stream_seed(i)}) for i in range(n)]
    comps = [oracle.compress(s, lv, fmt)[1] for s in srcs]
    got = eng.decompress_batch_raw(comps, fmt, [262144] * n)
    print("seg count", eng.last_seg_count(), "ok", [g[3] == s for g, s in zip(got, srcs)])
    cnt = struct.unpack("<2I", fetch(eng, 16, 8))
    print("counters", cnt)
    nb = cnt[0]
    B = fetch(eng, 17, 48 * nb)
    for b in range(nb):
        m, r, hdr, sym0, end, flags, lbits, dbits, dofs, nl, S, _ = struct.unpack_from("<12I", B, 48 * b)
        print("blk %d: m %d r %d hdr %d sym0 %d end %d flags %d lbits %d dbits %d nl %d S %d" % (
            b, m, r, hdr, sym0, end, flags, lbits, dbits, nl, S))
    LS = 4 * 19
    Lr = fetch(eng, 18, LS * 64 * nb)
    for b in range(nb):
        for l in range(64):
            v = struct.unpack_from("<19I", Lr, LS * (64 * b + l))
            if v[0] != 0xffffffff and (l < 3 or l > 50):
                print("  b%d l%d start %d end %d cnt %d last %d nev %d k0 %d ev %s O %d off %d dend %d dcnt %d BwwC %s act %d" % (
                    (b, l) + v[:6] + (list(v[6:10]),) + v[10:14] + (list(v[14:18]),) + (v[18],)))
    M = fetch(eng, 19, 32 * n)
    for m in range(n):
        print("mem %d:" % m, struct.unpack_from("<5I", M, 32 * m))
    F = fetch(eng, 20, 8 * 64 * n)
    for m in range(n):
        f = struct.unpack_from("<64Q", F, 8 * 64 * m)
        print("found %d:" % m, [x for x in f if x != 2 ** 64 - 1])


if __name__ == "__main__":
    main()
