"""Per-span clocks of zs_k_seg_decode (a -DZS_SEG_EXP=1 build: ZS_LIB=variants/segexp/libzsgpu.so):
when each span's wave started and ended, its longest lane's symbols and far reads.
python3 tools/dbg/seg_clock.py [n] [size] [option=value ...]"""
import ctypes
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
    import torch
    torch.cuda.init()
    import zsamd
    eng = zsamd.Engine(0)
    for kv in sys.argv[3:]:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    buf = bytes(zsamd.corpus("text", 0, n, size))
    srcs = [buf[i * size:(i + 1) * size] for i in range(n)]
    comps = eng.compress_batch(srcs, "deflate-raw", 6)
    for _ in range(2):
        got = eng.decompress_batch_raw(comps, "deflate-raw", [size] * n)
    print("ok", sum(g[3] == s for g, s in zip(got, srcs)), "of", n, "seg", eng.last_seg_count())
    L = eng._L
    L.zs_seg_dbg_fetch.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
    nb = 65536
    raw = ctypes.create_string_buffer(32 * nb)
    L.zs_seg_dbg_fetch(raw, 32 * nb)
    bb = ctypes.create_string_buffer(64 * nb)
    got_b = L.zs_debug_fetch(eng._ctx, 17, 0, bb, 64 * nb)
    rows = []
    for b in range(got_b // 64):
        m = struct.unpack_from("<I", bb.raw, 64 * b)[0]
        if m == 0xffffffff or m >= n:
            continue
        t0, t1, sy, far = struct.unpack_from("<4Q", raw.raw, 32 * b)
        if t1 == 0:
            continue
        rows.append((t0, t1, sy, far, b, m))
    t00 = min(r[0] for r in rows)
    T = max(r[1] for r in rows) - t00
    print("real spans", len(rows), "kernel extent %.3f ms (100 MHz ticks)" % (T / 1e5))
    durs = sorted((r[1] - r[0]) / 1e5 for r in rows)
    starts = sorted((r[0] - t00) / 1e5 for r in rows)
    q = lambda a, f: a[min(len(a) - 1, int(f * len(a)))]
    print("durations ms: p10 %.3f p50 %.3f p90 %.3f max %.3f" % (q(durs, .1), q(durs, .5), q(durs, .9), durs[-1]))
    print("starts ms: p10 %.3f p50 %.3f p90 %.3f max %.3f" % (q(starts, .1), q(starts, .5), q(starts, .9), starts[-1]))
    sy = sorted(r[2] for r in rows)
    fr = sorted(r[3] for r in rows)
    print("max-lane symbols p50 %d p90 %d; far reads p50 %d p90 %d" % (q(sy, .5), q(sy, .9), q(fr, .5), q(fr, .9)))
    rows.sort(key=lambda r: r[1] - r[0])
    for r in rows[-5:]:
        print("slowest: slot %d member %d dur %.3f start %.3f sym %d far %d" % (r[4], r[5], (r[1] - r[0]) / 1e5,
                                                                             (r[0] - t00) / 1e5, r[2], r[3]))


if __name__ == "__main__":
    main()
