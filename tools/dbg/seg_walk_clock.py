"""Per-entry clocks of zs_k_seg_walk (a -DZS_SEG_EXP=2 or 3 build):

  make -C zlib-streams-ts_amd/csrc BUILD=build_exp OUT=../../variants/segexp/libzsgpu.so \\
       HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DZS_SEG_EXP=3"
  ZS_LIB=variants/segexp/libzsgpu.so python3 tools/dbg/seg_walk_clock.py [n] [size] [fmt] [OPTION=VALUE ...]

For n T-corpus members of `size` bytes at L6: per entry the header cycles, the spans' phase 1 (lanes decoding
alone) and the rest (sync, records), blocks, spans, the busiest lane's symbols, reseeks."""
import ctypes
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
    fmt = sys.argv[3] if len(sys.argv) > 3 else "deflate-raw"
    import zsamd
    eng = zsamd.Engine(0)
    for kv in sys.argv[4:]:  # engine options NAME=VALUE
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    buf = bytes(zsamd.corpus("text", 0, n, size))
    srcs = [buf[i * size:(i + 1) * size] for i in range(n)]
    comps = eng.compress_batch(srcs, "deflate-raw" if fmt == "deflate64-raw" else fmt, 6)
    for _ in range(3):
        got = eng.decompress_batch_raw(comps, fmt, [size] * n)
    print("ok", sum(g[3] == s for g, s in zip(got, srcs)), "of", n, "seg", eng.last_seg_count())
    L = eng._L
    L.zs_seg_wdbg_fetch.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
    raw = ctypes.create_string_buffer(64 * n)
    L.zs_seg_wdbg_fetch(raw, 64 * n)
    rows = [struct.unpack_from("<8Q", raw, 64 * i) for i in range(n)]
    names = ["hdr", "span1", "span_rest", "blocks", "spans", "lane_syms", "total", "reseeks"]
    avg = [sum(r[i] for r in rows) / n for i in range(8)]
    print("avg", {k: round(v, 1) for k, v in zip(names, avg)})
    worst = max(rows, key=lambda r: r[6])
    print("worst", dict(zip(names, worst)))
    print("cycles per busiest-lane symbol (span1 / lane_syms): %.1f" % (avg[1] / max(1, avg[5])))


if __name__ == "__main__":
    main()
