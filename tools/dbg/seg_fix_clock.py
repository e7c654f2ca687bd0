"""Per-span decode clocks of the segmented decode on single deflate64 fixtures (a -DZS_SEG_EXP=1 build:
ZS_LIB=variants/segexp/libzsgpu.so): each span's wave duration, its longest lane's symbols and far reads,
and its lanes' output values -- where a high-expansion member's decode time goes.
python3 tools/dbg/seg_fix_clock.py [name-part ...]"""
import ctypes
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))


def fetch(eng, what, nbytes):
    buf = ctypes.create_string_buffer(nbytes)
    got = eng._L.zs_debug_fetch(eng._ctx, what, 0, buf, nbytes)
    return buf.raw[:got]


def main():
    import torch
    torch.cuda.init()
    import zsamd
    eng = zsamd.Engine(0)
    eng.set_option("seg_small_min", 256)
    L = eng._L
    L.zs_seg_dbg_fetch.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
    keep = sys.argv[1:]
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "inflate_small.json")))
    for c in g["cases"]:
        if not (c["name"].startswith("d64_") and c.get("ok")) or (keep and not any(k in c["name"] for k in keep)):
            continue
        d = open(os.path.join(ROOT, "tests", "golden", "d64", c["name"][4:]), "rb").read()
        for _ in range(2):
            r = eng.decompress_batch_raw([d], "deflate64-raw", [c["out_len"]])[0]
        print("%s in %d out %d seg %d st %d" % (c["name"], len(d), c["out_len"], eng.last_seg_count(), r[0]))
        B = fetch(eng, 17, 64 * 4096)
        nb = min(len(B) // 64, 4096)
        raw = ctypes.create_string_buffer(32 * nb)
        L.zs_seg_dbg_fetch(raw, 32 * nb)
        Lr = fetch(eng, 18, 76 * 64 * nb)
        nb = min(nb, len(Lr) // (76 * 64))
        t00 = None
        for b in range(nb):
            m = struct.unpack_from("<I", B, 64 * b)[0]
            if m == 0xffffffff:
                continue
            t0, t1, sy, far = struct.unpack_from("<4Q", raw.raw, 32 * b)
            if t1 == 0:
                continue
            t00 = t0 if t00 is None else min(t00, t0)
            lanes = []
            for l in range(64):
                v = struct.unpack_from("<19I", Lr, 76 * (64 * b + l))
                if v[0] != 0xffffffff:
                    lanes.append((l, v[0], v[12], v[13], v[18]))
            dc = sorted(x[3] for x in lanes)
            print("  span %d dur %.3f ms sym %d far %d lanes %d dcnt max %d sum %d bits %d..%d" % (
                b, (t1 - t0) / 1e5, sy, far, len(lanes), dc[-1] if dc else 0, sum(dc), lanes[0][1] if lanes else 0,
                max(x[2] for x in lanes) if lanes else 0))
            for x in sorted(lanes, key=lambda x: -x[3])[:3]:
                print("     lane %d start %d dend %d dcnt %d act %d" % x)


if __name__ == "__main__":
    main()
