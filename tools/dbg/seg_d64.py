"""Which deflate64 fixtures the segmented decode finishes, and the records of
those it does not (tools/dbg/seg_dump.py's layout)."""
import ctypes
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


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
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "inflate_small.json")))
    fx = [(c["name"], open(os.path.join(ROOT, "tests", "golden", "d64", c["name"][4:]), "rb").read(), c["out_len"])
          for c in g["cases"] if c["name"].startswith("d64_") and c.get("ok")]
    keep = sys.argv[1:]
    for name, d, n in fx:
        if keep and not any(k in name for k in keep):
            continue
        r = eng.decompress_batch_raw([d], "deflate64-raw", [n])[0]
        ok = eng.last_seg_count()
        cb = fetch(eng, 16, 8)
        if len(cb) < 8:
            print("%-28s in %7d out %8d st %d (not in the segmented decode)" % (name, len(d), n, r[0]), flush=True)
            continue
        cnt = struct.unpack("<2I", cb)
        line = "%-28s in %7d out %8d seg %d st %d blocks %d" % (name, len(d), n, ok, r[0], cnt[0])
        print(line, flush=True)
        if ok:
            continue
        M = struct.unpack_from("<5I", fetch(eng, 19, 32))
        print("   mem", M)
        B = fetch(eng, 17, 64 * 64)
        nb = len(B) // 64
        for b in range(nb):
            if struct.unpack_from("<I", B, 64 * b)[0] == 0xffffffff:
                continue
            v = struct.unpack_from("<16I", B, 64 * b)
            print("   blk", b, "m r hdr sym0 end flags lb db dofs nl S", v[:11])
        Lr = fetch(eng, 18, 76 * 64 * nb)
        for b in range(len(Lr) // (76 * 64)):
            if struct.unpack_from("<I", B, 64 * b)[0] == 0xffffffff:
                continue
            for l in range(64):
                v = struct.unpack_from("<19I", Lr, 76 * (64 * b + l))
                if v[0] != 0xffffffff:
                    print("     b%d l%d start %d end %d cnt %d last %d O %d off %d dend %d dcnt %d act %d" % (
                        b, l, v[0], v[1], v[2], v[3], v[10], v[11], v[12], v[13], v[18]))
        F = fetch(eng, 20, 8 * 64)
        print("   found", [x for x in struct.unpack_from("<64Q", F, 0) if x != 2 ** 64 - 1])


if __name__ == "__main__":
    main()
