"""Which of tests/test_gpu_seg.py's long-run members the segmented decode finishes, one member per batch,
and the member record (bad, total, consumed, want, pieces) of those it does not.
ZS_LIB=... python3 tools/dbg/seg_runs.py"""
import ctypes
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
    import oracle
    from test_gpu_seg import _runs_member
    eng = zsamd.Engine(0)
    eng.set_option("seg_small_min", 4096)
    eng.set_option("seg_bits", 1024)
    for refw in (1, 0):
        eng.set_option("inflate_ref_wrap", refw)
        for i in range(12):
            s = _runs_member(500 + i, 150000 + 7919 * i)
            c = oracle.compress(s, [1, 6, 9][i % 3], "deflate-raw")[1]
            r = eng.decompress_batch_raw([c], "deflate-raw", [len(s)])[0]
            ok = eng.last_seg_count()
            M = struct.unpack_from("<6I", fetch(eng, 19, 32))
            want = oracle.decompress(c, "deflate-raw", cap=len(s), reference_bugs=bool(refw))[1]
            print("refw %d member %d in %d out %d seg %d st %d same %s mem %s" % (refw, i, len(c), len(s), ok, r[0],
                                                                              r[3] == want, M), flush=True)
            if ok or i or not refw:
                continue
            E = fetch(eng, 21, 16 * 64)
            print("  entries", [struct.unpack_from("<4I", E, 16 * k) for k in range(64)
                                if struct.unpack_from("<4I", E, 16 * k)[3] or k == 0])
            B = fetch(eng, 17, 64 * M[5])
            for b in range(len(B) // 64):
                v = struct.unpack_from("<16I", B, 64 * b)
                print("  span %d m %d e %d hdr %d sym0 %d end %d flags %d nl %d S %d next %d" % (
                    (b,) + v[:6] + v[10:13]))
            Lr = fetch(eng, 18, 76 * 64 * M[5])
            for b in range(len(Lr) // (76 * 64)):
                for l in range(64):
                    v = struct.unpack_from("<19I", Lr, 76 * (64 * b + l))
                    if v[0] != 0xffffffff and v[0] != 0:
                        print("    b%d l%d start %d end %d cnt %d" % (b, l, v[0], v[1], v[2]))


if __name__ == "__main__":
    main()
