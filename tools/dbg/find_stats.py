"""Counters of the block-header finder (a ZS_FIND_EXP=8 build, tools/build_variant.sh):
chunks, queued candidates, full checks, clock cycles in the full checks (per wave)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    torch.cuda.init()
    import zsamd
    import corpus
    eng = zsamd.Engine(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    srcs = [corpus.text(corpus.stream_seed(i), 65536) for i in range(n)]
    gz = eng.compress_batch(srcs, "gzip", 6)
    eng.set_timing(True)
    out = eng.decompress_batch_raw(gz, "gzip", [65536] * n)
    print("find ms", eng.last_ms("seg_find"), "ok", all(o[3] == s for o, s in zip(out, srcs)))
    st = (ctypes.c_ulonglong * 4)()
    eng._L.zs_find_stats(st)
    print("chunks %d queued %d checked %d check-cycles/wave %d" % tuple(st))


if __name__ == "__main__":
    main()
