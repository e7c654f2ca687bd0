"""Times the decode of the largest deflate64 fixture alone, lane path vs exact
path (the member that bounds the C5-ii step).  usage: python tools/d64_single.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
import torch  # noqa: E402  (HIP runtime first, as the tests do)

torch.cuda.init()
import zsamd  # noqa: E402

data = open(os.path.join(ROOT, "tests", "golden", "d64", "100k_lines.deflate64"), "rb").read()
eng = zsamd.Engine(0)
eng.set_option("timing", 1)
for fast in (1, 0):
    eng.set_option("inflate_fast", fast)
    out = eng.decompress_batch([data], "deflate64-raw", out_caps=[4 << 20])[0]
    t0 = time.perf_counter()
    for _ in range(3):
        out = eng.decompress_batch([data], "deflate64-raw", out_caps=[4 << 20])[0]
    dt = (time.perf_counter() - t0) / 3
    print("inflate_fast=%d: %d -> %d bytes, %.2f ms wall, %.2f ms device" % (fast, len(data), len(out), dt * 1e3,
                                                                          eng.last_ms()))
