"""Times the decode of the largest deflate64 fixture alone: the split path
(default), the wave path (inflate_split=0) and the exact path (inflate_fast=0),
with the split path's phases.  usage: python tools/d64_single.py"""
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
for name, opts in (("split", {}), ("wave", {"inflate_split": 0}), ("exact", {"inflate_fast": 0})):
    for k, v in opts.items():
        eng.set_option(k, v)
    out = eng.decompress_batch([data], "deflate64-raw", out_caps=[4 << 20])[0]
    t0 = time.perf_counter()
    for _ in range(3):
        out = eng.decompress_batch([data], "deflate64-raw", out_caps=[4 << 20])[0]
    dt = (time.perf_counter() - t0) / 3
    ph = {p: round(eng.last_ms(p), 3) for p in ("split_find", "split_decode", "split_resolve", "inflate_wave", "inflate")
          if eng.last_ms(p) >= 0}
    print("%s: %d -> %d bytes, %.2f ms wall, %.2f ms device %s" % (name, len(data), len(out), dt * 1e3, eng.last_ms(), ph))
    eng.set_option("inflate_split", 1)
    eng.set_option("inflate_fast", 1)
