"""Decodes one large member through each inflate path (exact, lane, wave) with
zlib semantics and reports the first byte where each differs from the source.
usage: python tools/dbg_wave.py"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

torch.cuda.init()
import corpus  # noqa: E402
import oracle  # noqa: E402
import zsamd  # noqa: E402

eng = zsamd.Engine(0)
cases = [("rand", 100000, 9), ("text", 262144, 6), ("zeros", 300000, 6), ("mixed", 200000, 1)]
for kind, n, lvl in cases:
    src = corpus.make({"kind": kind, "n": n, "seed": 1234})
    for fmt in ("deflate-raw", "gzip"):
        comp = oracle.compress(src, lvl, fmt)[1]
        for name, opts in (("exact", dict(inflate_fast=0, inflate_ref_wrap=0)),
                           ("lane", dict(inflate_wave_min=0, inflate_ref_wrap=0)),
                           ("wave", dict(inflate_wave_min=1, inflate_ref_wrap=0))):
            for k, v in opts.items():
                eng.set_option(k, v)
            st, ph, msg, out, cons = eng.decompress_batch_raw([comp], fmt, out_caps=[n + 64])[0]
            lanes = eng.last_lane_count()
            for k in ("inflate_fast", "inflate_ref_wrap"):
                eng.set_option(k, 1)
            eng.set_option("inflate_wave_min", 32768)
            first = next((i for i in range(min(len(out), n)) if out[i] != src[i]), None)
            print(kind, n, lvl, fmt, name, "st", st, msg, "len", len(out), "cons", cons, "/", len(comp),
                  "lane_count", lanes, "first_diff", first, flush=True)
