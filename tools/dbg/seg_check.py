"""Diagnostic for the segmented decode (inflate_seg.hip) on the GPU: small
batches of members in every format, decoded with the segmented path on and off;
prints, per batch, how many members it finished and whether every output
equals the oracle's decode (reference_bugs = 1: the reference's window-wrap copy).

  python3 tools/dbg/seg_check.py
"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import corpus  # noqa: E402
import oracle  # noqa: E402


def main():
    import torch

    torch.cuda.init()
    import zsamd

    eng = zsamd.Engine(0)
    rng = random.Random(11)
    cases = []
    for fmt in ("deflate-raw", "deflate", "gzip"):
        for kind in ("text", "mixed"):
            for lv in (1, 6, 9):
                ms = []
                for _ in range(6):
                    n = rng.choice([20000, 65536, 150000, 262144, 500000])
                    s = corpus.make({"kind": kind, "n": n, "seed": corpus.stream_seed(rng.randrange(4096))})
                    ms.append((s, oracle.compress(s, lv, fmt)[1]))
                cases.append((fmt, kind, lv, ms))
    for fmt, kind, lv, ms in cases:
        comps = [c for _, c in ms]
        caps = [(len(s) + 3) & ~3 for s, _ in ms]
        want = [oracle.decompress(c, fmt, cap=len(s) + 16, reference_bugs=True) for s, c in ms]
        t0 = time.time()
        got = eng.decompress_batch_raw(comps, fmt, caps)
        nseg = eng.last_seg_count()
        dt = time.time() - t0
        ok = all(g[0] == w[0] and g[3] == w[1] and g[4] == w[2] for g, w in zip(got, want))
        print("%-11s %-5s L%d  seg %d/%d  ok %s  %.2fs" % (fmt, kind, lv, nseg, len(ms), ok, dt), flush=True)
        if not ok:
            for i, (g, w) in enumerate(zip(got, want)):
                if not (g[0] == w[0] and g[3] == w[1] and g[4] == w[2]):
                    nd = sum(1 for a, b in zip(g[3], w[1]) if a != b)
                    first = next((k for k, (a, b) in enumerate(zip(g[3], w[1])) if a != b), None)
                    print("   member %d: st %d/%d len %d/%d cons %d/%d diff %d first %s" % (
                        i, g[0], w[0], len(g[3]), len(w[1]), g[4], w[2], nd, first))
    # deflate64 fixtures
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "inflate_small.json")))
    fx = [(open(os.path.join(ROOT, "tests", "golden", "d64", c["name"][4:]), "rb").read(), c["out_len"])
          for c in g["cases"] if c["name"].startswith("d64_") and c.get("ok")]
    comps = [d for d, _ in fx]
    caps = [(n + 3) & ~3 for _, n in fx]
    got = eng.decompress_batch_raw(comps, "deflate64-raw", caps)
    nseg = eng.last_seg_count()
    want = [oracle.decompress(d, "deflate64-raw", cap=n + 16) for d, n in fx]
    ok = all(a[0] == b[0] and a[3] == b[1] for a, b in zip(got, want))
    print("d64 fixtures seg %d/%d ok %s" % (nseg, len(fx), ok), flush=True)


if __name__ == "__main__":
    main()
