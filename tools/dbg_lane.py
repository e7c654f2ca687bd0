import sys, random
sys.path.insert(0, 'zlib-streams-ts_amd'); sys.path.insert(0, 'tests')
import zsamd, oracle, corpus
eng = zsamd.Engine(0)
for fmt in ("deflate-raw", "deflate", "gzip", "deflate64-raw"):
    enc = "deflate-raw" if fmt == "deflate64-raw" else fmt
    for kind, n in (("text", 0), ("text", 5), ("text", 100), ("text", 5000), ("text", 65536), ("zeros", 3000), ("mixed", 40000)):
        s = corpus.make({"kind": kind, "n": n, "seed": 3})
        for lvl in (1, 6):
            c = oracle.compress(s, lvl, enc)[1]
            (st, ph, msg, out, cons), = eng.decompress_batch_raw([c], fmt, out_caps=[len(s) + 64])
            print(fmt, kind, n, lvl, st, out == s, "lane", eng.last_lane_count(), flush=True)
