"""Which stored-block members the segmented decode finishes (one member per batch), GPU diagnostic."""
import os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
import corpus, oracle, bitbuild, zsamd
e = zsamd.Engine()
src = corpus.text(11, 150000) + corpus.rand(12, 100000) + corpus.make({"kind": "mixed", "n": 100000, "seed": 13})
raw = [bitbuild.stored_mix(random.Random(i), 262144, src, level0=True)[0] for i in range(3)]
raw += [bitbuild.stored_mix(random.Random(10 + i), 200000, src)[0] for i in range(3)]
raw += [oracle.compress(corpus.rand(8, 262144), 6, "deflate-raw")[1]]
raw += [oracle.compress(corpus.patchwork(seed, 262144), lv, "deflate-raw")[1] for seed, lv in [(208, 6), (201, 1), (204, 9), (205, 6)]]
for i, c in enumerate(raw):
    w = oracle.decompress(c, "deflate-raw", cap=1 << 20, reference_bugs=True)
    for big in (0, 1):
        g = e.decompress_batch_detailed([c] * (1 + 3 * big), "deflate-raw", [len(w[1]) + 16] * (1 + 3 * big))
        print(i, len(c), len(w[1]), "batch", 1 + 3 * big, "seg", e.last_seg_count(), "ok", g[0][3] == w[1], g[0][0], flush=True)
