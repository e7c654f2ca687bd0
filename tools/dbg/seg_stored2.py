"""Bisect stored-block shapes the segmented decode leaves (one member per batch), GPU diagnostic."""
import os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
import corpus, oracle, bitbuild, zsamd
e = zsamd.Engine()
src = corpus.text(11, 150000) + corpus.rand(12, 100000)
rng = random.Random(3)
def F(n, dmax=30, lit=0.6):
    syms = []
    for i in range(n):
        if i < 40 or rng.random() < lit:
            syms.append(("lit", src[rng.randrange(len(src))]))
        else:
            syms.append(("copy", rng.choice([3, 4, 9, 17, 40]), rng.randint(1, dmax)))
    return ("fixed", syms)
def S(n, at=0):
    return ("stored", src[at:at + n])
shapes = {
    "F": [F(3000)],
    "Fbig": [F(12000)],
    "F S10": [F(3000), S(10)],
    "S10 F": [S(10), F(3000)],
    "S5000 F": [S(5000), F(3000)],
    "F100 F": [F(100), F(3000)],
    "F F100": [F(3000), F(100)],
    "F F d2000": [F(3000, 2000), F(3000, 2000)],
    "F F lit.9": [F(3000, 2000, 0.9), F(3000, 2000, 0.9)],
    "F S65535 S20001": [F(3000), S(65535), S(20001)],
    "F F S10": [F(3000), F(3000), S(10)],
}
for name, parts in shapes.items():
    m, want = bitbuild.blocks(parts)
    w = oracle.decompress(m, "deflate-raw", cap=1 << 20, reference_bugs=True)
    g = e.decompress_batch_detailed([m], "deflate-raw", [len(w[1]) + 16])
    print("%-18s in %6d out %6d seg %d ok %s" % (name, len(m), len(w[1]), e.last_seg_count(), g[0][3] == w[1] == want), flush=True)
