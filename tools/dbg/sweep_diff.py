"""Match table of zs_k_sweep vs the chain-walk kernels (match_sweep=0) on a few streams; prints mismatches."""
import struct, sys
sys.path.insert(0, "zlib-streams-ts_amd"); sys.path.insert(0, "tests")
import torch; torch.cuda.init()
import corpus, zsamd
e = zsamd.Engine(0)
lvl = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ins = [corpus.text(corpus.stream_seed(i), 65536) for i in range(2)] + [bytes(x & 0x7F for x in corpus.rand(91, 65536)), corpus.rand(5, 40000)]
tabs = []
for sw in (1, 0):
    e.set_option("match_sweep", sw)
    e.compress_batch_raw(ins, "deflate-raw", lvl)
    tabs.append([e.debug_fetch(1, i, 8 * len(d)) for i, d in enumerate(ins)])
for i, d in enumerate(ins):
    a = struct.unpack("<%dI" % (2 * len(d)), tabs[0][i]); b = struct.unpack("<%dI" % (2 * len(d)), tabs[1][i])
    bad = [p for p in range(len(d)) if a[2 * p:2 * p + 2] != b[2 * p:2 * p + 2]]
    print("stream", i, "mismatches", len(bad))
    for p in bad[:6]:
        print("  pos", p, "sweep %08x %08x" % a[2 * p:2 * p + 2], "walk %08x %08x" % b[2 * p:2 * p + 2])
