"""Cycle profile of zs_k_parse's passes (build with -DZS_PARSE_PROF; prints from the kernel)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, "zlib-streams-ts_amd")
import corpus
import zsamd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
eng = zsamd.Engine(0)
ins = [corpus.make({"kind": "text", "n": 65536, "seed": 5 + i}) for i in range(n)]
eng.compress_batch_raw(ins, "deflate-raw", 6)
