"""Cycle profile of zs_k_fast's phases (build with -DZS_FG_PROF; prints from the kernel)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, "zlib-streams-ts_amd")
import corpus
import zsamd

lvl = int(sys.argv[1]) if len(sys.argv) > 1 else 1
eng = zsamd.Engine(0)
ins = [corpus.make({"kind": "text", "n": 262144, "seed": 5 + i}) for i in range(4)]
eng.compress_batch_raw(ins, "deflate-raw", lvl)
