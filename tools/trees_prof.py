"""Wall-clock profile of zs_k_trees' phases on a C2-shaped batch (build with
-DZS_TR_PROF=1: tools/build_variant.sh trprof deflate_emit.hip -DZS_TR_PROF=1).
usage: ZS_LIB=variants/trprof/libzsgpu.so python3 tools/trees_prof.py [streams]"""
import ctypes, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
e = zsamd.Engine(0)
buf = bytes(zsamd.corpus("text", 0, n, 65536))
ins = [buf[i * 65536:(i + 1) * 65536] for i in range(n)]
e.compress_batch_raw(ins, "deflate-raw", 6)
L = zsamd.lib()
out = (ctypes.c_ulonglong * 8)()
L.zs_trees_stats(out)
blocks = max(1, out[7])
for i, nm in enumerate(["histogram", "L heap", "L lengths+codes", "D tree", "bl tree + header", "rest"]):
    print("%-18s %8.1f us per block" % (nm, out[i] / blocks / 100.0))
print("blocks", blocks)
