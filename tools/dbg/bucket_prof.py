# zs_k_bucket's passes (build with -DZS_BK_PROF=1): ZS_LIB=variants/bk/libzsgpu.so python3 tools/dbg/bucket_prof.py [streams]
import ctypes, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
e = zsamd.Engine(0)
buf = bytes(zsamd.corpus("text", 0, n, 65536))
e.compress_batch_raw([buf[i * 65536:(i + 1) * 65536] for i in range(n)], "deflate-raw", 6)
out = (ctypes.c_ulonglong * 4)()
zsamd.lib().zs_bucket_stats(out)
for i, nm in enumerate(["pass 1 (counts)", "scan", "pass 2 (claims + scatter)"]):
    print("%-26s %7.1f us per workgroup" % (nm, out[i] / max(1, out[3]) / 100.0))
