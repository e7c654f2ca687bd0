import ctypes, os, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd
e = zsamd.Engine(0)
buf = bytes(zsamd.corpus("text", 0, 4096, 65536))
ins = [buf[i * 65536:(i + 1) * 65536] for i in range(4096)]
e.compress_batch_raw(ins, "deflate-raw", 6)
out = (ctypes.c_ulonglong * 8)()
print("rc", zsamd.lib().zs_sw_stats(out))
names = ["chunks", "fast groups", "masked groups", "long branches", "wave steps"]
for i, nm in enumerate(names):
    print(nm, out[i], "per chunk %.2f" % (out[i] / max(1, out[0])))
