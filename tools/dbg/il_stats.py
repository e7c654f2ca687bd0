# Reads zs_il_stat from an instrumentation build (-DZS_IL_EXP=64) after a C3-shaped decode:
# ZS_LIB=variants/il64/libzsgpu.so python3 tools/dbg/il_stats.py
import ctypes, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd
e = zsamd.Engine(0)
buf = bytes(zsamd.corpus("mixed", 0, 4096, 65536))
ins = [buf[i * 65536:(i + 1) * 65536] for i in range(4096)]
comp = e.compress_batch(ins, "deflate-raw", 6)
res = e.decompress_batch(comp * 16, "deflate-raw", [65536] * len(comp) * 16)
assert all(r == ins[i % 4096] for i, r in enumerate(res))
out = (ctypes.c_ulonglong * 8)()
print("rc", zsamd.lib().zs_il_stats(out))
waves = len(res) // 64
names = ["lane symbols (max)", "wave steps", "cyc flush", "cyc global copies", "cyc ring copies",
         "cyc overlap copies", "cyc symbol loop (max)", "cyc total (max)"]
for i, nm in enumerate(names):
    print("%-18s per wave %.1f" % (nm, out[i] / waves))
