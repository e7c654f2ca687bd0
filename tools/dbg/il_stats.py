# Reads zs_il_stat from an instrumentation build (-DZS_IL_EXP=64) after a decode:
#   ZS_LIB=variants/il64/libzsgpu.so python3 tools/dbg/il_stats.py [c3|c5]
# c3: 4096 M-corpus raw L6 members x 16 (C3); c5: 8192 T-corpus gzip L6 members (C5-i, narrow workgroups)
import ctypes, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
e = zsamd.Engine(0)
if cfg == "c3":
    buf = bytes(zsamd.corpus("mixed", 0, 4096, 65536))
    ins = [buf[i * 65536:(i + 1) * 65536] for i in range(4096)]
    fmt, rep = "deflate-raw", 16
else:
    buf = bytes(zsamd.corpus("text", 0, 8192, 65536))
    ins = [buf[i * 65536:(i + 1) * 65536] for i in range(8192)]
    fmt, rep = "gzip", 1
comp = e.compress_batch(ins, fmt, 6)
res = e.decompress_batch(comp * rep, fmt, [65536] * len(comp) * rep)
assert all(r == ins[i % len(ins)] for i, r in enumerate(res))
out = (ctypes.c_ulonglong * 8)()
print("rc", zsamd.lib().zs_il_stats(out))
waves = len(res) // (64 if cfg == "c3" else 2)
names = ["lane symbols (max)", "wave steps", "cyc flush", "cyc global copies", "cyc ring copies",
         "cyc overlap copies", "cyc symbol loop (max)", "cyc total (max)"]
for i, nm in enumerate(names):
    print("%-18s per wave %.1f" % (nm, out[i] / waves))
