# Per-member lane times from an instrumentation build (-DZS_IL_EXP=128), C5-ii shaped batch
# (8,192 T-corpus members as deflate64-raw + the 9 reference fixtures):
#   ZS_LIB=variants/il128/libzsgpu.so python3 tools/dbg/il_members.py
import ctypes, os, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd
e = zsamd.Engine(0)
buf = bytes(zsamd.corpus("text", 0, 8192, 65536))
ins = [buf[i * 65536:(i + 1) * 65536] for i in range(8192)]
comp = e.compress_batch(ins, "deflate-raw", 6)
fx = sorted(os.listdir("tests/golden/d64"))
mem = comp[:4096] + [open("tests/golden/d64/" + f, "rb").read() for f in fx] + comp[4096:]
for _ in range(2):
    res = e.decompress_batch_raw(mem, "deflate64-raw", [4 << 20 if len(m) < 32768 and i >= 4096 and i < 4096 + len(fx) else 65536 for i, m in enumerate(mem)])
n = len(mem)
out = (ctypes.c_ulonglong * (2 * n))()
print("rc", zsamd.lib().zs_il_member_cycles(out, n))
t0 = min(out[2 * i] for i in range(n) if out[2 * i])
d = sorted(((out[2 * i + 1] - out[2 * i]) / 100.0, (out[2 * i] - t0) / 100.0, i) for i in range(n) if out[2 * i + 1])
print("members timed", len(d), "median us %.0f" % d[len(d) // 2][0])
for dur, st, i in d[-12:]:
    print("member %5d in %6d out %7d: start %7.0f us, %7.0f us" % (i, len(mem[i]), len(res[i][3]), st, dur))
