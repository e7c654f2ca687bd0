import ctypes, os, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd
e = zsamd.Engine(0)
data = open("tests/golden/d64/100k_lines.deflate64", "rb").read()
out = e.decompress_batch([data], "deflate64-raw", out_caps=[4 << 20])[0]
st = (ctypes.c_ulonglong * 4)()
zsamd.lib().zs_split_stats(st)
print("rest calls", st[0], "cycles total", st[1], "per call", st[1] / max(1, st[0]))
