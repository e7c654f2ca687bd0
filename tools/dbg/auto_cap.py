import os, sys
sys.path.insert(0, "zlib-streams-ts_amd"); sys.path.insert(0, "tests")
import torch; torch.cuda.init()
import zsamd
e = zsamd.Engine(0)
z = open("tests/golden/d64/zeros_100k.deflate64", "rb").read()
for caps in ([65536], [524288], [100000], [100004]):
    r = e.decompress_batch_raw([z], "deflate64-raw", out_caps=caps)
    st, ph, msg, out, cons = r[0]
    print(caps, st, ph, msg, len(out), cons, sum(out), out[:8])
r = e.decompress_batch_detailed([z], "deflate64-raw")
st, ph, msg, out, cons, chk = r[0]
print("auto", st, ph, msg, len(out), cons, sum(out), [i for i, b in enumerate(out) if b][:10])
