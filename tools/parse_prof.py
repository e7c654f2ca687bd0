"""Wall-clock profile of zs_k_parse's passes on a C2-shaped batch (build with
-DZS_PARSE_PROF=1: tools/build_variant.sh pp deflate_parse.hip -DZS_PARSE_PROF=1).
usage: ZS_LIB=variants/pp/libzsgpu.so python3 tools/parse_prof.py [streams]
Prints each pass's time summed over waves (wall_clock64 ticks, 100 MHz) per wave."""
import ctypes, sys
sys.path.insert(0, "zlib-streams-ts_amd")
import torch; torch.cuda.init()
import zsamd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
e = zsamd.Engine(0)
if len(sys.argv) > 2:
    e.set_option("parse_waves", int(sys.argv[2]))
if len(sys.argv) > 3:
    e.set_option("demand", int(sys.argv[3]))
buf = bytes(zsamd.corpus("text", 0, n, 65536))
ins = [buf[i * 65536:(i + 1) * 65536] for i in range(n)]
e.compress_batch_raw(ins, "deflate-raw", 6)
L = zsamd.lib()
out = (ctypes.c_ulonglong * 16)()
L.zs_parse_stats(out)
waves = max(1, out[5])
for i, nm in enumerate(["pass A", "phase 1 (pass B)", "splice", "block cuts (dw: walk phases)", "block records (dw: count)"]):
    print("%-18s %8.1f us per stream-wave" % (nm, out[i] / waves / 100.0))
print("dw: stages %.1f per stream, drain steps %.1f per stream, staging time %.1f us per stream-wave" % (
    out[8] / n, out[9] / n, out[10] / n / 100.0))
print("waves %d, demand walks %d (%.1f per stream), members walked %.1f per walk" % (
    out[5], out[6], out[6] / n, out[7] / max(1, out[6])))
