"""Header sub-phase clocks of zs_k_seg_walk (a -DZS_SEG_EXP=18 build: per-entry clocks + header phases):
  tools/build_variant.sh seghdr inflate_seg.hip -DZS_SEG_EXP=18
  ZS_LIB=variants/seghdr/libzsgpu.so python3 tools/dbg/seg_hdr_clock.py [n] [size] [fmt]
Prints, per dynamic header, the core clocks of: the code-length code table, the serial code-length decode, the
literal/length table and the distance table (inflate_table, zs_inftab.h)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools", "dbg"))
import seg_walk_clock  # noqa: E402

seg_walk_clock.main()
import zsamd  # noqa: E402

L = zsamd.lib()
L.zs_seg_hdbg_fetch.argtypes = [ctypes.c_void_p]
v = (ctypes.c_ulonglong * 8)()
L.zs_seg_hdbg_fetch(v)
h = max(1, v[4])
print("dynamic headers %d (summed over the timed runs), code lengths %.1f per header" % (v[4], v[5] / h))
for i, nm in enumerate(["code-length table", "code-length decode", "lit/len table", "dist table"]):
    print("%-20s %10.1f cycles per header" % (nm, v[i] / h))
