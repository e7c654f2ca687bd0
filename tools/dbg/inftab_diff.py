"""Runs zs_inftab_selfcheck and prints the first failing code set: lengths, the serial and wave tables' differing
entries (op, bits, val).  python3 tools/dbg/inftab_diff.py"""
import ctypes
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
import zsamd

e = zsamd.Engine(0)
L = e._L
L.zs_inftab_selfcheck.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.POINTER(ctypes.c_ulonglong)]
bad = ctypes.c_ulonglong(0)
print("rc", L.zs_inftab_selfcheck(0, 12345, 256, 32, ctypes.byref(bad)), "mismatches", bad.value)
EN = 852 + 8
n = 16 + 320 + 2 * EN
buf = ctypes.create_string_buffer(4 * n)
L.zs_inftab_dbg_fetch.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
L.zs_inftab_dbg_fetch(buf, 4 * n)
g = struct.unpack("<%dI" % n, buf.raw)
print("type", g[0], "d64", g[1], "codes", g[2], "ret", g[3], g[4], "root", g[5], g[6], "used", g[7], g[8])
lens = g[16:16 + g[2]]
print("lens", lens)
ta, tb = g[336:336 + EN], g[336 + EN:336 + 2 * EN]
f = lambda c: (c >> 24, (c >> 16) & 255, c & 0xffff)
d = [(i, f(ta[i]), f(tb[i])) for i in range(max(g[7], g[8])) if ta[i] != tb[i]]
print("differing entries", len(d))
for x in d[:30]:
    print(x)
