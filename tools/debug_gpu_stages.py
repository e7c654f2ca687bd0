"""Debug helper: compare GPU intermediate arrays (chain links, match table,
symbols) of one stream with the CPU emulation in tools/emu_pipeline.py."""
import ctypes, os, struct, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import corpus, oracle, zsamd, emu_pipeline as emu
L = zsamd.lib()
L.zs_debug_fetch.restype = ctypes.c_uint64
L.zs_debug_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
eng = zsamd.Engine(0)
def fetch(what, s, n):
    buf = ctypes.create_string_buffer(n)
    k = L.zs_debug_fetch(eng.handle, what, s, buf, n)
    return buf.raw[:k]
for name, d, level in [("zeros", bytes(65536), 6), ("ramp", bytes(j % 251 for j in range(70000)), 6),
                       ("text", corpus.text(corpus.stream_seed(0), 65536), 6)]:
    eng.compress_batch_raw([d], "deflate-raw", level)
    n = len(d)
    prevd = [0 if v == 0xffff else v for v in struct.unpack("<%dH" % n, fetch(0, 0, 2 * n))]  # 0xffff = no link
    m = struct.unpack("<%dI" % (2 * n), fetch(1, 0, 8 * n))
    st = fetch(4, 0, 64)
    nsym, nblk = struct.unpack_from("<II", st, 0)
    syms = struct.unpack("<%dI" % nsym, fetch(2, 0, 4 * nsym))
    e_prev, e_m, e_syms = emu.stages(d, level)
    bp = next((i for i in range(n) if prevd[i] != e_prev[i]), None)
    bm = next((i for i in range(n) if (m[2 * i], m[2 * i + 1]) != e_m[i]), None)
    bs = next((i for i in range(min(nsym, len(e_syms))) if syms[i] != e_syms[i]), None)
    print(name, "prevd first diff", bp, "" if bp is None else (prevd[bp], e_prev[bp]))
    print(name, "match first diff", bm, "" if bm is None else ((hex(m[2*bm]), hex(m[2*bm+1])), tuple(map(hex, e_m[bm]))))
    print(name, "syms", nsym, len(e_syms), "first diff", bs, "" if bs is None else (hex(syms[bs]), hex(e_syms[bs])), "nblk", nblk)
    blk = fetch(3, 0, 64 * nblk)
    for b in range(nblk):
        print("  blk", struct.unpack_from("<9I4x2Q", blk, 56 * b))
    gpu = eng.compress_batch_raw([d], "deflate-raw", level)[0][1]
    ref = oracle.compress(d, level, "deflate-raw")[1]
    print(name, "bytes equal", gpu == ref, len(gpu), len(ref), next((k for k in range(min(len(gpu), len(ref))) if gpu[k] != ref[k]), None))
    open(os.path.join(ROOT, "gpurun_out", "dbg_%s_gpu.bin" % name), "wb").write(gpu)
    open(os.path.join(ROOT, "gpurun_out", "dbg_%s_ref.bin" % name), "wb").write(ref)
    cod = fetch(5, 0, 4 * 316)
    hdr = fetch(6, 0, 4 * 160)
    open(os.path.join(ROOT, "gpurun_out", "dbg_%s_codes.bin" % name), "wb").write(cod + hdr)
