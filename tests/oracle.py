"""ctypes binding of the C oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE: the oracle is the parity checker, never the product.
Built by `make -C oracle` (also run by __graft_entry__.build()).
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")

Z_OK, Z_STREAM_END, Z_NEED_DICT = 0, 1, 2
Z_STREAM_ERROR, Z_DATA_ERROR, Z_MEM_ERROR, Z_BUF_ERROR = -2, -3, -4, -5
PHASE_NONE, PHASE_INIT, PHASE_PROCESS, PHASE_FINISH = 0, 1, 2, 3
WBITS = {"deflate-raw": -15, "deflate": 15, "gzip": 31, "deflate64-raw": -16}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB)
        L.zo_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                  ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]
        L.zo_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p)]
        L.zo_crc32.restype = ctypes.c_uint32
        L.zo_crc32.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.zo_adler32.restype = ctypes.c_uint32
        L.zo_adler32.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.zo_deflate_bound.restype = ctypes.c_size_t
        L.zo_deflate_bound.argtypes = [ctypes.c_size_t, ctypes.c_int]
        L.zo_set_reference_bugs.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def compress(data, level=6, fmt="deflate-raw"):
    """Returns (status, bytes, phase)."""
    L = lib()
    cap = L.zo_deflate_bound(len(data), WBITS[fmt]) + 64
    out = ctypes.create_string_buffer(cap)
    ol = ctypes.c_size_t()
    ph = ctypes.c_int()
    r = L.zo_compress(bytes(data), len(data), level, WBITS[fmt], out, cap, ctypes.byref(ol), ctypes.byref(ph))
    return r, out.raw[: ol.value], ph.value


def decompress(data, fmt="deflate-raw", cap=None, reference_bugs=True):
    """Returns (status, bytes, consumed, phase, msg)."""
    L = lib()
    L.zo_set_reference_bugs(1 if reference_bugs else 0)
    cap = cap or max(1 << 16, len(data) * 1100)
    out = ctypes.create_string_buffer(cap)
    ol, cons = ctypes.c_size_t(), ctypes.c_size_t()
    ph = ctypes.c_int()
    msg = ctypes.c_char_p()
    r = L.zo_decompress(bytes(data), len(data), WBITS[fmt], out, cap, ctypes.byref(ol), ctypes.byref(cons),
                        ctypes.byref(ph), ctypes.byref(msg))
    return r, out.raw[: ol.value], cons.value, ph.value, (msg.value or b"").decode()


def crc32(data, crc=0):
    return lib().zo_crc32(crc, bytes(data), len(data))


def adler32(data, adler=1):
    return lib().zo_adler32(adler, bytes(data), len(data))


def stream_error_text(status, phase):
    """The Error message the reference stream layer throws (streams.ts:53,117,170)."""
    if phase == PHASE_INIT:
        return "init failed: %d" % status
    if phase == PHASE_PROCESS:
        return "process error: %d" % status
    if phase == PHASE_FINISH:
        return "finalization error: %d" % status
    return ""
