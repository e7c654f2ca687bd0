"""zsamd -- Python host binding of the MI355X batched deflate/inflate engine.

Mirrors the reference's public surface (src/streams-api.ts, src/mod/streams.ts):

* ``CompressionStream(format, level=...)`` / ``DecompressionStream(format)`` with
  ``write()`` / ``close()`` / ``read()`` -- one stream, run as a batch of one.
* ``compress_batch(inputs, format, level)`` / ``decompress_batch(inputs, format)``
  -- the batch entry the north star adds to ``streams-api.ts``; stream i yields
  exactly what piping ``inputs[i]`` alone through the reference stream class
  (one ``write()`` then ``close()``) yields, or raises/reports the same error.

Everything runs on the GPU through the C-ABI in ``libzsgpu.so``
(include/zs_gpu.h).  There is no CPU fallback: if the library or a GPU is
missing, every entry point raises ``ZsUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZS_LIB overrides the library path (A/B runs of kernel variants)
LIB_PATH = os.environ.get("ZS_LIB") or os.path.join(os.path.dirname(_HERE), "libzsgpu.so")

Z_OK, Z_STREAM_END, Z_NEED_DICT = 0, 1, 2
Z_STREAM_ERROR, Z_DATA_ERROR, Z_MEM_ERROR, Z_BUF_ERROR = -2, -3, -4, -5
PHASE_NONE, PHASE_INIT, PHASE_PROCESS, PHASE_FINISH = 0, 1, 2, 3

# format -> windowBits, streams.ts:220 (compression) and :233 (decompression).
# Unknown strings fall through to 15 there ("deflate"); the same here.
def compress_wbits(fmt: str) -> int:
    return 31 if fmt == "gzip" else (-15 if fmt == "deflate-raw" else 15)


def decompress_wbits(fmt: str) -> int:
    if fmt == "gzip":
        return 31
    if fmt == "deflate-raw":
        return -15
    if fmt == "deflate64-raw":
        return -16
    return 15


class ZsUnavailable(RuntimeError):
    """The HIP engine (libzsgpu.so) or a GPU is not available."""


class ZsError(Exception):
    """Mirrors the Error the reference stream layer throws (streams.ts:53,117,170)."""

    def __init__(self, message: str, status: int = 0, phase: int = 0, msg: str = ""):
        super().__init__(message)
        self.status, self.phase, self.msg = status, phase, msg


def compress_level(level) -> int:
    """streams.ts:221: a level that is not a number means Z_DEFAULT_COMPRESSION (-1, deflate.ts:268-270)."""
    if isinstance(level, bool) or not isinstance(level, int):
        return -1
    return level


def stream_error_text(status: int, phase: int) -> str:
    if phase == PHASE_INIT:
        return "init failed: %d" % status
    if phase == PHASE_FINISH:
        return "finalization error: %d" % status
    return "process error: %d" % status


_lib = None
_P = ctypes.c_void_p
_U64P = ctypes.POINTER(ctypes.c_uint64)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_I32P = ctypes.POINTER(ctypes.c_int32)


def lib():
    """Load libzsgpu.so (raises ZsUnavailable when it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ZsUnavailable("libzsgpu.so not built: run `make -C zlib-streams-ts_amd/csrc` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    L.zs_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(_P)]
    L.zs_ctx_destroy.argtypes = [_P]
    L.zs_last_error.restype = ctypes.c_char_p
    L.zs_version.restype = ctypes.c_char_p
    L.zs_deflate_bound.restype = ctypes.c_uint64
    L.zs_deflate_bound.argtypes = [ctypes.c_uint64, ctypes.c_int]
    L.zs_deflate_batch_device.argtypes = [_P, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, _P, _U64P, _U32P, _P, _U64P,
                                          _U32P, _P, _P, _P]
    L.zs_deflate_batch.argtypes = [_P, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_char_p, _U64P, _U32P,
                                   _P, _U64P, _U32P, _I32P, _U32P]
    L.zs_deflate_batch_ex.argtypes = L.zs_deflate_batch.argtypes + [_U32P]
    L.zs_deflate_batch_device_ex.argtypes = [_P, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, _P, _U64P, _U32P, _P,
                                             _U64P, _U32P, _P, _P, _P, _P]
    _inf_host = [ctypes.c_int, ctypes.c_uint32, ctypes.c_char_p, _U64P, _U32P]
    _inf_res = [_I32P, _I32P, _I32P, _U32P, _U32P, _U32P]
    L.zs_inflate_batch_ex.argtypes = [_P] + _inf_host + [_P, _U64P, _U32P] + _inf_res
    L.zs_inflate_batch_auto.argtypes = [_P] + _inf_host + [ctypes.POINTER(_P), _U64P] + _inf_res
    L.zs_free.argtypes = [_P]
    L.zs_pool_create.argtypes = [ctypes.c_uint64, ctypes.POINTER(_P)]
    L.zs_pool_create_list.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(_P)]
    L.zs_pool_destroy.argtypes = [_P]
    L.zs_pool_size.argtypes = [_P]
    L.zs_pool_device.argtypes = [_P, ctypes.c_int]
    L.zs_pool_deflate_batch.argtypes = L.zs_deflate_batch_ex.argtypes
    L.zs_pool_inflate_batch.argtypes = L.zs_inflate_batch_ex.argtypes
    L.zs_pool_inflate_batch_auto.argtypes = L.zs_inflate_batch_auto.argtypes
    if hasattr(L, "zs_inflate_batch"):
        L.zs_inflate_batch.argtypes = [_P, ctypes.c_int, ctypes.c_uint32, ctypes.c_char_p, _U64P, _U32P, _P, _U64P,
                                       _U32P, _I32P, _I32P, _I32P, _U32P, _U32P]
        L.zs_inflate_batch_device.argtypes = [_P, ctypes.c_int, ctypes.c_uint32, _P, _U64P, _U32P, _P, _U64P, _U32P,
                                              _P, _P, _P, _P, _P, _P]
        L.zs_inflate_message.restype = ctypes.c_char_p
        L.zs_inflate_message.argtypes = [ctypes.c_int32]
    L.zs_crc32_batch_device.argtypes = [_P, ctypes.c_uint32, _P, _U64P, _U32P, _U32P, _P, _P]
    L.zs_adler32_batch_device.argtypes = [_P, ctypes.c_uint32, _P, _U64P, _U32P, _U32P, _P, _P]
    L.zs_crc32_batch.argtypes = [_P, ctypes.c_uint32, ctypes.c_char_p, _U64P, _U32P, _U32P, _U32P]
    L.zs_adler32_batch.argtypes = [_P, ctypes.c_uint32, ctypes.c_char_p, _U64P, _U32P, _U32P, _U32P]
    L.zs_last_batch_ms.restype = ctypes.c_double
    L.zs_last_batch_ms.argtypes = [_P]
    L.zs_last_inflate_lane_count.restype = ctypes.c_uint32
    L.zs_last_inflate_lane_count.argtypes = [_P]
    L.zs_last_inflate_seg_count.restype = ctypes.c_uint32
    L.zs_last_inflate_seg_count.argtypes = [_P]
    L.zs_last_phase_ms.restype = ctypes.c_double
    L.zs_last_phase_ms.argtypes = [_P, ctypes.c_char_p]
    L.zs_set_timing.argtypes = [_P, ctypes.c_int]
    L.zs_corpus.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _P, ctypes.c_int]
    L.zs_selftest.argtypes = [_P, _U64P]
    L.zs_set_option.argtypes = [_P, ctypes.c_char_p, ctypes.c_int]
    L.zs_debug_fetch.restype = ctypes.c_uint64
    L.zs_debug_fetch.argtypes = [_P, ctypes.c_int, ctypes.c_uint32, _P, ctypes.c_uint64]
    _lib = L
    return L


def build_id() -> str:
    """Identity of the engine build: sha256 (16 hex) over the sources libzsgpu.so
    is compiled from (csrc/*, include/zs_gpu.h).  Committed rocprofv3 summaries
    carry it ("_build_id"); bench.py uses a summary's traffic / counters only
    for the build that produced them."""
    import hashlib

    h = hashlib.sha256()
    csrc = os.path.join(os.path.dirname(_HERE), "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile")
    for f in files + ["../../include/zs_gpu.h"]:
        h.update(f.encode() + b"\0")
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _arr(ctype, values):
    a = (ctype * max(1, len(values)))(*values)
    return a


def deflate_bound(n: int, fmt: str = "deflate-raw") -> int:
    """deflateBound (deflate.ts:615-674) for a fresh stream, memLevel 8."""
    return int(lib().zs_deflate_bound(n, compress_wbits(fmt)))


def deflate_capacity(n: int, fmt: str = "deflate-raw") -> int:
    """deflate_bound rounded up to the engine's 4-byte output granularity."""
    return (deflate_bound(n, fmt) + 3) & ~3


class Engine:
    """One device context (one per GPU / process)."""

    def __init__(self, device: int = 0):
        L = lib()
        ctx = _P()
        r = L.zs_ctx_create(device, ctypes.byref(ctx))
        if r != 0:
            raise ZsUnavailable("zs_ctx_create(%d) failed: %s" % (device, L.zs_last_error().decode()))
        self._L, self._ctx, self.device = L, ctx, device

    def selftest(self) -> int:
        """Lane-order violations of same-address LDS atomics (0 expected; see selftest.hip)."""
        v = ctypes.c_uint64(0)
        r = self._L.zs_selftest(self._ctx, ctypes.byref(v))
        if r != 0:
            raise ZsError("zs_selftest failed: %s" % self._L.zs_last_error().decode())
        return int(v.value)

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.zs_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._ctx

    def set_option(self, name: str, value: int):
        """zs_set_option: "timing", "inflate_fast", "check_phases", "match_sweep" (see zs_gpu.h)."""
        if self._L.zs_set_option(self._ctx, name.encode(), int(value)) != 0:
            raise ZsError(self._L.zs_last_error().decode())

    def debug_fetch(self, what: int, stream: int, nbytes: int) -> bytes:
        """zs_debug_fetch: an intermediate array of `stream` from the last deflate batch
        (0 links/members u16, 1 match table u32x2 per position, 2 symbols, ...)."""
        buf = ctypes.create_string_buffer(max(1, nbytes))
        k = self._L.zs_debug_fetch(self._ctx, what, stream, buf, nbytes)
        return buf.raw[:k]

    def set_timing(self, on: bool):
        self._L.zs_set_timing(self._ctx, 1 if on else 0)

    def last_lane_count(self) -> int:
        """members of the last inflate batch decoded by the lane path"""
        return self._L.zs_last_inflate_lane_count(self._ctx)

    def last_seg_count(self) -> int:
        """members of the last inflate batch the segmented decode finished (inflate_seg.hip)"""
        return self._L.zs_last_inflate_seg_count(self._ctx)

    def last_ms(self, phase: Optional[str] = None) -> float:
        if phase is None:
            return self._L.zs_last_batch_ms(self._ctx)
        return self._L.zs_last_phase_ms(self._ctx, phase.encode())

    def _check(self, r: int, what: str):
        if r != 0:
            msg = self._L.zs_last_error().decode()
            if r == Z_STREAM_ERROR:
                raise ZsError("init failed: %d" % r, r, PHASE_INIT, msg)
            raise ZsUnavailable("%s failed (%d): %s" % (what, r, msg))

    # ---------------------------------------------------------- host buffers
    def compress_batch_raw(self, inputs: Sequence[bytes], fmt: str = "deflate-raw", level: int = -1
                           ) -> List[Tuple[int, bytes]]:
        """Returns [(status, bytes)] -- status Z_STREAM_END on success."""
        return [(st, b) for st, b, _ in self.compress_batch_detailed(inputs, fmt, level)]

    def compress_batch_detailed(self, inputs: Sequence[bytes], fmt: str = "deflate-raw", level: int = -1
                                ) -> List[Tuple[int, bytes, int]]:
        """Returns [(status, bytes, check)]: check = the reference's strm.adler after the
        stream (adler32 / crc32 of the input for deflate / gzip, 1 for deflate-raw)."""
        return _deflate_host(self._L, self._L.zs_deflate_batch_ex, self._ctx, inputs, fmt, level, self._check)

    def compress_batch(self, inputs: Sequence[bytes], fmt: str = "deflate-raw", level: int = -1) -> List[bytes]:
        return _ok_or_raise_c(self.compress_batch_raw(inputs, fmt, level))

    def decompress_batch_raw(self, inputs: Sequence[bytes], fmt: str = "deflate-raw",
                             out_caps: Optional[Sequence[int]] = None):
        """Returns [(status, phase, msg, bytes, consumed)].  out_caps None: unbounded
        output, as DecompressionStream (zs_inflate_batch_auto); else per-stream caps."""
        return [r[:5] for r in self.decompress_batch_detailed(inputs, fmt, out_caps)]

    def decompress_batch_detailed(self, inputs: Sequence[bytes], fmt: str = "deflate-raw",
                                  out_caps: Optional[Sequence[int]] = None):
        """Returns [(status, phase, msg, bytes, consumed, check)]."""
        L = self._L
        if out_caps is None:
            return _inflate_host_auto(L, L.zs_inflate_batch_auto, self._ctx, inputs, fmt, self._check)
        return _inflate_host(L, L.zs_inflate_batch_ex, self._ctx, inputs, fmt, out_caps, self._check)

    def decompress_batch(self, inputs: Sequence[bytes], fmt: str = "deflate-raw",
                         out_caps: Optional[Sequence[int]] = None) -> List[bytes]:
        return _ok_or_raise_d(self.decompress_batch_raw(inputs, fmt, out_caps))

    # ---------------------------------------------------- device-resident
    def compress_device(self, level: int, fmt: str, n: int, d_in: int, in_off, in_len, d_out: int, out_off, out_cap,
                        d_status: int, d_out_len: int, hip_stream: int = 0, d_check: int = 0):
        """Device pointers (ints) + host layout arrays (ctypes arrays)."""
        r = self._L.zs_deflate_batch_device_ex(self._ctx, compress_level(level), compress_wbits(fmt), n, _P(d_in),
                                               in_off, in_len, _P(d_out), out_off, out_cap, _P(d_status),
                                               _P(d_out_len), _P(d_check) if d_check else None,
                                               _P(hip_stream) if hip_stream else None)
        self._check(r, "zs_deflate_batch_device")

    def decompress_device(self, fmt: str, n: int, d_in: int, in_off, in_len, d_out: int, out_off, out_cap,
                          d_status: int, d_phase: int, d_msg: int, d_out_len: int, d_consumed: int,
                          hip_stream: int = 0):
        r = self._L.zs_inflate_batch_device(self._ctx, decompress_wbits(fmt), n, _P(d_in), in_off, in_len, _P(d_out),
                                            out_off, out_cap, _P(d_status), _P(d_phase), _P(d_msg), _P(d_out_len),
                                            _P(d_consumed), _P(hip_stream) if hip_stream else None)
        self._check(r, "zs_inflate_batch_device")

    def compress_host(self, level: int, fmt: str, n: int, h_in: int, in_off, in_len, h_out: int, out_off, out_cap,
                      status, out_len):
        """zs_deflate_batch on caller-owned host memory (pointers as ints,
        layout/result arrays as ctypes arrays): the end-to-end host->host path."""
        r = self._L.zs_deflate_batch(self._ctx, level, compress_wbits(fmt), n, ctypes.cast(h_in, ctypes.c_char_p),
                                     in_off, in_len, _P(h_out), out_off, out_cap, status, out_len)
        self._check(r, "zs_deflate_batch")

    def decompress_host(self, fmt: str, n: int, h_in: int, in_off, in_len, h_out: int, out_off, out_cap, status,
                        phase, msg, out_len, consumed):
        """zs_inflate_batch on caller-owned host memory (pointers as ints, layout /
        result arrays as ctypes arrays): the end-to-end host->host decode."""
        r = self._L.zs_inflate_batch(self._ctx, decompress_wbits(fmt), n, ctypes.cast(h_in, ctypes.c_char_p), in_off,
                                     in_len, _P(h_out), out_off, out_cap, status, phase, msg, out_len, consumed)
        self._check(r, "zs_inflate_batch")

    def checksum_device(self, kind: str, n: int, d_in: int, in_off, in_len, d_check: int, hip_stream: int = 0,
                        seeds=None):
        """crc32 / adler32 of n device-resident streams (seeds: ctypes u32 array or None)"""
        fn = self._L.zs_crc32_batch_device if kind == "crc32" else self._L.zs_adler32_batch_device
        r = fn(self._ctx, n, _P(d_in), in_off, in_len, seeds, _P(d_check), _P(hip_stream) if hip_stream else None)
        self._check(r, "checksum")

    def checksum(self, kind: str, bufs: Sequence[bytes], seeds: Optional[Sequence[int]] = None) -> List[int]:
        """[crc32(seed, buf)] or [adler32(seed, buf)] per buffer (common/crc32.ts:26,
        common/adler32.ts:4 semantics; seeds None = initial values)."""
        n = len(bufs)
        if n == 0:
            return []
        offs, lens, o = [], [], 0
        for b in bufs:
            offs.append(o)
            lens.append(len(b))
            o += len(b)
        sd = (ctypes.c_uint32 * n)(*[x & 0xffffffff for x in seeds]) if seeds is not None else None
        out = (ctypes.c_uint32 * n)()
        fn = self._L.zs_crc32_batch if kind == "crc32" else self._L.zs_adler32_batch
        r = fn(self._ctx, n, b"".join(bufs), (ctypes.c_uint64 * n)(*offs), (ctypes.c_uint32 * n)(*lens), sd, out)
        self._check(r, "checksum")
        return list(out)

    def crc32(self, bufs: Sequence[bytes], seeds: Optional[Sequence[int]] = None) -> List[int]:
        return self.checksum("crc32", bufs, seeds)

    def adler32(self, bufs: Sequence[bytes], seeds: Optional[Sequence[int]] = None) -> List[int]:
        return self.checksum("adler32", bufs, seeds)


def _layout(inputs):
    offs, lens, o = [], [], 0
    for b in inputs:
        offs.append(o)
        lens.append(len(b))
        o += len(b)
    return b"".join(inputs), offs, lens


def _deflate_host(L, fn, handle, inputs, fmt, level, check):
    n = len(inputs)
    if n == 0:
        return []
    wbits = compress_wbits(fmt)
    blob, offs, lens = _layout(inputs)
    caps = [(int(L.zs_deflate_bound(len(b), wbits)) + 3) & ~3 for b in inputs]
    ooffs, oo = [], 0
    for c in caps:
        ooffs.append(oo)
        oo += c
    out = ctypes.create_string_buffer(max(1, oo))
    status, olen, chk = (ctypes.c_int32 * n)(), (ctypes.c_uint32 * n)(), (ctypes.c_uint32 * n)()
    r = fn(handle, compress_level(level), wbits, n, blob, _arr(ctypes.c_uint64, offs), _arr(ctypes.c_uint32, lens),
           out, _arr(ctypes.c_uint64, ooffs), _arr(ctypes.c_uint32, caps), status, olen, chk)
    check(r, "deflate batch")
    raw = out.raw
    return [(status[i], raw[ooffs[i]: ooffs[i] + olen[i]], chk[i]) for i in range(n)]


def _inflate_results(L, n, raw, ooffs, status, phase, msg, olen, cons, chk):
    return [(status[i], phase[i], L.zs_inflate_message(msg[i]).decode(), raw[ooffs[i]: ooffs[i] + olen[i]], cons[i],
             chk[i]) for i in range(n)]


def _inflate_host(L, fn, handle, inputs, fmt, out_caps, check):
    n = len(inputs)
    if n == 0:
        return []
    blob, offs, lens = _layout(inputs)
    # the caller's capacities exactly (Z_BUF_ERROR past them); the host entries decode into their own
    # word-aligned staging and copy out only the produced bytes, so these regions need no alignment
    caps = [min(0xffffffff, int(c)) for c in out_caps]
    ooffs, oo = [], 0
    for c in caps:
        ooffs.append(oo)
        oo += c
    out = ctypes.create_string_buffer(max(1, oo))
    res = [(ctypes.c_int32 * n)() for _ in range(3)] + [(ctypes.c_uint32 * n)() for _ in range(3)]
    r = fn(handle, decompress_wbits(fmt), n, blob, _arr(ctypes.c_uint64, offs), _arr(ctypes.c_uint32, lens), out,
           _arr(ctypes.c_uint64, ooffs), _arr(ctypes.c_uint32, caps), *res)
    check(r, "inflate batch")
    return _inflate_results(L, n, out.raw, ooffs, *res)


def _inflate_host_auto(L, fn, handle, inputs, fmt, check):
    n = len(inputs)
    if n == 0:
        return []
    blob, offs, lens = _layout(inputs)
    res = [(ctypes.c_int32 * n)() for _ in range(3)] + [(ctypes.c_uint32 * n)() for _ in range(3)]
    ooffs = (ctypes.c_uint64 * n)()
    outp = _P()
    r = fn(handle, decompress_wbits(fmt), n, blob, _arr(ctypes.c_uint64, offs), _arr(ctypes.c_uint32, lens),
           ctypes.byref(outp), ooffs, *res)
    check(r, "inflate batch")
    try:
        olen = res[3]
        total = max((ooffs[i] + olen[i] for i in range(n)), default=0)
        raw = ctypes.string_at(outp, total) if total else b""
    finally:
        L.zs_free(outp)
    return _inflate_results(L, n, raw, list(ooffs), *res)


def _ok_or_raise_c(results):
    out = []
    for st, b in results:
        if st != Z_STREAM_END:
            raise ZsError(stream_error_text(st, PHASE_FINISH), st, PHASE_FINISH)
        out.append(b)
    return out


def _ok_or_raise_d(results):
    out = []
    for st, ph, msg, b, _ in results:
        if st != Z_STREAM_END:
            raise ZsError(stream_error_text(st, ph), st, ph, msg)
        out.append(b)
    return out


class Pool:
    """A multi-GPU batch engine (zs_pool, SURVEY.md 8(b) device mask / 8(e)): one
    context per device; each batch is split into contiguous stream ranges, one
    per device, run in parallel -- results identical to one device's."""

    def __init__(self, devices: Optional[Sequence[int]] = None, repeat: bool = False):
        """devices: device indices (None / empty: every visible device).  repeat=True
        takes the list as given, in shard order, a device possibly more than once
        (zs_pool_create_list: the sharding rehearsed on one GPU)."""
        L = lib()
        p = _P()
        if repeat:
            ds = [int(d) for d in devices or []]
            r = L.zs_pool_create_list((ctypes.c_int * max(1, len(ds)))(*ds), len(ds), ctypes.byref(p))
        else:
            mask = 0
            for d in devices or []:
                if not 0 <= int(d) < 64:  # the C mask is 64 bits (ctypes would truncate it to "every device")
                    raise ValueError("device index %r outside 0..63" % (d,))
                mask |= 1 << int(d)
            r = L.zs_pool_create(mask, ctypes.byref(p))
        if r != 0:
            err = L.zs_last_error().decode()
            if r == Z_STREAM_ERROR and ("device mask" in err or "device list" in err or "invalid arg" in err):
                raise ValueError(err)
            raise ZsUnavailable("zs_pool_create failed: %s" % err)
        self._L, self._pool = L, p
        self.devices = [L.zs_pool_device(p, k) for k in range(L.zs_pool_size(p))]

    def close(self):
        if getattr(self, "_pool", None):
            self._L.zs_pool_destroy(self._pool)
            self._pool = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, r: int, what: str):
        Engine._check(self, r, what)

    def compress_batch_detailed(self, inputs, fmt="deflate-raw", level=-1):
        return _deflate_host(self._L, self._L.zs_pool_deflate_batch, self._pool, inputs, fmt, level, self._check)

    def compress_batch_raw(self, inputs, fmt="deflate-raw", level=-1):
        return [(st, b) for st, b, _ in self.compress_batch_detailed(inputs, fmt, level)]

    def compress_batch(self, inputs, fmt="deflate-raw", level=-1):
        return _ok_or_raise_c(self.compress_batch_raw(inputs, fmt, level))

    def decompress_batch_detailed(self, inputs, fmt="deflate-raw", out_caps=None):
        L = self._L
        if out_caps is None:
            return _inflate_host_auto(L, L.zs_pool_inflate_batch_auto, self._pool, inputs, fmt, self._check)
        return _inflate_host(L, L.zs_pool_inflate_batch, self._pool, inputs, fmt, out_caps, self._check)

    def decompress_batch_raw(self, inputs, fmt="deflate-raw", out_caps=None):
        return [r[:5] for r in self.decompress_batch_detailed(inputs, fmt, out_caps)]

    def decompress_batch(self, inputs, fmt="deflate-raw", out_caps=None):
        return _ok_or_raise_d(self.decompress_batch_raw(inputs, fmt, out_caps))


_default: Optional[Engine] = None


def default_engine() -> Engine:
    global _default
    if _default is None:
        _default = Engine(0)
    return _default


def compress_batch(inputs: Sequence[bytes], fmt: str = "deflate-raw", level: int = -1) -> List[bytes]:
    return default_engine().compress_batch(inputs, fmt, level)


def decompress_batch(inputs: Sequence[bytes], fmt: str = "deflate-raw") -> List[bytes]:
    return default_engine().decompress_batch(inputs, fmt)


class _OneShotStream:
    """write()/close()/read() over a single-stream GPU batch (streams.ts semantics:
    the whole input is collected, then processed as ONE write() + close())."""

    def __init__(self):
        self._chunks: List[bytes] = []
        self._out: Optional[bytes] = None

    def write(self, chunk: bytes):
        if self._out is not None:
            raise ZsError("stream closed")
        self._chunks.append(bytes(chunk))

    def read(self) -> bytes:
        if self._out is None:
            raise ZsError("stream not closed")
        return self._out


class CompressionStream(_OneShotStream):
    """streams.ts:242-251 (format 'deflate' | 'gzip' | 'deflate-raw', {level})."""

    def __init__(self, fmt: str = "deflate", level: Optional[int] = None):
        super().__init__()
        self.format, self.level = fmt, compress_level(level)

    def close(self) -> bytes:
        self._out = default_engine().compress_batch([b"".join(self._chunks)], self.format, self.level)[0]
        return self._out


class DecompressionStream(_OneShotStream):
    """streams.ts:253-262 (format 'deflate' | 'gzip' | 'deflate-raw' | 'deflate64-raw')."""

    def __init__(self, fmt: str = "deflate"):
        super().__init__()
        self.format = fmt

    def close(self) -> bytes:
        self._out = default_engine().decompress_batch([b"".join(self._chunks)], self.format)[0]
        return self._out


def corpus(kind: str, first_index: int, n_streams: int, length: int, threads: int = 8) -> bytearray:
    """Synthetic T ('text') / M ('mixed') / 'rand' corpora."""
    k = {"text": 0, "mixed": 1, "rand": 2}[kind]
    buf = bytearray(n_streams * length)
    cbuf = (ctypes.c_char * len(buf)).from_buffer(buf)
    lib().zs_corpus(k, first_index, n_streams, length, ctypes.cast(cbuf, _P), threads)
    return buf
