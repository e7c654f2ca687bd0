"""GPU parity of the checksum entry points (zs_crc32_batch / zs_adler32_batch and
their _device forms) with the reference's crc32(crc, buf) / adler32(adler, buf):
its known-answer tests (coverage-crc32.spec.ts:9-14,16-21,
coverage-adler32.spec.ts:10-21,23-29) and seeded continuations."""
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu


def ref_adler32(adler, buf):
    """adler32.ts:4-25 restated (2000-byte blocks, reduction after each)"""
    lo, s2, pos, n = adler & 0xffff, (adler >> 16) & 0xffff, 0, len(buf)
    while n > 0:
        k = min(n, 2000)
        n -= k
        for _ in range(k):
            lo = (lo + buf[pos]) & 0xffffffff
            s2 = (s2 + lo) & 0xffffffff
            pos += 1
        lo %= 65521
        s2 %= 65521
    return ((s2 << 16) | lo) & 0xffffffff


def test_reference_known_answers(engine):
    assert engine.crc32([b"hello"], [0]) == [0x3610A686]
    assert engine.crc32([bytes([1, 2, 3, 4, 5])], [0]) == [zlib.crc32(bytes([1, 2, 3, 4, 5]))]
    assert engine.adler32([bytes([5])], [0]) == [(5 << 16) | 5]
    assert engine.adler32([bytes([1, 2, 3])], [0]) == [(10 << 16) | 6]
    big = bytes(i & 0xFF for i in range(5552 + 10))  # the NMAX-loop case
    assert engine.adler32([big], [1]) == [zlib.adler32(big)]
    # initial values: crc32 of nothing is 0, adler32 is 1
    assert engine.crc32([b""]) == [0] and engine.adler32([b""]) == [1]


def test_seeded_continuation(engine):
    rng = random.Random(9)
    bufs, seeds = [], []
    for k in range(300):
        n = rng.choice([0, 1, 2, 3, 7, 63, 64, 65, 1000, 2000, 2001, 4095, 70000, rng.randrange(1, 300000)])
        bufs.append(bytes(rng.randrange(256) for _ in range(min(n, 2048))) * (n // 2048 + 1))
        bufs[-1] = bufs[-1][:n]
        seeds.append(rng.choice([0, 1, 0xFFFFFFFF, 0xFFF0FFF0, rng.randrange(1 << 32)]))
    crc = engine.crc32(bufs, seeds)
    adl = engine.adler32(bufs, seeds)
    for b, s, c, a in zip(bufs, seeds, crc, adl):
        assert c == zlib.crc32(b, s), (len(b), s)
        assert a == ref_adler32(s, b), (len(b), s)
    # a checksum continued over a split buffer equals the checksum of the whole
    whole = bufs[-1] + bufs[-2]
    head = engine.crc32([bufs[-1]])[0]
    assert engine.crc32([bufs[-2]], [head]) == [zlib.crc32(whole)]
    head = engine.adler32([bufs[-1]])[0]
    assert engine.adler32([bufs[-2]], [head]) == [zlib.adler32(whole)]


def test_device_entry_points(engine):
    import ctypes

    import torch

    data = [b"hello", b"", bytes(range(256)) * 40]
    blob = torch.tensor(list(b"".join(data)) + [0], dtype=torch.uint8, device="cuda")
    offs = (ctypes.c_uint64 * 3)(0, 5, 5)
    lens = (ctypes.c_uint32 * 3)(5, 0, 10240)
    out = torch.zeros(3, dtype=torch.int64, device="cuda")
    seeds = (ctypes.c_uint32 * 3)(0, 1234, 77)
    engine.checksum_device("crc32", 3, blob.data_ptr(), offs, lens, out.data_ptr(), seeds=seeds)
    torch.cuda.synchronize()
    got = [int(x) & 0xFFFFFFFF for x in out.view(torch.int32).cpu().tolist()[:3]]
    assert got == [0x3610A686, 1234, zlib.crc32(data[2], 77)]
