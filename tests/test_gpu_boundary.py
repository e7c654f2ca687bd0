"""GPU parity of the drop-in boundary's semantics and of the
two configs decoded at their full size:

* DecompressionStream has no output cap (src/mod/streams.ts:46,132-182): the
  default batch decode returns any member whole (zs_inflate_batch_auto);
* formats and levels map as streams.ts:220-221,233 (unknown -> windowBits 15,
  a non-number level -> the default);
* the per-stream check value is the reference's strm.adler after the stream
  (deflate.ts:155-159,462; inflate.ts:105,1014,1080);
* the multi-GPU pool (device mask) returns what one device returns;
* C3 -- all 65,536 members -- and C5-i -- the gunzip of all 8,192 gzip
  members with their CRC-32 -- decode to their sources.
"""
import ctypes
import hashlib
import os
import zlib

import pytest

import corpus
import golden_io
import oracle

pytestmark = pytest.mark.gpu


def test_default_decode_is_unbounded(engine):
    """zeros_100k.deflate64 (369 B -> 100,000 B, the reference's test/data) and a
    1 MiB zero stream in every format decode with default options."""
    z64 = open(os.path.join(golden_io.GOLDEN, "d64", "zeros_100k.deflate64"), "rb").read()
    assert engine.decompress_batch([z64], "deflate64-raw") == [bytes(100000)]
    zeros = bytes(1 << 20)
    for fmt in ("deflate-raw", "deflate", "gzip"):
        comp = engine.compress_batch([zeros, b"", b"x" * 70000], fmt, 6)
        assert len(comp[0]) < 2000  # ratio > 500: far beyond any first-pass capacity guess
        assert engine.decompress_batch(comp, fmt) == [zeros, b"", b"x" * 70000]
    # mixed batch: small and huge ratios, corrupt members keep their reference errors
    srcs = [bytes(3 << 20), corpus.text(corpus.stream_seed(5), 65536), bytes(200000), b"abc"]
    comps = [oracle.compress(s, 9, "deflate-raw")[1] for s in srcs]
    bad = bytearray(comps[2])
    bad[len(bad) // 2] ^= 0x40
    comps.append(bytes(bad))
    res = engine.decompress_batch_raw(comps, "deflate-raw")
    for s, (st, ph, msg, out, cons) in zip(srcs, res):
        assert st == 1 and out == s
    ost, oout, ocons, oph, omsg = oracle.decompress(comps[4], "deflate-raw", cap=1 << 22)
    st, ph, msg, out, cons = res[4]
    assert (st, ph, msg) == (ost, oph, omsg)
    assert msg != "output capacity exceeded"


def test_explicit_cap_is_a_cap(engine):
    c = oracle.compress(bytes(100000), 6, "deflate-raw")[1]
    (st, ph, msg, out, cons), = engine.decompress_batch_raw([c], "deflate-raw", out_caps=[1000])
    assert st == -5 and msg == "output capacity exceeded"


def test_format_and_level_fall_through(engine):
    xs = [corpus.text(corpus.stream_seed(i), 20000 + i) for i in range(3)]
    assert engine.compress_batch(xs, "bogus", 6) == engine.compress_batch(xs, "deflate", 6)
    assert engine.compress_batch(xs, "deflate-raw", "9") == engine.compress_batch(xs, "deflate-raw", 6)
    assert engine.compress_batch(xs, "deflate-raw", None) == engine.compress_batch(xs, "deflate-raw", -1)
    comp = engine.compress_batch(xs, "deflate", 6)
    assert engine.decompress_batch(comp, "no-such-format") == xs


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_check_values_are_strm_adler(engine, fmt):
    xs = [b"", b"hello", corpus.text(corpus.stream_seed(3), 65536), corpus.rand(4, 100000)]
    for level in (0, 1, 6, 9):
        res = engine.compress_batch_detailed(xs, fmt, level)
        for x, (st, out, chk) in zip(xs, res):
            want = {"deflate-raw": 1, "deflate": zlib.adler32(x), "gzip": zlib.crc32(x)}[fmt]
            assert st == 1 and chk == want, (fmt, level, len(x))
        back = engine.decompress_batch_detailed([o for _, o, _ in res], fmt)
        for x, (st, ph, msg, out, cons, chk) in zip(xs, back):
            want = {"deflate-raw": 0, "deflate": zlib.adler32(x), "gzip": zlib.crc32(x)}[fmt]
            assert st == 1 and out == x and chk == want


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_level0_short_capacity_reports_buf_error_and_writes_nothing(engine, fmt):
    """Level 0 (zs_k_stored) with a capacity below its output: Z_BUF_ERROR,
    out_len 0, and no byte of the output region is touched -- the other levels'
    rule (zs_k_finish)."""
    import torch
    import zsamd

    data = [corpus.text(corpus.stream_seed(1), 50000), corpus.text(corpus.stream_seed(2), 40000)]
    blob = b"".join(data)
    d_in = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    caps = [1024, zsamd.deflate_capacity(40000, fmt)]
    d_out = torch.full((caps[0] + caps[1] + 4096,), 0xA5, dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(2, dtype=torch.int32, device="cuda")
    d_len = torch.zeros(2, dtype=torch.int32, device="cuda")
    u64, u32 = ctypes.c_uint64 * 2, ctypes.c_uint32 * 2
    engine.compress_device(0, fmt, 2, d_in.data_ptr(), u64(0, 50000), u32(50000, 40000), d_out.data_ptr(),
                           u64(0, caps[0]), u32(*caps), d_st.data_ptr(), d_len.data_ptr())
    torch.cuda.synchronize()
    assert d_st.tolist() == [-5, 1] and d_len.tolist()[0] == 0
    assert bool((d_out[:caps[0]] == 0xA5).all())  # the failed stream wrote nothing
    o = d_out[caps[0]: caps[0] + d_len.tolist()[1]].cpu().numpy().tobytes()
    # the stream layer's stored layout (32 KiB sub-chunks + the final remainder, deflate.ts:1140-1279;
    # pinned against the reference in test_level0_stored_layout_matches_reference_goldens)
    wrap = {"deflate-raw": 0, "deflate": 6, "gzip": 18}[fmt]
    assert len(o) == wrap + 5 * (40000 // 32768 + 1) + 40000
    st, out, *_ = oracle.decompress(o, fmt, cap=65536)
    assert st == 1 and out == data[1]
    # the host path reports the same and leaves the caller's bytes alone
    st = engine.compress_batch_raw(data, fmt, 0)
    assert [s for s, _ in st] == [1, 1]


def test_pool_on_one_device_equals_engine(engine):
    import zsamd

    pool = zsamd.Pool([0])
    assert pool.devices == [0]
    xs = [corpus.text(corpus.stream_seed(i), 65536) for i in range(64)] + [b"", b"abc"]
    for fmt in ("deflate-raw", "gzip"):
        a = pool.compress_batch_detailed(xs, fmt, 6)
        assert a == engine.compress_batch_detailed(xs, fmt, 6)
        back = pool.decompress_batch([o for _, o, _ in a], fmt)
        assert back == xs
    with pytest.raises(ValueError):
        zsamd.Pool([63])  # no such device
    pool.close()


def test_pool_on_every_visible_device_equals_engine(engine):
    """zs_pool over every visible device (mask 0): the batch is sharded across
    them (8 on the driver's node, 1 here) and must return what one engine does."""
    import torch
    import zsamd

    pool = zsamd.Pool()
    assert pool.devices == list(range(torch.cuda.device_count()))
    xs = [corpus.text(corpus.stream_seed(i), 65536) for i in range(48)] + [corpus.mixed(5, 200000)]
    a = pool.compress_batch_detailed(xs, "gzip", 6)
    assert a == engine.compress_batch_detailed(xs, "gzip", 6)
    comps = [o for _, o, _ in a]
    # (the M-corpus member may meet the reference's window-wrap copy: compare outcomes, not sources)
    assert pool.decompress_batch_raw(comps, "gzip") == engine.decompress_batch_raw(comps, "gzip")
    assert pool.decompress_batch(comps[:48], "gzip") == xs[:48]
    pool.close()


def test_pool_sharding_rehearsed_with_two_contexts_on_one_device(engine):
    """The pool's sharding (contiguous shard_range ranges, one host thread per
    context, each writing its shard straight into the caller's arrays) with two
    contexts on device 0 -- the multi-device code path without a second GPU."""
    import zsamd

    pool = zsamd.Pool([0, 0], repeat=True)
    assert pool.devices == [0, 0]
    xs = [corpus.text(corpus.stream_seed(i), 65536) for i in range(37)] + [b"", corpus.mixed(9, 262144)]
    for fmt in ("deflate-raw", "deflate"):
        a = pool.compress_batch_detailed(xs, fmt, 6)
        assert a == engine.compress_batch_detailed(xs, fmt, 6)
        comps = [o for _, o, _ in a]
        assert pool.decompress_batch_raw(comps, fmt) == engine.decompress_batch_raw(comps, fmt)
        assert pool.decompress_batch(comps[:38], fmt) == xs[:38]
        caps = [len(x) + 8 for x in xs]
        assert pool.decompress_batch_detailed(comps, fmt, caps) == engine.decompress_batch_detailed(comps, fmt, caps)
    pool.close()
    with pytest.raises(ValueError):
        zsamd.Pool([0, 999], repeat=True)


@pytest.mark.slow
def test_c3_all_65536_members_decode(engine):
    """BASELINE.json configs[2] at its full size: the 4,096 unique M-corpus
    members (pinned by the reference golden batch_m64_l6_raw) x 16 = 65,536
    members in one batch, default lane_block, every output equal to its source."""
    import torch
    import zsamd

    recs = golden_io.batch("m64_l6_raw")
    S, R, L = 4096, 16, 65536
    host = zsamd.corpus("mixed", 0, S, L)
    src = [bytes(host[i * L:(i + 1) * L]) for i in range(S)]
    comp = engine.compress_batch(src, "deflate-raw", 6)
    bad = [i for i, c in enumerate(comp) if (len(c), hashlib.sha256(c).digest()[:16]) != recs[i]]
    assert not bad, bad[:10]
    assert sum(len(c) for c in comp) == 123877078
    members = comp * R
    blob = b"".join(members)
    N = len(members)
    offs, o = [], 0
    for m in members:
        offs.append(o)
        o += len(m)
    d_in = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    d_out = torch.zeros(N * L, dtype=torch.uint8, device="cuda")
    i32 = lambda: torch.zeros(N, dtype=torch.int32, device="cuda")
    d_st, d_ph, d_msg, d_len, d_cons = i32(), i32(), i32(), i32(), i32()
    engine.decompress_device("deflate-raw", N, d_in.data_ptr(), (ctypes.c_uint64 * N)(*offs),
                             (ctypes.c_uint32 * N)(*[len(m) for m in members]), d_out.data_ptr(),
                             (ctypes.c_uint64 * N)(*[i * L for i in range(N)]), (ctypes.c_uint32 * N)(*([L] * N)),
                             d_st.data_ptr(), d_ph.data_ptr(), d_msg.data_ptr(), d_len.data_ptr(), d_cons.data_ptr())
    torch.cuda.synchronize()
    assert int((d_st != 1).sum()) == 0
    assert int((d_len != L).sum()) == 0
    assert d_cons.tolist() == [len(m) for m in members]
    want = torch.frombuffer(host, dtype=torch.uint8).cuda().view(1, S, L)
    same = (d_out.view(R, S, L) == want).all(dim=2)
    assert bool(same.all()), [(int(r), int(s)) for r, s in (~same).nonzero()[:10]]
    assert engine.last_lane_count() == N  # every member on the lane fast path


@pytest.mark.slow
def test_c5_gunzip_all_8192_members_with_crc(engine):
    """C5-i decode at its full size: the 8,192 gzip L6 members (pinned by the
    reference golden batch_t64_l6_gzip) gunzipped in one batch, each output equal
    to its source, each trailer's CRC-32 verified by the engine and returned as the
    check value (= zlib.crc32 of the source)."""
    import torch
    import zsamd

    recs = golden_io.batch("t64_l6_gzip")
    N, L = 8192, 65536
    host = zsamd.corpus("text", 0, N, L)
    src = [bytes(host[i * L:(i + 1) * L]) for i in range(N)]
    gz = []
    for lo in (0, 4096):
        gz += engine.compress_batch(src[lo:lo + 4096], "gzip", 6)
    bad = [i for i, c in enumerate(gz) if (len(c), hashlib.sha256(c).digest()[:16]) != recs[i]]
    assert not bad, bad[:10]
    blob = b"".join(gz)
    offs, o = [], 0
    for m in gz:
        offs.append(o)
        o += len(m)
    d_in = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    d_out = torch.zeros(N * L, dtype=torch.uint8, device="cuda")
    i32 = lambda: torch.zeros(N, dtype=torch.int32, device="cuda")
    d_st, d_ph, d_msg, d_len, d_cons, d_chk = i32(), i32(), i32(), i32(), i32(), i32()
    lib = engine._L
    r = lib.zs_inflate_batch_device_ex(engine.handle, 31, N, ctypes.c_void_p(d_in.data_ptr()),
                                       (ctypes.c_uint64 * N)(*offs), (ctypes.c_uint32 * N)(*[len(m) for m in gz]),
                                       ctypes.c_void_p(d_out.data_ptr()),
                                       (ctypes.c_uint64 * N)(*[i * L for i in range(N)]),
                                       (ctypes.c_uint32 * N)(*([L] * N)), ctypes.c_void_p(d_st.data_ptr()),
                                       ctypes.c_void_p(d_ph.data_ptr()), ctypes.c_void_p(d_msg.data_ptr()),
                                       ctypes.c_void_p(d_len.data_ptr()), ctypes.c_void_p(d_cons.data_ptr()),
                                       ctypes.c_void_p(d_chk.data_ptr()), None)
    assert r == 0
    torch.cuda.synchronize()
    assert int((d_st != 1).sum()) == 0 and int((d_len != L).sum()) == 0
    assert bool((d_out.view(N, L) == torch.frombuffer(host, dtype=torch.uint8).cuda().view(N, L)).all())
    chk = [c & 0xffffffff for c in d_chk.tolist()]
    assert chk == [zlib.crc32(s) for s in src]
    assert d_cons.tolist() == [len(m) for m in gz]


def test_large_members_decode_as_the_reference(engine):
    """4,096 T-corpus 256 KiB streams at deflate-raw L6 (compressed here and
    checked against the reference's compress golden) decoded with default
    options, as DecompressionStream decodes them: ~100 KB of input each, so
    every member is "large" and takes the path the host picks for a batch of
    4,096 large members (capi.cpp), which tracks the reference's inflate()
    calls (32 KiB input sub-chunks, 64 KiB output buffers, streams.ts:78-93)
    and reproduces the window-wrap copy of inffast.ts:127-147.  Bytes =
    tests/golden/batch_t256_l6_raw_dec.bin (the reference's own decode; it
    differs from the source for some members); no member falls back to the
    exact kernel; the exact kernel agrees on the members the copy changes.
    The per-rank shard sizes of the 8-GPU configs are test_large_member_shard_*."""
    import zsamd

    L, N = 262144, 4096
    buf = bytes(zsamd.corpus("text", 0, N, L))
    srcs = [buf[i * L:(i + 1) * L] for i in range(N)]
    comps = engine.compress_batch(srcs, "deflate-raw", 6)
    recs = golden_io.batch("t256_l6_raw")
    assert all((len(c), hashlib.sha256(c).digest()[:16]) == recs[i] for i, c in enumerate(comps))
    assert min(len(c) for c in comps) > 32768
    outs = engine.decompress_batch(comps, "deflate-raw", [L] * N)
    assert engine.last_lane_count() == N
    assert engine.last_seg_count() == N  # every member finished by the segmented decode (inflate_seg.hip)
    drecs = golden_io.batch("t256_l6_raw_dec")
    assert all((len(o), hashlib.sha256(o).digest()[:16]) == drecs[i] for i, o in enumerate(outs))
    changed = [i for i in range(N) if outs[i] != srcs[i]]
    assert changed  # the set exercises the window-wrap copy
    try:
        engine.set_option("inflate_fast", 0)  # the exact kernel for every member
        exact = engine.decompress_batch([comps[i] for i in changed], "deflate-raw", [L] * len(changed))
        assert engine.last_lane_count() == 0
    finally:
        engine.set_option("inflate_fast", 1)
    assert all(exact[k] == outs[i] for k, i in enumerate(changed))


def _t256_l6_raw(engine, lo, hi):
    import zsamd

    L = 262144
    buf = bytes(zsamd.corpus("text", lo, hi - lo, L))
    srcs = [buf[i * L:(i + 1) * L] for i in range(hi - lo)]
    comps = engine.compress_batch(srcs, "deflate-raw", 6)
    recs = golden_io.batch("t256_l6_raw")[lo:hi]
    assert all((len(c), hashlib.sha256(c).digest()[:16]) == r for c, r in zip(comps, recs))
    return srcs, comps


@pytest.mark.parametrize("n", [512, 64, 1])
def test_large_member_shard_decodes_as_the_reference(engine, n):
    """BASELINE configs[3] at the per-rank size of 8 GPUs: a shard of the 4,096
    T-corpus 256 KiB L6 streams (streams 0..n-1) decoded with default options
    -- the path the host picks for a batch of few large members -- against the
    reference's OWN decode of each (batch_t256_l6_raw_dec.bin, DecompressionStream
    with one write(), window-wrap copy of inffast.ts:127-147 included), every
    member finished without the exact kernel."""
    L = 262144
    srcs, comps = _t256_l6_raw(engine, 0, n)
    outs = engine.decompress_batch(comps, "deflate-raw", [L] * n)
    assert engine.last_lane_count() == n
    assert engine.last_seg_count() == n  # the segmented decode finished every member
    drecs = golden_io.batch("t256_l6_raw_dec")[:n]
    bad = [i for i, o in enumerate(outs) if (len(o), hashlib.sha256(o).digest()[:16]) != drecs[i]]
    assert not bad, bad[:10]


def test_mixed_large_members_with_window_wrap_copies(engine):
    """M-corpus members of 200-500 KB at L6 / L9: the reference's window-wrap
    copy (inffast.ts:127-147) fires in most of them (short inflate() calls in
    output over the incompressible kilobytes).  Every member equals the oracle
    with the reference's defect (reference_bugs) and the exact kernel."""
    import random

    rng = random.Random(2024)
    members, caps, want, srcs = [], [], [], []
    for k in range(24):
        n = rng.choice([200000, 262144, 500000])
        s = corpus.mixed(corpus.stream_seed(rng.randrange(4096)), n)
        c = oracle.compress(s, rng.choice([6, 9]), "deflate-raw")[1]
        members.append(c)
        srcs.append(s)
        caps.append((n + 3) & ~3)
        want.append(oracle.decompress(c, "deflate-raw", cap=n, reference_bugs=True))
    assert any(w[1] != s for w, s in zip(want, srcs))  # the set exercises the window-wrap copy
    got = engine.decompress_batch_raw(members, "deflate-raw", caps)
    assert engine.last_lane_count() == len(members)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g[0] == 1 and g[3] == w[1] and g[4] == w[2], i
    try:
        engine.set_option("inflate_fast", 0)
        exact = engine.decompress_batch_raw(members, "deflate-raw", caps)
    finally:
        engine.set_option("inflate_fast", 1)
    assert exact == got


@pytest.mark.slow
def test_c5_gunzip_shard_of_1024_members(engine):
    """C5-i at the per-rank size of 8 GPUs: gzip members 0..1023 of the C5 set
    (pinned by the reference golden batch_t64_l6_gzip) gunzipped with default
    options, each equal to its source with its CRC-32 check value."""
    import zsamd

    N, L = 1024, 65536
    host = zsamd.corpus("text", 0, N, L)
    src = [bytes(host[i * L:(i + 1) * L]) for i in range(N)]
    gz = engine.compress_batch(src, "gzip", 6)
    recs = golden_io.batch("t64_l6_gzip")[:N]
    assert all((len(c), hashlib.sha256(c).digest()[:16]) == r for c, r in zip(gz, recs))
    res = engine.decompress_batch_detailed(gz, "gzip", [L] * N)
    assert engine.last_lane_count() == N
    assert engine.last_seg_count() == N  # the per-rank shard runs on the segmented decode
    for s, r in zip(src, res):
        assert r[0] == 1 and r[3] == s and (r[5] & 0xffffffff) == zlib.crc32(s)


def test_c5_deflate64_shard_of_rank_0(engine):
    """C5-ii at the per-rank size of 8 GPUs, built as bench.py builds it: the 8,192 T-corpus raw-L6 members
    (pinned by the reference golden batch_t64_l6_raw) with the reference's test/data deflate64 fixtures interleaved
    (inflate_small.json digests), sharded by shard_range; rank 0's 1,025 entries decoded as deflate64-raw with
    default options, every corpus member equal to its source and every fixture to its digest."""
    import json
    import os
    import zsamd
    import zsamd.shard as shard

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = json.load(open(os.path.join(root, "tests", "golden", "inflate_small.json")))
    fx = [(open(os.path.join(root, "tests", "golden", "d64", c["name"][4:]), "rb").read(), c["out_len"],
           c["out_sha256"]) for c in g["cases"] if c["name"].startswith("d64_") and c.get("ok")]
    S, L = 8192, 65536
    gstep = S // len(fx)
    entries = []
    for i in range(S):
        if i % gstep == gstep // 2 and i // gstep < len(fx):
            entries.append(("f", i // gstep))
        entries.append(("u", i))
    lo, hi = shard.shard_range(len(entries), 8, 0)
    mine = entries[lo:hi]
    us = [e[1] for e in mine if e[0] == "u"]
    host = zsamd.corpus("text", us[0], len(us), L)
    src = {u: bytes(host[k * L:(k + 1) * L]) for k, u in enumerate(us)}
    comp = dict(zip(us, engine.compress_batch([src[u] for u in us], "deflate-raw", 6)))
    recs = golden_io.batch("t64_l6_raw")
    assert all((len(comp[u]), hashlib.sha256(comp[u]).digest()[:16]) == recs[u] for u in us)
    members = [comp[e[1]] if e[0] == "u" else fx[e[1]][0] for e in mine]
    caps = [L if e[0] == "u" else (fx[e[1]][1] + 3) & ~3 for e in mine]
    res = engine.decompress_batch_raw(members, "deflate64-raw", caps)
    assert len(mine) == 1025 and sum(1 for e in mine if e[0] == "f") >= 1
    for e, r in zip(mine, res):
        assert r[0] == 1, e
        if e[0] == "u":
            assert r[3] == src[e[1]], e
        else:
            assert len(r[3]) == fx[e[1]][1] and hashlib.sha256(r[3]).hexdigest() == fx[e[1]][2], e


def test_device_inflate_rejects_unaligned_capacities(engine):
    """The device entry points' output capacities are multiples of 4 (the decoders store whole words): an
    unaligned one is ZS_STREAM_ERROR before anything runs; the host entry takes any capacity."""
    import torch
    import zsamd

    comp = engine.compress_batch([b"hello hello hello"], "deflate-raw", 6)[0]
    d_in = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    d_out = torch.zeros(64, dtype=torch.uint8, device="cuda")
    i32 = lambda: torch.zeros(1, dtype=torch.int32, device="cuda")
    bufs = [i32() for _ in range(5)]
    args = ("deflate-raw", 1, d_in.data_ptr(), (ctypes.c_uint64 * 1)(0), (ctypes.c_uint32 * 1)(len(comp)),
            d_out.data_ptr(), (ctypes.c_uint64 * 1)(0))
    with pytest.raises(zsamd.ZsError):
        engine.decompress_device(*args, (ctypes.c_uint32 * 1)(17), *[b.data_ptr() for b in bufs])
    engine.decompress_device(*args, (ctypes.c_uint32 * 1)(20), *[b.data_ptr() for b in bufs])
    torch.cuda.synchronize()
    assert int(bufs[0][0]) == 1 and bytes(d_out[:17].cpu().numpy()) == b"hello hello hello"
    assert engine.decompress_batch([comp], "deflate-raw", [17]) == [b"hello hello hello"]


@pytest.mark.gpu
def test_host_inflate_takes_exact_unaligned_capacities(engine):
    """zs_inflate_batch (the C host entry, called directly through ctypes, no Python rounding) takes any capacity
    and any output offset: a 17-byte member fits a capacity of 17 at offset 0, an 18-byte member with a capacity of
    17 is Z_BUF_ERROR "output capacity exceeded" (the exact cap, not one rounded up to a word), and a member at the
    unaligned offset 34 decodes in place (capi.cpp inflate_device's caller_regions)."""
    L = engine._L
    a, b = b"hello hello hello", b"hello hello hello!"
    comps = [oracle.compress(x, 6, "deflate-raw")[1] for x in (a, b, a)]
    blob = b"".join(comps)
    n = len(comps)
    in_off = (ctypes.c_uint64 * n)(0, len(comps[0]), len(comps[0]) + len(comps[1]))
    in_len = (ctypes.c_uint32 * n)(*map(len, comps))
    out_off = (ctypes.c_uint64 * n)(0, 17, 34)
    out_cap = (ctypes.c_uint32 * n)(17, 17, 17)
    out = ctypes.create_string_buffer(51)
    st, ph, msg = [(ctypes.c_int32 * n)() for _ in range(3)]
    olen, cons = [(ctypes.c_uint32 * n)() for _ in range(2)]
    r = L.zs_inflate_batch(engine._ctx, -15, n, blob, in_off, in_len, out, out_off, out_cap, st, ph, msg, olen, cons)
    assert r == 0
    assert list(st) == [1, -5, 1]
    assert L.zs_inflate_message(msg[1]).decode() == "output capacity exceeded"
    assert out.raw[0:17] == a and out.raw[34:51] == a and list(olen)[0::2] == [17, 17]
    # the same through the Python mirror: exact caps, not rounded
    res = engine.decompress_batch_raw([comps[0], comps[1]], "deflate-raw", out_caps=[17, 17])
    assert [x[0] for x in res] == [1, -5] and res[0][3] == a
    # zs_deflate_batch likewise: a capacity of exactly the output's length (unaligned) fits, one byte less is
    # Z_BUF_ERROR, and the streams land at unaligned offsets
    src = [b"abcabcabcabcabcabcabc xyz", b"the quick brown fox jumps"]
    want = [oracle.compress(x, 6, "deflate-raw")[1] for x in src]
    ln = [len(w) for w in want]
    for caps, ok in (([ln[0], ln[1]], [1, 1]), ([ln[0] - 1, ln[1]], [-5, 1])):
        n = 2
        blob2 = b"".join(src)
        out2 = ctypes.create_string_buffer(sum(caps) + 1)
        st2 = (ctypes.c_int32 * n)()
        ol2 = (ctypes.c_uint32 * n)()
        r = L.zs_deflate_batch(engine._ctx, 6, -15, n, blob2, (ctypes.c_uint64 * n)(0, len(src[0])),
                               (ctypes.c_uint32 * n)(*map(len, src)), out2, (ctypes.c_uint64 * n)(1, 1 + caps[0]),
                               (ctypes.c_uint32 * n)(*caps), st2, ol2)
        assert r == 0 and list(st2) == ok
        for i in range(n):
            if ok[i] == 1:
                o = 1 + sum(caps[:i])
                assert ol2[i] == ln[i] and out2.raw[o:o + ln[i]] == want[i]


@pytest.mark.gpu
def test_host_batch_packs_produced_bytes_over_several_chunks(engine):
    """The host-buffer decode of a batch of >= 32 MB input runs as four chunks and packs each chunk's outputs by the
    bytes produced, not by capacity: a last chunk that expands far past 4x the batch input grows the pack buffers
    once the chunks before it are scattered, and every member comes back exact (capi.cpp host_batch_run)."""
    import numpy as np

    rng = np.random.default_rng(5)
    srcs = [rng.integers(0, 256, 600_000, dtype=np.uint8).tobytes() for _ in range(56)] + [bytes(40 << 20)] * 8
    comp = engine.compress_batch(srcs, "deflate-raw", 1)
    assert sum(map(len, comp)) >= 32 << 20
    got = engine.decompress_batch(comp, "deflate-raw", [len(s) for s in srcs])
    assert [len(g) for g in got] == [len(s) for s in srcs]
    assert all(g == s for g, s in zip(got, srcs))
