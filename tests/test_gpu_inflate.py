"""GPU parity: the HIP inflate engine against the reference's goldens and the oracle
(the reference's DecompressionStream semantics: status, phase, message, bytes)."""
import hashlib
import json
import os
import random

import pytest

import corpus
import golden_io
import oracle

pytestmark = pytest.mark.gpu


def _err(st, ph):
    return "" if st == 1 else oracle.stream_error_text(st, ph)


def test_inflate_small_goldens(engine):
    items = [(c, d) for c, d in golden_io.inflate_cases() if d is not None]
    by_fmt = {}
    for c, d in items:
        by_fmt.setdefault(c["format"], []).append((c, d))
    bad = []
    for fmt, its in by_fmt.items():
        res = engine.decompress_batch_raw([d for _, d in its], fmt, out_caps=[max(1 << 17, 40 * len(d)) for _, d in its])
        for (c, d), (st, ph, msg, out, cons) in zip(its, res):
            ok = st == 1
            if ok != c["ok"] or _err(st, ph) != c["err"] or corpus.sha256(out) != c["out_sha256"]:
                bad.append((c["name"], st, ph, msg, c["err"], len(out), c["out_len"]))
    assert not bad, bad


def test_inflate_errors_match_oracle_messages(engine):
    items = [(c, d) for c, d in golden_io.inflate_cases() if d is not None and c["name"].startswith("corrupt_")]
    for fmt in ("deflate-raw", "deflate", "gzip"):
        its = [(c, d) for c, d in items if c["format"] == fmt]
        res = engine.decompress_batch_raw([d for _, d in its], fmt, out_caps=[1 << 17] * len(its))
        for (c, d), (st, ph, msg, out, cons) in zip(its, res):
            ost, oout, ocons, oph, omsg = oracle.decompress(d, fmt, cap=1 << 18)
            assert (st, ph, msg, out) == (ost, oph, omsg, oout), c["name"]
            if st == 1:
                assert cons == ocons


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_roundtrip_random_inputs(engine, fmt):
    rng = random.Random(77)
    srcs = []
    for k in range(40):
        n = rng.choice([0, 1, 5, 258, 259, 4096, 32768, 65536, 100000, rng.randrange(1, 300000)])
        srcs.append(corpus.make({"kind": rng.choice(["text", "mixed", "rand", "zeros"]), "n": n,
                                 "seed": rng.randrange(1 << 32)}))
    comps = [oracle.compress(s, rng.choice([1, 6, 9]), fmt)[1] for s in srcs]
    # default: the reference's bytes, including its inflate_fast window-wrap copy (inffast.ts:133-147)
    res = engine.decompress_batch_raw(comps, fmt, out_caps=[len(s) + 64 for s in srcs])
    for s, c, (st, ph, msg, out, cons) in zip(srcs, comps, res):
        ost, oout, ocons, oph, omsg = oracle.decompress(c, fmt, cap=len(s) + 64)
        assert (st, ph, msg, out, cons) == (ost, oph, omsg, oout, ocons), (len(s), st, ph, msg)
    # inflate_ref_wrap = 0: zlib semantics, the source bytes
    try:
        engine.set_option("inflate_ref_wrap", 0)
        res = engine.decompress_batch_raw(comps, fmt, out_caps=[len(s) + 64 for s in srcs])
    finally:
        engine.set_option("inflate_ref_wrap", 1)
    for s, c, (st, ph, msg, out, cons) in zip(srcs, comps, res):
        assert st == 1 and out == s and cons == len(c), (len(s), st, ph, msg)


def test_trailing_garbage_and_second_member_ignored(engine):
    a = oracle.compress(b"first member ", 6, "gzip")[1]
    b = oracle.compress(b"second", 6, "gzip")[1]
    res = engine.decompress_batch_raw([a + b, a + b"garbage"], "gzip")
    assert res[0][3] == b"first member " and res[0][4] == len(a)
    assert res[1][3] == b"first member " and res[1][4] == len(a)
    r = oracle.compress(b"raw data", 6, "deflate-raw")[1]
    res = engine.decompress_batch_raw([r + b"\x00\xff junk"], "deflate-raw")
    assert res[0][0] == 1 and res[0][3] == b"raw data"


def test_deflate64_fixtures_and_kats(engine):
    names = sorted(os.listdir(os.path.join(golden_io.GOLDEN, "d64")))
    data = [open(os.path.join(golden_io.GOLDEN, "d64", f), "rb").read() for f in names]
    res = engine.decompress_batch_raw(data, "deflate64-raw", out_caps=[3 << 20] * len(data))
    cases = {c["name"]: c for c, _ in golden_io.inflate_cases()}
    for f, (st, ph, msg, out, cons) in zip(names, res):
        c = cases["d64_" + f]
        assert st == 1 and corpus.sha256(out) == c["out_sha256"], f
    # test-inflate9-length-code-285.spec.ts:9-15
    (st, ph, msg, out, cons), = engine.decompress_batch_raw([bytes.fromhex("4b1cfdff07a3e5030000")], "deflate64-raw",
                                                            out_caps=[70000])
    assert st == 1 and out == b"a" * 66539
    (st, ph, msg, out, cons), = engine.decompress_batch_raw([bytes.fromhex("4b1c0500")], "deflate-raw")
    assert st == 1 and out == b"a" * 259


@pytest.mark.parametrize("lane_block", [0, 1, 8, 64])
def test_deflate64_lane_path_fixtures(engine, lane_block):
    """The reference's deflate64 fixtures (distances > 32 KiB, codes 30/31,
    length 285 with 16 extra bits) through the lane decoder at several
    workgroup shapes, against the reference's output hashes."""
    names = sorted(os.listdir(os.path.join(golden_io.GOLDEN, "d64")))
    data = [open(os.path.join(golden_io.GOLDEN, "d64", f), "rb").read() for f in names]
    data.append(bytes.fromhex("4b1cfdff07a3e5030000"))  # test-inflate9-length-code-285.spec.ts:9-15
    cases = {c["name"]: c for c, _ in golden_io.inflate_cases()}
    try:
        engine.set_option("lane_block", lane_block)
        res = engine.decompress_batch_raw(data * 3, "deflate64-raw", out_caps=[3 << 20] * (3 * len(data)))
    finally:
        engine.set_option("lane_block", 0)
    for i, (st, ph, msg, out, cons) in enumerate(res):
        k = i % len(data)
        if k == len(names):
            assert st == 1 and out == b"a" * 66539
        else:
            assert st == 1 and corpus.sha256(out) == cases["d64_" + names[k]]["out_sha256"], names[k]


@pytest.mark.slow
def test_c5_deflate64_decode_8192_streams(engine):
    """C5-ii: the 8,192 T-corpus deflate-raw L6 streams --
    the bodies of the C5 gzip members, pinned by the reference's golden hashes --
    decoded as deflate64-raw give back their sources (no length-258 match, so
    they are valid deflate64 with identical output), interleaved with the
    reference's deflate64 fixtures."""
    import zsamd

    recs = golden_io.batch("t64_l6_gzip")
    n = len(recs)
    buf = bytes(zsamd.corpus("text", 0, n, 65536))
    srcs = [buf[i * 65536:(i + 1) * 65536] for i in range(n)]
    gz = engine.compress_batch(srcs, "gzip", 6)
    bad = [i for i, c in enumerate(gz) if (len(c), hashlib.sha256(c).digest()[:16]) != recs[i]]
    assert not bad, bad[:10]
    raw = [c[10:-8] for c in gz]
    names = sorted(os.listdir(os.path.join(golden_io.GOLDEN, "d64")))
    fx = [open(os.path.join(golden_io.GOLDEN, "d64", f), "rb").read() for f in names]
    cases = {c["name"]: c for c, _ in golden_io.inflate_cases()}
    fcap = [cases["d64_" + f]["out_len"] + 64 for f in names]
    items, caps = [], []
    for i, r in enumerate(raw):
        items.append(r)
        caps.append(65536 + 64)
        if i % 1024 == 0:
            items.extend(fx)
            caps.extend(fcap)
    res = engine.decompress_batch_raw(items, "deflate64-raw", out_caps=caps)
    outs = iter(res)
    for i in range(n):
        st, ph, msg, out, cons = next(outs)
        assert st == 1 and out == srcs[i], i
        if i % 1024 == 0:
            for f in names:
                st, ph, msg, out, cons = next(outs)
                assert st == 1 and corpus.sha256(out) == cases["d64_" + f]["out_sha256"], f


def test_capacity_too_small(engine):
    c = oracle.compress(bytes(100000), 6, "deflate-raw")[1]
    (st, ph, msg, out, cons), = engine.decompress_batch_raw([c], "deflate-raw", out_caps=[1000])
    assert st == -5 and ph == 0 and msg == "output capacity exceeded"


def test_inffast_window_wrap_defect_is_reproduced(engine):
    """tests/golden/inffast_wrap_defect.json: a 256 KiB M-corpus stream that the
    reference itself decodes to DIFFERENT bytes than its source (inffast.ts:133-147
    copies from output[0..] instead of window[0..]).  The engine returns the
    reference's bytes by default, and the source with inflate_ref_wrap = 0."""
    j = json.load(open(os.path.join(golden_io.GOLDEN, "inffast_wrap_defect.json")))
    src = corpus.make(j["source"])
    comp = oracle.compress(src, 6, "deflate-raw")[1]
    assert corpus.sha256(comp) == j["compressed_sha256"]
    (st, ph, msg, out, cons), = engine.decompress_batch_raw([comp], "deflate-raw", out_caps=[len(src) + 64])
    assert st == 1 and len(out) == j["ref_out_len"] and corpus.sha256(out) == j["ref_out_sha256"]
    assert out != src
    try:
        engine.set_option("inflate_ref_wrap", 0)
        (st, ph, msg, out, cons), = engine.decompress_batch_raw([comp], "deflate-raw", out_caps=[len(src) + 64])
    finally:
        engine.set_option("inflate_ref_wrap", 1)
    assert st == 1 and out == src


@pytest.mark.slow
def test_c3_members_decode(engine):
    """BASELINE.json configs[2] source: M-corpus 64 KiB members at L6, here 1024 of them."""
    import zsamd

    recs = golden_io.batch("m64_l6_raw")
    buf = bytes(zsamd.corpus("mixed", 0, 1024, 65536))
    srcs = [buf[i * 65536:(i + 1) * 65536] for i in range(1024)]
    comps = engine.compress_batch(srcs, "deflate-raw", 6)
    for i, c in enumerate(comps):
        assert (len(c), hashlib.sha256(c).digest()[:16]) == recs[i]
    outs = engine.decompress_batch(comps, "deflate-raw")
    assert outs == srcs


def _fast_vs_exact_corpus():
    rng = random.Random(2024)
    items = []
    for c, d in golden_io.inflate_cases():
        if d is not None:
            items.append((c["format"], d, max(1 << 17, 40 * len(d))))
    for k in range(80):
        # deflate64-raw over deflate-raw streams: valid deflate64 unless a
        # length-258 match appears (then a different, still deterministic decode)
        fmt = rng.choice(["deflate-raw", "deflate", "gzip", "deflate64-raw"])
        n = rng.choice([0, 1, 7, 258, 5000, 65536, 70000, rng.randrange(1, 200000)])
        src = corpus.make({"kind": rng.choice(["text", "mixed", "rand", "zeros", "ramp"]), "n": n,
                           "seed": rng.randrange(1 << 32)})
        comp = oracle.compress(src, rng.choice([1, 3, 6, 9]), "deflate-raw" if fmt == "deflate64-raw" else fmt)[1]
        cap = len(src) + 64
        variant = k % 6
        if variant == 1 and len(comp) > 4:
            comp = comp[: rng.randrange(1, len(comp))]  # truncated
        elif variant == 2:
            comp = comp + bytes(rng.randrange(256) for _ in range(9))  # trailing bytes
        elif variant == 3 and len(comp) > 8:
            b = bytearray(comp)
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)  # bit flip
            comp = bytes(b)
        elif variant == 4 and len(src) > 10:
            cap = (len(src) // 2 + 3) & ~3  # too small
        items.append((fmt, comp, cap))
    return items


def test_lane_fast_path_matches_exact_path(engine):
    """The lane-per-member decoder (inflate_fast option) and the exact stream-layer
    state machine agree on status, phase, message, bytes and consumed input."""
    items = _fast_vs_exact_corpus()
    for fmt in ("deflate-raw", "deflate", "gzip", "deflate64-raw"):
        its = [(d, cap) for f, d, cap in items if f == fmt]
        engine.set_option("inflate_fast", 1)
        fast = engine.decompress_batch_raw([d for d, _ in its], fmt, out_caps=[c for _, c in its])
        engine.set_option("inflate_fast", 0)
        exact = engine.decompress_batch_raw([d for d, _ in its], fmt, out_caps=[c for _, c in its])
        engine.set_option("inflate_fast", 1)
        for i, (a, b) in enumerate(zip(fast, exact)):
            assert a == b, (fmt, i, a[:3], b[:3], len(a[3]), len(b[3]), a[4], b[4])


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip", "deflate64-raw"])
def test_lane_path_decodes_clean_members(engine, fmt):
    """Clean members (one reference inflate() call: <= 32 KiB in, <= 64 KiB out)
    decode on the lane path, not through the exact fallback."""
    rng = random.Random(5)
    srcs = [corpus.make({"kind": k, "n": n, "seed": rng.randrange(1 << 32)})
            for k in ("text", "mixed", "zeros", "ramp") for n in (1, 100, 5000, 40000, 65536)]
    srcs.append(b"")
    enc = "deflate-raw" if fmt == "deflate64-raw" else fmt
    comps = [oracle.compress(s, lvl, enc)[1] for s, lvl in zip(srcs, [1, 6, 9] * 20)]
    # deflate64 over deflate streams: only those without a length-258 match are valid
    keep = [(s, c) for s, c in zip(srcs, comps)
            if len(c) <= 32768 and oracle.decompress(c, fmt, cap=len(s) + 64)[1] == s]
    res = engine.decompress_batch_raw([c for _, c in keep], fmt, out_caps=[len(s) + 64 for s, _ in keep])
    for (s, c), (st, ph, msg, out, cons) in zip(keep, res):
        assert st == 1 and out == s
    assert engine.last_lane_count() == len(keep)


def _decode_with(engine, items, fmt, caps, **opts):
    try:
        for k, v in opts.items():
            engine.set_option(k, v)
        return engine.decompress_batch_raw(items, fmt, out_caps=caps)
    finally:
        engine.set_option("inflate_wave_min", 32768)
        engine.set_option("inflate_ref_wrap", 1)
        engine.set_option("inflate_fast", 1)


def test_wave_path_deflate64_fixtures(engine):
    """Large members decode one per wave (inflate_wave.hip) beside the lane
    kernel: the reference's deflate64 fixtures (>32 KiB distances, codes 30/31,
    length 285) at every threshold -- all on the wave path (1), the default
    split, none (0) -- against the reference's output hashes."""
    names = sorted(os.listdir(os.path.join(golden_io.GOLDEN, "d64")))
    data = [open(os.path.join(golden_io.GOLDEN, "d64", f), "rb").read() for f in names]
    data.append(bytes.fromhex("4b1cfdff07a3e5030000"))  # test-inflate9-length-code-285.spec.ts:9-15
    cases = {c["name"]: c for c, _ in golden_io.inflate_cases()}
    caps = [3 << 20] * len(data)
    for wmin in (1, 4096, 32768, 0):
        res = _decode_with(engine, data, "deflate64-raw", caps, inflate_wave_min=wmin)
        assert engine.last_lane_count() == len(data), wmin  # every member ended on a fast path
        for k, (st, ph, msg, out, cons) in enumerate(res):
            if k == len(names):
                assert st == 1 and out == b"a" * 66539 and cons == len(data[k])
            else:
                c = cases["d64_" + names[k]]
                assert st == 1 and corpus.sha256(out) == c["out_sha256"], (wmin, names[k])
                assert cons == len(data[k])


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_wave_path_large_members_zlib_semantics(engine, fmt):
    """With the window-wrap reproduction off (inflate_ref_wrap=0), large members
    of the three formats -- text, mixed, runs, incompressible (stored blocks),
    fixed-Huffman -- decode on the wave path to their sources, and damaged ones
    (flipped bit, truncation, short capacity) report exactly what the exact
    state machine reports."""
    rng = random.Random(11)
    srcs = [corpus.make({"kind": k, "n": n, "seed": rng.randrange(1 << 32)})
            for k, n in (("text", 262144), ("mixed", 1 << 20), ("zeros", 2 << 20), ("rand", 300000),
                         ("ramp", 500000), ("text", 40000))]
    comps = [oracle.compress(s, lvl, fmt)[1] for s, lvl in zip(srcs, (6, 6, 9, 6, 1, 6))]
    comps.append(zlib_fixed(srcs[0], fmt))
    srcs.append(srcs[0])
    caps = [len(s) + 64 for s in srcs]
    res = _decode_with(engine, comps, fmt, caps, inflate_ref_wrap=0, inflate_wave_min=1)
    assert engine.last_lane_count() == len(comps)
    for i, (s, (st, ph, msg, out, cons)) in enumerate(zip(srcs, res)):
        assert st == 1 and out == s and cons == len(comps[i]), (fmt, i, st, msg)
    bad = []
    for c in comps[:3]:
        flip = bytearray(c)
        flip[len(c) // 2] ^= 0x10
        bad += [bytes(flip), c[: len(c) * 2 // 3]]
    bcaps = [len(srcs[0]) + 64, len(srcs[0]) + 64, len(srcs[1]) + 64, len(srcs[1]) + 64, 1 << 20, 1 << 20]
    bad.append(comps[0])
    bcaps.append(len(srcs[0]) // 2)  # output capacity too small
    wave = _decode_with(engine, bad, fmt, bcaps, inflate_ref_wrap=0, inflate_wave_min=1)
    exact = _decode_with(engine, bad, fmt, bcaps, inflate_ref_wrap=0, inflate_fast=0)
    for i, (a, b) in enumerate(zip(wave, exact)):
        assert a == b, (fmt, i, a[:3], b[:3], len(a[3]), len(b[3]), a[4], b[4])


def zlib_fixed(data, fmt):
    """A fixed-Huffman stream of `data` (Python's zlib with Z_FIXED): block type 1 at size."""
    import zlib
    wb = {"deflate-raw": -15, "deflate": 15, "gzip": 31}[fmt]
    co = zlib.compressobj(6, zlib.DEFLATED, wb, 8, zlib.Z_FIXED)
    return co.compress(data) + co.flush()


def test_wave_table_builder_equals_inflate_table(engine):
    """zs_inflate_table_wave (zs_inftab.h: the decoding tables of a dynamic header built by the 64 lanes of a wave
    -- ballot-sorted symbols, each root entry the canonical decode of its own bits, sub-tables sized and placed as
    inflate_table allocates them, inftrees.ts:62-279) against the serial inflate_table on 8,192 random complete
    code sets (literal/length, distance, code-length and deflate64 distance alphabets): same return value, root
    bits, size and every entry."""
    import ctypes

    L = engine._L
    L.zs_inftab_selfcheck.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_ulonglong)]
    bad = ctypes.c_ulonglong(0)
    assert L.zs_inftab_selfcheck(0, 12345, 256, 32, ctypes.byref(bad)) == 0
    assert bad.value == 0
