"""GPU parity of the split decode of large members (inflate_split.hip): a
member cut at its block boundaries, the pieces decoded in parallel with
markers for the unknown history, then resolved in order.  It must produce
exactly what the one-piece paths produce -- the wave kernel and the exact
stream-layer kernel (inflate.ts:332-1185) -- bytes, statuses, phases and
messages, for the reference's deflate64 fixtures (test/data, pinned by
inflate_small.json) and for raw deflate without the window-wrap copy; and of
the lane kernel's large-member instance, which tracks the reference's calls."""
import hashlib
import json
import os
import random

import pytest

import corpus
import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D64 = os.path.join(ROOT, "tests", "golden", "d64")


def _fixtures():
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "inflate_small.json")))
    return [(c["name"][4:], open(os.path.join(D64, c["name"][4:]), "rb").read(), c["out_len"], c["out_sha256"])
            for c in g["cases"] if c["name"].startswith("d64_") and c.get("ok")]


class _opts:
    """Engine options for the duration of a block (restored to the defaults after)."""

    DEFAULTS = {"inflate_split": 1, "inflate_wave_min": 32768, "inflate_ref_wrap": 1, "inflate_fast": 1,
                "lane_large_min": 2304, "inflate_seg": 1}

    def __init__(self, engine, **kw):
        self.e, self.kw = engine, kw

    def __enter__(self):
        for k, v in self.kw.items():
            self.e.set_option(k, v)

    def __exit__(self, *a):
        for k in self.kw:
            self.e.set_option(k, self.DEFAULTS[k])


def _decode(engine, members, fmt, caps, **kw):
    kw.setdefault("inflate_seg", 0)  # (the segmented decode has its own tests: test_gpu_seg.py)
    with _opts(engine, **kw):
        res = engine.decompress_batch_raw(members, fmt, out_caps=caps)
        return res, engine.last_lane_count()


def test_large_d64_fixture_splits_and_matches_golden(engine):
    fx = {name: (d, n, h) for name, d, n, h in _fixtures()}
    d, n, h = fx["100k_lines.deflate64"]
    engine.set_timing(True)
    try:
        res, fast = _decode(engine, [d], "deflate64-raw", [n])
        split_ms = engine.last_ms("split_resolve")
    finally:
        engine.set_timing(False)
    st, ph, msg, out, cons = res[0]
    assert st == 1 and len(out) == n and hashlib.sha256(out).hexdigest() == h
    assert cons == len(d)
    assert fast == 1, "the member left the split path"
    assert split_ms >= 0, "no split phase ran"


def test_every_d64_fixture_through_the_split_path(engine):
    # inflate_wave_min = 1: every fixture (even the 369-byte one) is a "large" member
    fxs = _fixtures()
    members = [d for _, d, _, _ in fxs]
    res, fast = _decode(engine, members, "deflate64-raw", [(n + 3) & ~3 for _, _, n, _ in fxs], inflate_wave_min=1)
    for (name, d, n, h), (st, ph, msg, out, cons) in zip(fxs, res):
        assert st == 1 and len(out) == n and hashlib.sha256(out).hexdigest() == h, name
        assert cons == len(d), name
    assert fast == len(fxs)


def test_split_equals_wave_path_on_raw_without_window_wrap(engine):
    """Raw deflate with inflate_ref_wrap = 0 (zlib semantics): multi-MB and
    multi-block members at several levels decode to their source."""
    rng = random.Random(5150)
    srcs = []
    for kind, n in (("text", 3 << 20), ("mixed", 1 << 20), ("text", 300000), ("zeros", 2 << 20), ("rand", 200000),
                    ("text", 70000)):
        srcs.append(corpus.make({"kind": kind, "n": n, "seed": rng.randrange(1 << 32)}))
    for level in (1, 6, 9):
        comps = engine.compress_batch(srcs, "deflate-raw", level)
        caps = [len(s) + 64 for s in srcs]
        res, fast = _decode(engine, comps, "deflate-raw", caps, inflate_ref_wrap=0)
        for s, c, (st, ph, msg, out, cons) in zip(srcs, comps, res):
            assert st == 1 and out == s and cons == len(c), (level, len(s))
        assert fast == len(srcs), level
        res_w, _ = _decode(engine, comps, "deflate-raw", caps, inflate_ref_wrap=0, inflate_split=0)
        assert [r[3] for r in res_w] == [r[3] for r in res]


def test_split_errors_match_the_exact_path(engine):
    """Corrupted large members: whatever the pieces see, the member's outcome
    (status, phase, message, bytes, consumed) is the exact kernel's."""
    fx = {name: d for name, d, _, _ in _fixtures()}
    base = fx["100k_lines.deflate64"]
    rng = random.Random(99)
    members = []
    for k in range(12):
        b = bytearray(base)
        for _ in range(rng.choice([1, 3, 20])):
            i = rng.randrange(len(b))
            b[i] ^= 1 << rng.randrange(8)
        if k % 4 == 3:
            b = b[:rng.randrange(40000, len(b))]  # truncated
        members.append(bytes(b))
    members.append(bytes(rng.randrange(256) for _ in range(70000)))  # noise
    caps = [2188890 + 1024] * len(members)
    got, _ = _decode(engine, members, "deflate64-raw", caps)
    want, _ = _decode(engine, members, "deflate64-raw", caps, inflate_fast=0)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, i


def test_split_capacity_short_is_the_exact_paths_error(engine):
    fx = {name: (d, n) for name, d, n, _ in _fixtures()}
    d, n = fx["100k_lines.deflate64"]
    got, _ = _decode(engine, [d], "deflate64-raw", [n // 2])
    want, _ = _decode(engine, [d], "deflate64-raw", [n // 2], inflate_fast=0)
    assert got == want and got[0][0] != 1


def test_unbounded_decode_of_a_large_member(engine):
    """decompress_batch without caps (DecompressionStream, streams.ts:132-182):
    the first capacity guess is too small for the fixture, the retry splits."""
    fx = {name: (d, n, h) for name, d, n, h in _fixtures()}
    d, n, h = fx["100k_lines.deflate64"]
    out = engine.decompress_batch([d, fx["10k_lines.deflate64"][0]], "deflate64-raw")
    assert hashlib.sha256(out[0]).hexdigest() == h and len(out[1]) == fx["10k_lines.deflate64"][1]


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_large_member_lanes_equal_the_reference_and_the_exact_path(engine, fmt):
    """The lane kernel's large-member instance (the reference's inflate() calls
    tracked per lane; used when a batch has lane_large_min large members, here
    forced with a small minimum) in every wrapped format: clean members equal the
    oracle with the reference's window-wrap copy (reference_bugs), damaged ones
    the exact kernel's status / phase / message / bytes."""
    rng = random.Random(4242)
    members, caps = [], []
    for k in range(24):
        s = corpus.make({"kind": rng.choice(["text", "mixed"]), "n": rng.choice([70000, 150000, 262144]),
                         "seed": rng.randrange(1 << 32)})
        c = oracle.compress(s, rng.choice([1, 6, 9]), fmt)[1]
        if k % 6 == 5:  # damaged: a bit flip or a truncation
            b = bytearray(c)
            if k % 12 == 5:
                b[rng.randrange(len(b) // 2, len(b))] ^= 1 << rng.randrange(8)
            else:
                b = b[:rng.randrange(len(b) // 2, len(b))]
            c = bytes(b)
        members.append(c)
        caps.append((len(s) + 64 + 3) & ~3)
    j = json.load(open(os.path.join(ROOT, "tests", "golden", "inffast_wrap_defect.json")))
    if fmt == "deflate-raw":  # the member whose decode the reference's defect changes
        src = corpus.make(j["source"])
        members.append(oracle.compress(src, 6, fmt)[1])
        caps.append((len(src) + 64 + 3) & ~3)
    got, fast = _decode(engine, members, fmt, caps, lane_large_min=4)
    want, _ = _decode(engine, members, fmt, caps, inflate_fast=0)
    for i, (g, w, c, cap) in enumerate(zip(got, want, members, caps)):
        assert g == w, i
        ost, oout, ocons, oph, omsg = oracle.decompress(c, fmt, cap=cap, reference_bugs=True)
        assert g[0] == ost, (i, g[0], g[1], g[2], ost, oph, omsg)
        if ost == 1:
            assert g[3] == oout and g[4] == ocons, (i, len(g[3]), len(oout))
    assert fast >= sum(1 for w in want if w[0] == 1)  # every clean member finished on the lanes
    if fmt == "deflate-raw":
        assert corpus.sha256(got[-1][3]) == j["ref_out_sha256"]


@pytest.mark.parametrize("fmt", ["deflate-raw", "gzip"])
def test_retry_pass_decodes_large_members_on_the_lanes(engine, fmt):
    """inflate_wave_min = 0: every member starts on the single-call lanes, which
    bail on those longer than one reference inflate() call; the retry pass (the
    call-tracking instance, no member list) must finish the clean ones -- equal
    to the exact kernel and to the oracle with the reference's defect -- and
    leave damaged ones to the exact path."""
    rng = random.Random(777)
    members, caps = [], []
    for k in range(16):
        s = corpus.make({"kind": rng.choice(["text", "mixed"]), "n": rng.choice([20000, 70000, 150000]),
                         "seed": rng.randrange(1 << 32)})
        c = oracle.compress(s, rng.choice([1, 6, 9]), fmt)[1]
        if k % 8 == 7:
            c = c[:len(c) * 3 // 4]  # truncated
        members.append(c)
        caps.append((len(s) + 64 + 3) & ~3)
    got, fast = _decode(engine, members, fmt, caps, inflate_wave_min=0)
    want, _ = _decode(engine, members, fmt, caps, inflate_fast=0)
    assert got == want
    for g, c, cap in zip(got, members, caps):
        ost, oout, ocons, oph, omsg = oracle.decompress(c, fmt, cap=cap, reference_bugs=True)
        assert g[0] == ost and (ost != 1 or (g[3] == oout and g[4] == ocons))
    assert fast >= sum(1 for w in want if w[0] == 1)


@pytest.mark.parametrize("path", ["lanes", "wave", "split", "exact"])
def test_deflate64_copies_longer_than_the_window(engine, path):
    """deflate64 length code 285 (3 + 16 extra bits, inflate/constants.ts:12,28):
    copies of 65,537 / 65,538 bytes -- longer than the 64 KiB history ring of the
    wave and split decoders -- at distances that do not divide 65,536, and
    distance 65,536 behind them (tests/bitbuild.py builds the streams; the
    expected bytes are the plain LZ77 expansion, checked against the oracle)."""
    import bitbuild

    cases = bitbuild.long_copies()
    members = [c for c, _ in cases]
    caps = [(len(e) + 3) & ~3 for _, e in cases]
    kw = {"lanes": {}, "wave": {"inflate_wave_min": 1, "inflate_split": 0},
          "split": {"inflate_wave_min": 1, "inflate_split": 1}, "exact": {"inflate_fast": 0}}[path]
    res, fast = _decode(engine, members, "deflate64-raw", caps, **kw)
    for (c, e), (st, ph, msg, out, cons) in zip(cases, res):
        assert st == 1 and out == e and cons == len(c), (path, len(e), st, msg)
        assert oracle.decompress(c, "deflate64-raw", cap=len(e) + 16)[1] == e
    if path != "exact":
        assert fast == len(cases), "a member left the %s path" % path
