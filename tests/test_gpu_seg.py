"""GPU parity of the segmented decode (inflate_seg.hip): a member's blocks cut
into lane-sized pieces that synchronise, markers for the history before a
piece, the reference's inflate() call state per piece (window-wrap copy of
inffast.ts:127-147).  Every member it finishes must equal the oracle with the
reference's defect (reference_bugs, oracle/inflate.c) -- i.e. what
DecompressionStream (streams.ts:253-262) returns for one write() -- and every
member it does not finish must take the other paths to the same outcome."""
import hashlib
import json
import os
import random

import pytest

import corpus
import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _opts:
    DEFAULTS = {"inflate_seg": 1, "seg_bits": 0, "seg_small_batch": 16384, "seg_small_min": 4096,
                "inflate_fast": 1, "inflate_ref_wrap": 1, "inflate_wave_min": 32768, "seg_scratch_mb": 16384,
                "seg_wide": 1, "seg_big_bits": 1 << 21, "timing": 0, "check_phases": 0, "seg_split": 2}

    def __init__(self, engine, **kw):
        self.e, self.kw = engine, kw

    def __enter__(self):
        for k, v in self.kw.items():
            self.e.set_option(k, v)

    def __exit__(self, *a):
        for k in self.kw:
            self.e.set_option(k, self.DEFAULTS[k])


def _members(rng, fmt, kinds, levels, sizes, count):
    out = []
    for _ in range(count):
        n = rng.choice(sizes)
        s = corpus.make({"kind": rng.choice(kinds), "n": n, "seed": corpus.stream_seed(rng.randrange(4096))})
        out.append((s, oracle.compress(s, rng.choice(levels), fmt)[1]))
    return out


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_segmented_decode_equals_the_reference(engine, fmt):
    """T- and M-corpus members of 20 KB .. 500 KB at levels 1 / 6 / 9: every one
    finished by the segmented decode, and the outcome equal to the oracle's decode
    with the reference's window-wrap copy -- for zlib / gzip that includes the
    reference's own "incorrect data check" when the copy changes bytes that the
    trailer's checksum covers (the reference reports its defect that way)."""
    rng = random.Random({"deflate-raw": 1, "deflate": 2, "gzip": 3}[fmt])
    ms = _members(rng, fmt, ["text", "mixed"], [1, 6, 9], [20000, 65536, 150000, 262144, 500000], 24)
    comps = [c for _, c in ms]
    caps = [len(s) + 16 for s, _ in ms]
    got = engine.decompress_batch_detailed(comps, fmt, caps)
    assert engine.last_seg_count() == len(ms)  # every member finished by the segmented decode
    ok = 0
    for i, ((s, c), g) in enumerate(zip(ms, got)):
        st, out, cons, ph, msg = oracle.decompress(c, fmt, cap=len(s) + 16, reference_bugs=True)
        # status, phase, message and consumed bytes of every member, the failing ones too
        assert (g[0], g[1], g[2], g[4]) == (st, ph, msg, cons), (i, g[:3], g[4], st, ph, msg, cons)
        if st == 1:
            ok += 1
            assert g[3] == out and cons == len(c), i
            if fmt != "deflate-raw":
                assert (g[5] & 0xffffffff) == (oracle.crc32(out) if fmt == "gzip" else oracle.adler32(out)), i
    # the seeded corpus pinned: the members the reference itself decodes cleanly (the rest end in its
    # "incorrect data check" through the window-wrap defect), so a generator change cannot hide a regression
    assert ok == {"deflate-raw": 24, "deflate": 22, "gzip": 19}[fmt]


@pytest.mark.parametrize("opt", [("seg_big_bits", 65536), ("seg_wide", 0), ("check_phases", 1), ("timing", 1),
                                 ("seg_split", 0), ("seg_split", 1)])
def test_walk_options_do_not_change_bytes(engine, opt):
    """seg_big_bits (members over it also walk from the block starts zs_k_split_find proposes), seg_wide (the
    2,048-bit sync window), seg_split (pieces cut in two at the walk's mid points), check_phases and timing only
    change how the decode runs: T- and M-corpus members of
    100 .. 500 KB at L6 / L9, every one finished by the segmented decode, equal the oracle with the reference's
    window-wrap copy, status and message included."""
    rng = random.Random(sum(opt[0].encode()))
    ms = _members(rng, "deflate-raw", ["text", "mixed"], [6, 9], [100000, 262144, 500000], 8)
    comps = [c for _, c in ms]
    caps = [len(s) + 16 for s, _ in ms]
    with _opts(engine, **{opt[0]: opt[1]}):
        got = engine.decompress_batch_detailed(comps, "deflate-raw", caps)
        assert engine.last_seg_count() == len(ms)
    for i, ((s, c), g) in enumerate(zip(ms, got)):
        st, out, cons, ph, msg = oracle.decompress(c, "deflate-raw", cap=len(s) + 16, reference_bugs=True)
        assert (g[0], g[1], g[2], g[4]) == (st, ph, msg, cons) and g[3] == out, (opt, i)


@pytest.mark.parametrize("bits", [1024, 8192])
def test_piece_size_does_not_change_bytes(engine, bits):
    """seg_bits (input bits per piece) only changes how a member is cut: the
    bytes of M-corpus members at L6 (window-wrap copies in most) are the same."""
    rng = random.Random(bits)
    ms = _members(rng, "deflate-raw", ["mixed"], [6, 9], [262144, 500000], 8)
    comps = [c for _, c in ms]
    caps = [len(s) for s, _ in ms]
    with _opts(engine, seg_bits=bits):
        got = engine.decompress_batch_raw(comps, "deflate-raw", caps)
        nseg = engine.last_seg_count()
    want = [oracle.decompress(c, "deflate-raw", cap=len(s), reference_bugs=True) for s, c in ms]
    assert nseg == len(ms)
    assert [g[3] for g in got] == [w[1] for w in want]


def test_segmented_decode_without_the_window_wrap_copy(engine):
    """inflate_ref_wrap = 0: zlib semantics (no call bookkeeping); the members
    decode to their sources."""
    rng = random.Random(77)
    ms = _members(rng, "deflate-raw", ["mixed", "text"], [6, 9], [200000, 500000], 8)
    with _opts(engine, inflate_ref_wrap=0):
        got = engine.decompress_batch_raw([c for _, c in ms], "deflate-raw", [len(s) for s, _ in ms])
        nseg = engine.last_seg_count()
    assert nseg == len(ms)
    assert [g[3] for g in got] == [s for s, _ in ms]


def test_deflate64_fixtures_in_a_small_batch(engine):
    """The reference's test/data deflate64 fixtures (decoded sizes / digests
    pinned by inflate_small.json), each a "large" member of a small batch: the
    high-expansion ones (long copies: a cap past 64 KiB, >= 8 output bytes per
    input byte) take the split decode, the others the segmented one."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "inflate_small.json")))
    fx = [(open(os.path.join(ROOT, "tests", "golden", "d64", c["name"][4:]), "rb").read(), c["out_len"],
           c["out_sha256"]) for c in g["cases"] if c["name"].startswith("d64_") and c.get("ok")]
    with _opts(engine, seg_small_min=256):
        got = engine.decompress_batch_raw([d for d, _, _ in fx], "deflate64-raw", [n for _, n, _ in fx])
    for (d, n, h), r in zip(fx, got):
        assert r[0] == 1 and len(r[3]) == n and hashlib.sha256(r[3]).hexdigest() == h and r[4] == len(d)
    # the same fixtures with caps that hide the expansion (<= 64 KiB where they fit): the segmented decode
    small = [(d, n, h) for d, n, h in fx if n <= 65536]
    with _opts(engine, seg_small_min=256):
        got = engine.decompress_batch_raw([d for d, _, _ in small], "deflate64-raw", [65536] * len(small))
        nseg = engine.last_seg_count()
    for (d, n, h), r in zip(small, got):
        assert r[0] == 1 and len(r[3]) == n and hashlib.sha256(r[3]).hexdigest() == h and r[4] == len(d)
    # all five finished there: payload_63k / repeat_63k end with a 1-bit end-of-block code, whose
    # zeros past the input end the walk must not take for the block's end
    assert nseg == len(small) == 5


def _runs_member(seed, n):
    """T-corpus stretches between runs of period 1 .. 7 (1 .. 3,000 values): long copies of distance 1 .. 7,
    at every alignment to the pieces' 8-value units, and far repeats of 64 .. 258 bytes.  (Stretches of
    random bytes are not used: their near-uniform 8-bit literal codes keep a lane started at the wrong bit
    offset from synchronising, and such members leave the segmented decode for the wave kernel.)"""
    rng = random.Random(seed)
    text = corpus.make({"kind": "text", "n": 1 << 16, "seed": corpus.stream_seed(seed)})
    out = bytearray()
    while len(out) < n:
        at = rng.randrange(0, len(text) - 1200)
        out += text[at:at + rng.randrange(200, 1200)]
        p = rng.randrange(1, 8)
        pat = bytes(rng.randrange(256) for _ in range(p))
        k = rng.choice([rng.randrange(1, 64), rng.randrange(64, 400), rng.randrange(400, 3000)])
        out += (pat * (k // p + 1))[:k]
        if len(out) > 31000 and rng.random() < 0.5:  # a far repeat: long copies from before most pieces
            at = len(out) - rng.randrange(300, 30000)
            out += out[at:at + rng.randrange(64, 259)]
    return bytes(out[:n])


def test_long_runs_and_far_markers_in_the_segmented_decode(engine):
    """Copies of 64 values and more leave a piece as whole 16-byte units (zs_sg_out::run): distance-1/2/4
    runs, runs of the other periods, and markers for history far before a piece start -- the bytes equal the oracle's,
    every member finished by the segmented decode."""
    ms = []
    for i in range(12):
        s = _runs_member(500 + i, 150000 + 7919 * i)
        ms.append((s, oracle.compress(s, [1, 6, 9][i % 3], "deflate-raw")[1]))
    with _opts(engine, seg_bits=1024):
        got = engine.decompress_batch_raw([c for _, c in ms], "deflate-raw", [len(s) for s, _ in ms])
        nseg = engine.last_seg_count()
    # (the oracle with the reference's window-wrap copy decides the bytes)
    want = [oracle.decompress(c, "deflate-raw", cap=len(s), reference_bugs=True)[1] for s, c in ms]
    assert nseg == len(ms)
    assert [g[3] for g in got] == want


def test_damaged_members_take_the_other_paths(engine):
    """Bit flips and truncations: whatever the pieces see, each member's outcome
    (status, phase, message, bytes, consumed) equals the exact kernel's."""
    rng = random.Random(31)
    members = []
    for k, (s, c) in enumerate(_members(rng, "deflate-raw", ["text", "mixed"], [1, 6], [70000, 262144], 16)):
        b = bytearray(c)
        if k % 3 == 0:
            for _ in range(rng.choice([1, 4])):
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        elif k % 3 == 1:
            b = b[:rng.randrange(len(b) // 3, len(b))]
        members.append(bytes(b))
    caps = [300000] * len(members)
    got = engine.decompress_batch_raw(members, "deflate-raw", caps)
    with _opts(engine, inflate_fast=0):
        want = engine.decompress_batch_raw(members, "deflate-raw", caps)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, i


def test_segmented_and_lane_paths_agree_on_a_mixed_batch(engine):
    """One batch with tiny members (lanes) and large ones (segmented), in gzip:
    the same outcome as with the segmented decode off."""
    rng = random.Random(5)
    ms = _members(rng, "gzip", ["text", "mixed"], [6], [300, 3000, 9000, 65536, 262144], 40)
    comps = [c for _, c in ms]
    caps = [len(s) + 8 for s, _ in ms]
    got = engine.decompress_batch_detailed(comps, "gzip", caps)
    assert engine.last_seg_count() == sum(1 for c in comps if len(c) > 4096)
    with _opts(engine, inflate_seg=0):
        want = engine.decompress_batch_detailed(comps, "gzip", caps)
    assert got == want
    for (s, c), g in zip(ms, got):  # (the window-wrap copy can fail a gzip member's CRC, as in the reference)
        st, out, cons, ph, msg = oracle.decompress(c, "gzip", cap=len(s) + 8, reference_bugs=True)
        assert (g[0], g[1]) == (st, ph) and (st != 1 or g[3] == out)


def test_scratch_budget_sends_the_rest_to_the_other_paths(engine):
    """The segmented decode's u16 piece scratch (2 bytes per byte of capacity) is bounded per batch (option
    seg_scratch_mb): with a 1 MiB budget only the first few members of 256 take it, the others the wave kernel,
    and every member still equals its source."""
    import zsamd

    N, L = 256, 65536
    host = zsamd.corpus("text", 0, N, L)
    src = [bytes(host[i * L:(i + 1) * L]) for i in range(N)]
    comp = engine.compress_batch(src, "deflate-raw", 6)
    with _opts(engine, seg_scratch_mb=1):
        got = engine.decompress_batch(comp, "deflate-raw", [L] * N)
        nseg = engine.last_seg_count()
    engine.set_option("seg_scratch_mb", 16384)
    assert 0 < nseg < N // 4
    assert got == src


def _dyn_stored_member(rng, n, src, empty_at=None):
    """A member of about n output bytes: stored blocks (0 .. 20,001 bytes) between dynamic blocks taken verbatim
    from L6 members of src stretches (the encoder's own blocks, so lanes meet as in its members); with empty_at, an
    empty stored block whose LEN / NLEN straddle input byte empty_at (a sub-chunk end) and a coded block after it."""
    import sys

    import bitbuild

    sys.path.insert(0, os.path.join(ROOT, "tools", "emu"))
    import emu_seg

    parts, pos, made = [], 0, 0  # pos: the member's bits so far

    def stored(k):
        nonlocal pos, made
        parts.append(("stored", src[made % len(src):made % len(src) + k]))
        pos = ((pos + 3 + 7) & ~7) + 32 + 8 * len(parts[-1][1])
        made += len(parts[-1][1])

    def coded():
        nonlocal pos, made
        while True:
            a = rng.randrange(len(src) - 40000)
            chunk = src[a:a + rng.choice([3000, 12000, 30000])]
            c = oracle.compress(chunk, 6, "deflate-raw")[1]
            _, blks, end = emu_seg.decode(c)
            if len(blks) == 1 and c[0] & 6 == 4:  # one dynamic block
                break
        parts.append(("bits", c, end, chunk))
        pos += end
        made += len(chunk)

    while made < n:
        if empty_at is not None and 0 < empty_at - pos // 8 < 60000:
            q = (pos + 3 + 7) >> 3  # the filler's LEN
            stored(empty_at - 3 - q - 4)
            stored(0)  # header byte at empty_at - 3, LEN / NLEN over the boundary
            assert (pos >> 3) == empty_at + 2
            coded()
            empty_at = None
        elif rng.random() < 0.5:
            stored(rng.choice([0, 1, 7, 999, 5003, 20001]))
        else:
            coded()
    m, exp = bitbuild.blocks(parts)
    assert oracle.decompress(m, "deflate-raw", cap=len(exp), reference_bugs=False)[1] == exp
    return m


def test_stored_blocks_in_the_segmented_decode(engine):
    """Stored blocks (BTYPE 0, inflate.ts:631-672) walked and copied by the segmented decode: 256 KiB members of
    R-corpus bytes at L6 and of M/R/T patchworks at L1 / L6 / L9 (the encoder's stored blocks among coded ones; one
    has a window-wrap copy behind them), level-0 members (the engine's, and hand-built ones of stored blocks of 0 ..
    65,535 bytes, not multiples of 4: the oracle does not restate level 0) and hand-built mixes of stored blocks and
    an encoder's dynamic blocks (one with an empty stored block whose LEN / NLEN straddle a sub-chunk end, a coded
    block after it) -- every member finished by the segmented decode, its outcome equal to the oracle's."""
    import bitbuild

    src = corpus.text(11, 150000) + corpus.rand(12, 100000) + corpus.make({"kind": "mixed", "n": 100000, "seed": 13})
    raw = [bitbuild.stored_mix(random.Random(i), 262144, src, level0=True)[0] for i in range(3)]
    raw += [_dyn_stored_member(random.Random(20 + i), 262144, src, 65536 if i == 0 else None) for i in range(3)]
    raw += [oracle.compress(corpus.rand(8, 262144), 6, "deflate-raw")[1]]
    raw += [oracle.compress(corpus.patchwork(seed, 262144), lv, "deflate-raw")[1]
            for seed, lv in [(208, 6), (201, 1), (204, 9), (205, 6)]]
    # the engine's level 0 (zs_k_stored, pinned to the reference's level-0 goldens): 32,768-byte stored blocks
    lvl0 = [corpus.patchwork(209, 262144), corpus.text(14, 200000)]
    raw += engine.compress_batch(lvl0, "deflate-raw", 0)
    gz = [oracle.compress(corpus.patchwork(seed, 262144), 6, "gzip")[1] for seed in (208, 202)]
    gz += engine.compress_batch(lvl0, "gzip", 0)
    for fmt, comps in (("deflate-raw", raw), ("gzip", gz)):
        want = [oracle.decompress(c, fmt, cap=1 << 20, reference_bugs=True) for c in comps]
        got = engine.decompress_batch_detailed(comps, fmt, [len(w[1]) + 16 for w in want])
        assert engine.last_seg_count() == len(comps), fmt  # every member finished by the segmented decode
        for i, (g, (st, out, cons, ph, msg)) in enumerate(zip(got, want)):
            assert st == 1 or fmt == "gzip", i
            assert (g[0], g[1], g[2], g[4]) == (st, ph, msg, cons), (fmt, i, g[:3], g[4], st, ph, msg, cons)
            assert st != 1 or g[3] == out, (fmt, i)
