"""GPU parity: the HIP deflate engine against the reference's goldens and the oracle."""
import hashlib
import random

import pytest

import corpus
import golden_io
import oracle

pytestmark = pytest.mark.gpu

GPU_LEVELS = [1, 2, 3, 4, 5, 6, 7, 8, 9]


def test_small_goldens(engine):
    cases = [(c, d) for c, d in golden_io.deflate_cases() if c["level"] in GPU_LEVELS]
    groups = {}
    for c, d in cases:
        groups.setdefault((c["level"], c["format"]), []).append((c, d))
    bad = []
    for (level, fmt), items in sorted(groups.items()):
        res = engine.compress_batch_raw([d for _, d in items], fmt, level)
        for (c, d), (st, out) in zip(items, res):
            if st != 1 or corpus.sha256(out) != c["out_sha256"]:
                bad.append((c["spec"].get("kind"), c["in_len"], level, fmt, st, len(out), c["out_len"]))
    assert not bad, bad[:10]


def test_empty_and_hello(engine):
    assert engine.compress_batch([b""], "deflate-raw", 6) == [bytes([3, 0])]
    assert engine.compress_batch([b"hello"], "deflate-raw", 6)[0].hex() == "cb48cdc9c90700"
    assert engine.compress_batch([b""], "gzip", 6)[0].hex() == "1f8b08000000000000ff0300" + "00" * 8


@pytest.mark.parametrize("level", GPU_LEVELS)
def test_random_inputs_vs_oracle(engine, level):
    rng = random.Random(1000 + level)
    inputs = []
    for k in range(24):
        n = rng.choice([0, 1, 2, 3, 4, 257, 258, 259, 1000, 4095, 32768, 32769, 65535, 65536, 65537, 65538, 70001,
                        rng.randrange(1, 140000)])
        kind = rng.choice(["text", "mixed", "rand", "zeros", "ramp"])
        spec = {"kind": kind, "n": n, "seed": rng.randrange(1 << 32)}
        inputs.append(corpus.make(spec))
    for fmt in ["deflate-raw", "deflate", "gzip"]:
        res = engine.compress_batch_raw(inputs, fmt, level)
        for d, (st, out) in zip(inputs, res):
            ost, ref, _ = oracle.compress(d, level, fmt)
            assert st == 1 and out == ref, (len(d), fmt, level, len(out), len(ref))


def test_block_boundaries_and_stored_blocks(engine):
    # > 16383 symbols per stream (multi-block), incompressible data (stored blocks),
    # lengths that are multiples of 16383 symbols and tiny tails
    inputs = [corpus.rand(corpus.stream_seed(1), 16383), corpus.rand(corpus.stream_seed(2), 16384),
              corpus.rand(corpus.stream_seed(3), 50000), bytes(200000), corpus.text(corpus.stream_seed(4), 262144),
              corpus.rand(corpus.stream_seed(5), 16383 * 2), corpus.rand(corpus.stream_seed(6), 16383 * 2 + 1)]
    for level in (1, 3, 4, 6, 9):
        res = engine.compress_batch_raw(inputs, "deflate-raw", level)
        for d, (st, out) in zip(inputs, res):
            assert st == 1 and out == oracle.compress(d, level, "deflate-raw")[1], (len(d), level)


@pytest.mark.parametrize("level", [4, 5, 6, 7, 8, 9])
def test_sweep_match_table_equals_chain_walk(engine, level):
    """zs_k_bucket + zs_k_sweep (deflate_sweep.hip; streams over 65,537 B in
    windows) and zs_k_prev + zs_k_match (deflate_match.hip, the chain walk: option
    match_sweep = 0) compute the same longest_match table -- both budgets and the
    slide-NIL flag -- at every position, and the same output bytes (= the oracle's)."""
    rng = random.Random(500 + level)
    inputs = []
    for k in range(20):
        n = rng.choice([0, 1, 2, 3, 4, 5, 9, 10, 11, 258, 259, 300, 4097, 32506, 32507, 32769, 65535, 65536, 65537,
                        rng.randrange(1, 65538)])
        kind = rng.choice(["text", "mixed", "rand", "zeros", "ramp"])
        inputs.append(corpus.make({"kind": kind, "n": n, "seed": rng.randrange(1 << 32)}))
    b = bytearray(corpus.rand(77, 65536))  # a candidate at exactly MAX_DIST
    b[40000:40020] = b[40000 - 32506:40000 - 32506 + 20]
    inputs.append(bytes(b))
    # 7-bit streams (the sweep's 8-byte signature form): hash collisions with different first bytes,
    # deep chains over a small alphabet, text after 7-bit noise
    inputs.append(bytes(x & 0x7F for x in corpus.rand(91 + level, 65536)))
    inputs.append(bytes(0x41 + (x & 3) for x in corpus.rand(92 + level, 65536)))
    inputs.append(bytes(x & 0x7F for x in corpus.rand(93, 20000)) + corpus.text(94, 45537))
    # streams over 65,537 bytes: the sweep in windows (a first one owning 65,520 positions, then 32,752 own positions
    # after a 32,768-position look-back each, capi.cpp sweep_table), at and around the window boundaries and up to
    # 256 KiB
    for n, kind in ((65538, "text"), (98302, "mixed"), (98303, "text"), (130836, "zeros"), (262144, "text"),
                    (200001, "mixed"), (70000, "rand")):
        inputs.append(corpus.make({"kind": kind, "n": n, "seed": rng.randrange(1 << 32)}))
    # match_sweep: the sweep, and the chain walk (zs_k_prev + zs_k_match) as the cross-check
    tables, outs = [], []
    try:
        for sweep in (1, 0):
            engine.set_option("match_sweep", sweep)
            outs.append(engine.compress_batch_raw(inputs, "deflate-raw", level))
            tables.append([engine.debug_fetch(1, i, 8 * len(d)) for i, d in enumerate(inputs)])
    finally:
        engine.set_option("match_sweep", 1)
    for i, d in enumerate(inputs):
        assert tables[0][i] == tables[1][i], (i, len(d))
        want = oracle.compress(d, level, "deflate-raw")[1]
        assert outs[0][i] == outs[1][i] and outs[0][i][1] == want, (i, len(d))


def test_output_capacity_too_small_reports_buf_error(engine):
    import ctypes
    import zsamd

    L = zsamd.lib()
    d = corpus.rand(corpus.stream_seed(9), 4000)
    out = ctypes.create_string_buffer(64)
    st = (ctypes.c_int32 * 1)()
    ol = (ctypes.c_uint32 * 1)()
    r = L.zs_deflate_batch(engine.handle, 6, -15, 1, d, (ctypes.c_uint64 * 1)(0), (ctypes.c_uint32 * 1)(len(d)),
                           out, (ctypes.c_uint64 * 1)(0), (ctypes.c_uint32 * 1)(64), st, ol)
    assert r == 0 and st[0] == zsamd.Z_BUF_ERROR


def test_invalid_arguments_are_init_errors(engine):
    import zsamd

    with pytest.raises(zsamd.ZsError) as e:
        engine.compress_batch([b"x"], "deflate-raw", 10)
    assert str(e.value) == "init failed: -2"  # streams.ts:53 with deflate.ts:281-294


@pytest.mark.slow
def test_c2_full_batch_matches_reference_goldens(engine):
    """BASELINE.json configs[1]: 4096 x 64 KiB T-corpus, deflate-raw L6, byte-identical."""
    import zsamd

    recs = golden_io.batch("t64_l6_raw")
    buf = bytes(zsamd.corpus("text", 0, 4096, 65536))
    inputs = [buf[i * 65536:(i + 1) * 65536] for i in range(4096)]
    res = engine.compress_batch_raw(inputs, "deflate-raw", 6)
    bad = [i for i, (st, out) in enumerate(res) if st != 1 or (len(out), hashlib.sha256(out).digest()[:16]) != recs[i]]
    assert not bad, bad[:10]
    assert sum(len(o) for _, o in res) == 91855591


@pytest.mark.parametrize("level", [1, 2, 3])
def test_group_fast_parser_equals_serial_replay(engine, level):
    """zs_k_fast (group-speculative, default) against zs_k_fast_serial (step by step): same bytes on
    streams that slide several times, all-zero and random streams, and sizes around the group and
    slide boundaries; both also against the oracle on the short ones."""
    specs = [("text", 262144), ("mixed", 200000), ("rand", 40000), ("zeros", 100000), ("ramp", 70000),
             ("text", 0), ("text", 1), ("text", 3), ("text", 4), ("text", 59), ("text", 64), ("text", 259),
             ("text", 32769), ("text", 65535), ("text", 65536), ("text", 65537), ("zeros", 65537),
             ("text", 98304 + 300), ("mixed", 131072 + 17)]
    inputs = [corpus.make({"kind": k, "n": n, "seed": 9300 + i}) for i, (k, n) in enumerate(specs)]
    b = bytearray(corpus.rand(78, 90000))  # a candidate at exactly MAX_DIST
    b[40000:40020] = b[40000 - 32506:40000 - 32506 + 20]
    inputs.append(bytes(b))
    try:
        engine.set_option("fast_group", 0)
        ref = engine.compress_batch_raw(inputs, "deflate-raw", level)
        engine.set_option("fast_group", 1)
        res = engine.compress_batch_raw(inputs, "deflate-raw", level)
    finally:
        engine.set_option("fast_group", 1)
    bad = [i for i in range(len(inputs)) if res[i] != ref[i]]
    assert not bad, [(specs[i] if i < len(specs) else "dist", len(res[i][1]), len(ref[i][1])) for i in bad]
    for d, (st, out) in zip(inputs, res):
        if len(d) <= 65536:
            assert st == 1 and out == oracle.compress(d, level, "deflate-raw")[1]


@pytest.mark.parametrize("level", [4, 6, 9])
def test_two_wave_parse_equals_one_wave_parse(engine, level):
    """zs_k_parse_2w / _4w (two / four waves per stream, 512 / 256-position segments; two waves are the default
    below 2048 streams) against zs_k_parse (one wave, 1 KiB segments): same bytes on 64 KiB, 256 KiB (slides, several super-rounds) and
    ragged streams, and the C2 goldens of 1,000 streams with two waves forced."""
    import zsamd

    specs = [("text", 65536), ("mixed", 65536), ("text", 262144), ("mixed", 200000 + 13), ("zeros", 131072),
             ("rand", 40000), ("text", 32768), ("text", 32769), ("text", 511), ("text", 512), ("text", 513),
             ("text", 0), ("text", 5), ("text", 98304 + 300)]
    inputs = [corpus.make({"kind": k, "n": n, "seed": 9500 + i}) for i, (k, n) in enumerate(specs)]
    outs = []
    try:
        for w in (1, 2, 4):
            engine.set_option("parse_waves", w)
            outs.append(engine.compress_batch_raw(inputs, "deflate-raw", level))
        assert outs[0] == outs[1] == outs[2]
        if level == 6:
            recs = golden_io.batch("t64_l6_raw")
            buf = bytes(zsamd.corpus("text", 0, 1000, 65536))
            res = engine.compress_batch_raw([buf[i * 65536:(i + 1) * 65536] for i in range(1000)], "deflate-raw", 6)
            bad = [i for i, (st, out) in enumerate(res)
                   if st != 1 or (len(out), hashlib.sha256(out).digest()[:16]) != recs[i]]
            assert not bad, bad[:10]
    finally:
        engine.set_option("parse_waves", 0)
    for d, (st, out) in zip(inputs, outs[1]):
        if len(d) <= 65536:
            assert st == 1 and out == oracle.compress(d, level, "deflate-raw")[1]


@pytest.mark.slow
def test_c5_gzip_batch_matches_reference_goldens(engine):
    import zsamd

    recs = golden_io.batch("t64_l6_gzip")
    for lo in (0, 4096):
        buf = bytes(zsamd.corpus("text", lo, 4096, 65536))
        inputs = [buf[i * 65536:(i + 1) * 65536] for i in range(4096)]
        res = engine.compress_batch_raw(inputs, "gzip", 6)
        bad = [lo + i for i, (st, out) in enumerate(res)
               if st != 1 or (len(out), hashlib.sha256(out).digest()[:16]) != recs[lo + i]]
        assert not bad, bad[:10]


@pytest.mark.slow
@pytest.mark.parametrize("name,level", [("t256_l1_raw", 1), ("t256_l9_raw", 9)])
def test_c4_256k_streams_match_reference_goldens(engine, name, level):
    """BASELINE.json configs[3]: 4096 x 256 KiB T-corpus streams at L1 (deflate_fast) and L9 (slides, chain 4096)."""
    import zsamd

    recs = golden_io.batch(name)
    # all 4096 streams of the config, in four batches of 1024 (the per-GPU share at 8 GPUs is 512)
    total = 0
    for lo in range(0, 4096, 1024):
        buf = bytes(zsamd.corpus("text", lo, 1024, 262144))
        inputs = [buf[i * 262144:(i + 1) * 262144] for i in range(1024)]
        res = engine.compress_batch_raw(inputs, "deflate-raw", level)
        bad = [lo + i for i, (st, out) in enumerate(res)
               if st != 1 or (len(out), hashlib.sha256(out).digest()[:16]) != recs[lo + i]]
        assert not bad, bad[:10]
        total += sum(len(o) for _, o in res)
    assert total == {1: 419870313, 9: 351529571}[level]  # SURVEY 8(d) C4 totals


@pytest.mark.gpu
def test_lds_atomic_lane_order_selftest(engine):
    """The fast chain builders' hardware assumption (selftest.hip) holds on this part."""
    assert engine.selftest() == 0


@pytest.mark.parametrize("level", [1, 2, 3, 4, 6, 9])
def test_ballot_ranked_builders_equal_lane_ordered_ones(engine, level):
    """lane_order = 0: zs_k_bucket / zs_k_prev / zs_k_fast rank equal hashes by
    ballots (zs_wave_match) instead of relying on same-address LDS atomics of one
    instruction applying in lane order -- the form a device failing the self-test
    runs.  Same bytes as the default on C2 streams (65536 B: bucket + sweep), C4
    256 KiB streams (prev + match at L4-9, zs_k_fast at L1-3), all-zero streams
    (one hash per group), random and ragged streams; the C2 goldens at L6."""
    import zsamd

    specs = [("zeros", 65536), ("zeros", 200000), ("rand", 65536), ("rand", 70001), ("mixed", 131072 + 17),
             ("text", 1), ("text", 3), ("text", 64), ("text", 65537), ("ramp", 70000)]
    inputs = [corpus.make({"kind": k, "n": n, "seed": 9700 + i}) for i, (k, n) in enumerate(specs)]
    inputs += [bytes(b) for b in (zsamd.corpus("text", 0, 1, 262144), zsamd.corpus("text", 1, 1, 262144))]
    c2 = bytes(zsamd.corpus("text", 0, 64, 65536))
    inputs += [c2[i * 65536:(i + 1) * 65536] for i in range(64)]
    outs = []
    try:
        for order in (1, 0):
            engine.set_option("lane_order", order)
            outs.append(engine.compress_batch_raw(inputs, "deflate-raw", level))
    finally:
        engine.set_option("lane_order", 1)
    bad = [i for i in range(len(inputs)) if outs[0][i] != outs[1][i]]
    assert not bad, bad[:10]
    if level == 6:
        recs = golden_io.batch("t64_l6_raw")
        k0 = len(inputs) - 64
        assert all((len(outs[1][k0 + i][1]), hashlib.sha256(outs[1][k0 + i][1]).digest()[:16]) == recs[i]
                   for i in range(64))
    for d, (st, out) in zip(inputs[:len(specs)], outs[1]):
        assert st == 1 and out == oracle.compress(d, level, "deflate-raw")[1], len(d)


def test_level0_stored_layout_matches_reference_goldens(engine):
    """Level 0 (deflate_stored, deflate.ts:1140-1279) through the stream layer:
    tests/golden/deflate_level0.json, made by the reference bundle for sizes
    0..1 MiB in the three formats (gen_golden.mjs level0)."""
    import json
    import os

    g = json.load(open(os.path.join(golden_io.GOLDEN, "deflate_level0.json")))
    by_fmt = {}
    for c in g["cases"]:
        by_fmt.setdefault(c["format"], []).append(c)
    for fmt, cases in by_fmt.items():
        inputs = [corpus.text(corpus.stream_seed(c["seed_index"]), c["n"]) for c in cases]
        res = engine.compress_batch_raw(inputs, fmt, 0)
        for c, (st, out) in zip(cases, res):
            assert st == 1 and len(out) == c["out_len"] and corpus.sha256(out) == c["out_sha256"], (fmt, c["n"])
    # and they decode (stored blocks) to their inputs
    comp = engine.compress_batch(inputs, "gzip", 0)
    assert engine.decompress_batch(comp, "gzip") == inputs
