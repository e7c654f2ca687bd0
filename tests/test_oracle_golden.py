"""The C oracle (oracle/) pinned against vectors produced by the reference itself.

Goldens come from running the reference bundle in place (tests/golden/gen_golden.mjs);
the KATs are the reference's own tests (cited inline)."""
import hashlib
import json
import os

import pytest

import corpus
import golden_io
import oracle


def test_deflate_goldens_all_levels_formats():
    cases = golden_io.deflate_cases()
    assert len(cases) > 500
    bad = []
    for c, data in cases:
        assert corpus.sha256(data) == c["in_sha256"]
        st, out, ph = oracle.compress(data, c["level"], c["format"])
        assert st == oracle.Z_STREAM_END
        if corpus.sha256(out) != c["out_sha256"] or len(out) != c["out_len"]:
            bad.append((c["spec"].get("kind"), c["in_len"], c["level"], c["format"]))
        if "out_hex" in c:
            assert out.hex() == c["out_hex"]
    assert not bad, bad[:10]


def test_empty_and_hello_kats():
    # test/round-trip/test-streams-empty-input.ts:32-35 -> [3, 0]
    assert oracle.compress(b"", 6, "deflate-raw")[1] == bytes([3, 0])
    # SURVEY A10 (probed with the bundle): "hello" at L6
    assert oracle.compress(b"hello", 6, "deflate-raw")[1].hex() == "cb48cdc9c90700"
    assert oracle.compress(b"", 6, "deflate")[1].hex() == "789c030000000001"
    assert oracle.compress(b"", 6, "gzip")[1].hex() == "1f8b08000000000000ff0300" + "00" * 8


def test_checksum_kats():
    # test/coverage-targets/coverage-crc32.spec.ts:9-14
    assert oracle.crc32(b"hello") == 0x3610A686
    assert oracle.crc32(b"") == 0
    # test/coverage-targets/coverage-adler32.spec.ts:10-21 (initial adler 0)
    assert oracle.adler32(bytes([5]), 0) == (5 << 16) | 5
    assert oracle.adler32(bytes([1, 2, 3]), 0) == (10 << 16) | 6


def test_inflate_goldens():
    bad = []
    for c, data in golden_io.inflate_cases():
        if data is None:
            continue
        st, out, cons, ph, msg = oracle.decompress(data, c["format"], cap=4 << 20)
        ok = st == oracle.Z_STREAM_END
        err = "" if ok else oracle.stream_error_text(st, ph)
        if ok != c["ok"] or err != c["err"] or corpus.sha256(out) != c["out_sha256"]:
            bad.append((c["name"], st, ph, msg, c["err"]))
    assert not bad, bad


def test_inflate_roundtrip_goldens_regenerated():
    # rt_* cases: reference-compressed corpora decoded by the reference
    spec_by_kind = {"text": {"kind": "text", "seed": corpus.stream_seed(20), "n": 65536},
                    "mixed": {"kind": "mixed", "seed": corpus.stream_seed(21), "n": 65536},
                    "rand": {"kind": "rand", "seed": 22, "n": 5000}, "zeros": {"kind": "zeros", "n": 70000}}
    cfmt = {"deflate-raw": "deflate-raw", "deflate": "deflate", "gzip": "gzip", "deflate64-raw": "deflate-raw"}
    n = 0
    for c, data in golden_io.inflate_cases():
        if not c["name"].startswith("rt_"):
            continue
        dfmt = c["format"]
        kind = c["name"].split("_")[-1]
        src = corpus.make(spec_by_kind[kind])
        st, comp, _ = oracle.compress(src, 6, cfmt[dfmt])
        assert corpus.sha256(comp) == c["in_sha256"]
        st, out, cons, ph, msg = oracle.decompress(comp, dfmt, cap=1 << 20)
        ok = st == oracle.Z_STREAM_END
        assert ok == c["ok"] and ("" if ok else oracle.stream_error_text(st, ph)) == c["err"], (c["name"], st, ph)
        assert corpus.sha256(out) == c["out_sha256"]
        if dfmt != "deflate64-raw" or kind != "zeros":  # zeros use length 258 = deflate64 code 285 (3 + 16 bits)
            assert out == src
        n += 1
    assert n == 16


def test_inffast_window_wrap_defect_is_reproduced():
    """The reference's inflate_fast mis-copies when a window-sourced match wraps the
    ring and the remainder fits in w_next (inffast.ts:139-147 reads `output` from 0).
    The oracle reproduces the reference's corrupt bytes exactly (reference_bugs=True)
    and decodes correctly otherwise.  The GPU engine reproduces the reference's bytes
    by default and decodes with zlib semantics under inflate_ref_wrap = 0
    (tests/test_gpu_inflate.py::test_inffast_window_wrap_defect_is_reproduced)."""
    j = json.load(open(os.path.join(golden_io.GOLDEN, "inffast_wrap_defect.json")))
    src = corpus.make(j["source"])
    st, comp, _ = oracle.compress(src, 6, "deflate-raw")
    assert corpus.sha256(comp) == j["compressed_sha256"]
    assert j["ref_equals_source"] is False
    st, out, *_ = oracle.decompress(comp, "deflate-raw", cap=1 << 19, reference_bugs=True)
    assert corpus.sha256(out) == j["ref_out_sha256"]
    st, out, *_ = oracle.decompress(comp, "deflate-raw", cap=1 << 19, reference_bugs=False)
    assert out == src


@pytest.mark.parametrize("name,n", [("t64_l6_raw", 8), ("m64_l6_raw", 4), ("t64_l6_gzip", 4)])
def test_batch_goldens_first_streams(name, n):
    recs = golden_io.batch(name)
    gen = corpus.mixed if name.startswith("m") else corpus.text
    fmt = "gzip" if name.endswith("gzip") else "deflate-raw"
    level = int(name.split("_")[1][1:])
    for i in range(n):
        st, out, _ = oracle.compress(gen(corpus.stream_seed(i), 65536), level, fmt)
        assert (len(out), hashlib.sha256(out).digest()[:16]) == recs[i]


def test_batch_golden_totals_match_survey():
    # SURVEY.md Appendix B / BASELINE.md
    assert sum(l for l, _ in golden_io.batch("t64_l6_raw")) == 91855591
    assert sum(l for l, _ in golden_io.batch("m64_l6_raw")) == 123877078
    assert sum(l for l, _ in golden_io.batch("t64_l6_gzip")) == 183855998


def test_oracle_decodes_long_deflate64_copies():
    """The hand-built deflate64 members of tests/bitbuild.py (length code 285 up to
    65,538 bytes, distance 65,536): the oracle gives their plain LZ77 expansion,
    and the reference's own length-285 KAT (test-inflate9-length-code-285.spec.ts:9-15)
    goes through the same builder's path."""
    import bitbuild

    for comp, exp in bitbuild.long_copies():
        st, out, cons, ph, msg = oracle.decompress(comp, "deflate64-raw", cap=len(exp) + 16)
        assert st == 1 and out == exp and cons == len(comp)
    kat = bytes.fromhex("4b1cfdff07a3e5030000")
    st, out, cons, _, _ = oracle.decompress(kat, "deflate64-raw", cap=70000)
    assert st == 1 and out == b"a" * 66539
