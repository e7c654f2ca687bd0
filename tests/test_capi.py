"""CPU-side checks of the drop-in boundary: libzsgpu.so loads and exports every
symbol include/zs_gpu.h declares; host helpers behave without a GPU."""
import ctypes
import os
import re

import pytest

import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "zs_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zs_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import zsamd

    L = zsamd.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_no_gpu_means_loud_failure():
    import zsamd

    if os.environ.get("ZS_EXPECT_GPU"):
        pytest.skip("GPU box")
    try:
        import torch

        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(zsamd.ZsUnavailable):
        zsamd.Engine(0)


def test_deflate_bound_matches_reference_formula():
    import zsamd

    # deflate.ts:615-674 (memLevel 8, wbits 15): n + n>>12 + n>>14 + n>>25 + 7 + wraplen
    for n in [0, 1, 100, 65536, 262144, 10 ** 7]:
        for fmt, wl in [("deflate-raw", 0), ("deflate", 6), ("gzip", 18)]:
            b = n + (n >> 12) + (n >> 14) + (n >> 25) + 7 + wl
            assert zsamd.deflate_bound(n, fmt) == b
            assert zsamd.deflate_capacity(n, fmt) == (b + 3) & ~3


def test_corpus_generator_matches_spec():
    import zsamd

    t = zsamd.corpus("text", 0, 2, 65536)
    assert bytes(t[:65536]) == corpus.text(corpus.stream_seed(0), 65536)
    # SURVEY.md Appendix B first-stream digest
    assert corpus.sha256(bytes(t[:65536])).startswith("baed0f1f7ad2479ec442f59de3e63465")
    m = zsamd.corpus("mixed", 7, 1, 50000)
    assert bytes(m) == corpus.mixed(corpus.stream_seed(7), 50000)
    r = zsamd.corpus("rand", 3, 1, 1000)
    assert bytes(r) == corpus.rand(corpus.stream_seed(3), 1000)


def test_format_wbits_mapping():
    import zsamd

    # streams.ts:220,233
    assert [zsamd.compress_wbits(f) for f in ("gzip", "deflate-raw", "deflate", "other")] == [31, -15, 15, 15]
    assert [zsamd.decompress_wbits(f) for f in ("gzip", "deflate-raw", "deflate64-raw", "deflate")] == [31, -15, -16, 15]
