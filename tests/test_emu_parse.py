"""CPU check of the two-kernel lazy parse's algorithm (tools/emu_parse_split.py
models zs_k_parse_a / zs_k_parse_b of deflate_parse2.hip lane by lane: the
per-range speculative segments, the lock-step merges, the serial range
fallback and the per-stream joins) against the serial lazy parse of
deflate_slow (deflate.ts:1352-1448) on the same match table.  Small segments
stress the merges and joins.  No GPU needed; the kernels are checked against
the one-wave parse and the oracle by tests/test_gpu_deflate.py."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import corpus  # noqa: E402
from emu_parse_split import split_parse  # noqa: E402
from emu_pipeline import stages  # noqa: E402


@pytest.mark.parametrize("kind,seed,n", [("text", 3, 777), ("text", 4, 9000), ("mixed", 5, 6000), ("rand", 1, 3000),
                                         ("zeros", 0, 5000), ("text", 6, 2049)])
@pytest.mark.parametrize("level", [4, 6, 9])
def test_split_parse_model_matches_serial_parse(kind, seed, n, level):
    data = bytes(n) if kind == "zeros" else getattr(corpus, kind)(seed, n)
    _, enc, syms = stages(data, level)
    for seg, lanes in ((64, 64), (8, 16), (4, 8)):
        got, _ = split_parse(data, enc, level, seg, lanes)
        assert got == syms, (seg, lanes)
