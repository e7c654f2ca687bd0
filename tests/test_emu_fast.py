"""CPU check of the group-speculative deflate_fast parser (levels 1..3) that
zs_k_fast (deflate_fast.hip) implements: tools/emu/emu_fast_group.c replays
groups of 64 positions from speculative per-lane chain walks over the superset
of inserted positions, re-walking only the steps whose walk met a position
deflate_fast skips (deflate.ts:1310-1322), and must produce the symbols and
block cuts of a serial transcription of deflate_fast (deflate.ts:1281-1350)
with the same head[]/prev[] tables and slide schedule (deflate.ts:180-190).
No GPU needed; the kernel itself is pinned by the reference goldens in
tests/test_gpu_deflate.py."""
import shutil
import struct
import subprocess
import os

import pytest

import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "emu", "emu_fast_group.c")

# (chain, max_lazy, nice) per level, deflate.ts:84-100 configuration_table
LEVELS = {1: (4, 4, 8), 2: (8, 5, 16), 3: (32, 6, 32)}


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path_factory.mktemp("emu") / "emu_fast_group")
    subprocess.run(["gcc", "-O2", "-o", exe, SRC], check=True)
    return exe


def _streams():
    specs = [("text", 262144), ("mixed", 200000), ("rand", 40000), ("zeros", 100000), ("ramp", 70000),
             ("text", 1), ("text", 3), ("text", 4), ("text", 13), ("text", 259), ("mixed", 1000),
             ("text", 32769), ("text", 65535), ("text", 65537), ("zeros", 65537), ("text", 98304 + 300)]
    out = [corpus.make({"kind": k, "n": n, "seed": 9100 + i}) for i, (k, n) in enumerate(specs)]
    b = bytearray(corpus.rand(78, 90000))  # a candidate at exactly MAX_DIST
    b[40000:40020] = b[40000 - 32506:40000 - 32506 + 20]
    out.append(bytes(b))
    return out


@pytest.mark.parametrize("level", sorted(LEVELS))
def test_group_parse_matches_serial_deflate_fast(emu, level):
    chain, lazy, nice = LEVELS[level]
    blob = b"".join(struct.pack("<4I", chain, lazy, nice, len(s)) + s for s in _streams())
    r = subprocess.run([emu], input=blob, capture_output=True, timeout=600)
    out = r.stdout.decode()
    assert r.returncode == 0, out + r.stderr.decode()
    assert "MISMATCH" not in out, out


REC_SRC = os.path.join(ROOT, "tools", "emu", "emu_fast_rec.c")


@pytest.fixture(scope="module")
def emu_rec(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path_factory.mktemp("emu") / "emu_fast_rec")
    subprocess.run(["gcc", "-O2", "-o", exe, REC_SRC], check=True)
    return exe


@pytest.mark.parametrize("level", sorted(LEVELS))
def test_member_run_walks_match_serial_deflate_fast(emu_rec, level):
    """zs_k_fast_mr's construction (a variant, not in the product: tools/variants/deflate_fast_mr.hip, measured
    slower): chains read as runs of the superset in
    which every position is inserted (the bucket sort's members, 32 entries per lane walk), filtered by a bitmap of
    the truly inserted positions before the group and speculative inside it, the walks that run out of entries
    left to the replay's slow step -- the symbols and block cuts of the serial deflate_fast with the reference's
    head[] / prev[] tables and slide schedule."""
    chain, lazy, nice = LEVELS[level]
    blob = b"".join(struct.pack("<5I", chain, lazy, nice, len(s), 32) + s for s in _streams())
    r = subprocess.run([emu_rec], input=blob, capture_output=True, timeout=600)
    out = r.stdout.decode()
    assert r.returncode == 0, out + r.stderr.decode()
    assert "MISMATCH" not in out and out.count("ok n=") == len(_streams()), out
