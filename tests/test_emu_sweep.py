"""CPU check of the L4..L9 match finder's algorithm (tools/emu/emu_bucket_sweep.c
models zs_k_bucket + zs_k_sweep of deflate_sweep.hip over capi.cpp's windows):
the counting sort by (hash, position), the lock-step sweep over bucket predecessors with 12-byte signatures, the liveness keys,
the chain >> 2 snapshot and the deferred long candidates (with the re-walk
after a fifth) reproduce a direct longest_match (deflate.ts:1053-1115) at
every position, for both budgets and the slide-NIL flag, at the level
configurations of deflate.ts:84-100 (L4..L9).  No GPU needed; the kernels
themselves are checked against the chain-walk kernel and the oracle by
tests/test_gpu_deflate.py (test_sweep_match_table_equals_chain_walk)."""
import os
import shutil
import struct
import subprocess

import pytest

import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "emu", "emu_bucket_sweep.c")

# (chain, nice) per level, deflate.ts:84-100 configuration_table
LEVELS = {4: (16, 16), 5: (32, 32), 6: (128, 128), 7: (256, 128), 8: (1024, 258), 9: (4096, 258)}


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path_factory.mktemp("emu") / "emu_bucket_sweep")
    subprocess.run(["gcc", "-O2", "-o", exe, SRC], check=True)
    return exe


def _streams():
    specs = [("text", 65536), ("mixed", 65536), ("rand", 40000), ("zeros", 65536), ("ramp", 65536),
             ("text", 3), ("text", 4), ("text", 13), ("text", 259), ("mixed", 1000), ("text", 32769),
             ("text", 65535), ("text", 65537), ("zeros", 65537)]
    out = [corpus.make({"kind": k, "n": n, "seed": 7000 + i}) for i, (k, n) in enumerate(specs)]
    # 7-bit streams take the 8-byte signature [X, b3..b9]: random 7-bit bytes collide in the 15-bit hash with
    # different first three bytes everywhere; a small alphabet gives long matches and deep chains
    out.append(bytes(x & 0x7F for x in corpus.rand(91, 65536)))
    out.append(bytes(0x41 + (x & 3) for x in corpus.rand(92, 65536)))
    out.append(bytes(x & 0x7F for x in corpus.rand(93, 20000)) + corpus.text(94, 45536))
    b = bytearray(corpus.rand(77, 65536))  # a head candidate at exactly MAX_DIST
    b[40000:40020] = b[40000 - 32506:40000 - 32506 + 20]
    out.append(bytes(b))
    return out


@pytest.mark.parametrize("level", sorted(LEVELS))
def test_sweep_model_matches_longest_match(emu, tmp_path, level):
    streams = _streams()
    blob = struct.pack("<I", len(streams)) + struct.pack("<%dI" % len(streams), *map(len, streams)) + b"".join(streams)
    f = tmp_path / "streams.bin"
    f.write_bytes(blob)
    chain, nice = LEVELS[level]
    r = subprocess.run([emu, str(f), str(chain), str(nice)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout, r.stdout
    assert " 0 in 7-bit" not in r.stdout  # both signature forms were exercised


def _long_streams():
    specs = [("text", 65538), ("mixed", 100000), ("text", 262144), ("zeros", 131073), ("rand", 98317)]
    out = [corpus.make({"kind": k, "n": n, "seed": 8100 + i}) for i, (k, n) in enumerate(specs)]
    b = bytearray(corpus.rand(78, 200000))  # head candidates at exactly MAX_DIST around the window seams
    for at in (65519, 65520, 98272, 150001):
        b[at:at + 40] = b[at - 32506:at - 32506 + 40]
    out.append(bytes(b))
    out.append(bytes(x & 0x7F for x in corpus.rand(95, 150000)))
    return out


@pytest.mark.parametrize("level", [4, 7])
def test_windowed_sweep_model_matches_longest_match(emu, tmp_path, level):
    """Streams over 65,537 bytes: the sweep's windows (capi.cpp sweep_table -- a first window owning [0, 65520),
    then 32,752 own positions after a 32,768-position look-back, u16 window-relative members) give every position
    exactly once the result of a direct longest_match over the whole stream's chain."""
    streams = _long_streams()
    blob = struct.pack("<I", len(streams)) + struct.pack("<%dI" % len(streams), *map(len, streams)) + b"".join(streams)
    f = tmp_path / "long.bin"
    f.write_bytes(blob)
    chain, nice = LEVELS[level]
    r = subprocess.run([emu, str(f), str(chain), str(nice)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout, r.stdout
    assert "checked %d positions" % sum(len(s) - 2 for s in streams) in r.stdout, r.stdout


DEMAND_SRC = os.path.join(ROOT, "tools", "emu", "emu_demand.c")
# (chain, nice, good, lazy) per level, deflate.ts:84-100 configuration_table
LEVELS_DW = {4: (16, 16, 4, 4), 5: (32, 32, 8, 16), 6: (128, 128, 8, 16), 7: (256, 128, 8, 32), 8: (1024, 258, 32, 128),
             9: (4096, 258, 32, 258)}


@pytest.fixture(scope="module")
def emu_demand(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path_factory.mktemp("emu") / "emu_demand")
    subprocess.run(["gcc", "-O2", "-o", exe, DEMAND_SRC], check=True)
    return exe


@pytest.mark.parametrize("level", sorted(LEVELS_DW))
def test_demand_walk_model_matches_serial_parse(emu_demand, tmp_path, level):
    """The demand-mode variant (tools/variants/r05_paths.patch, not in the product: zs_k_sweep takes chain >> 2
    steps, zs_k_parse_dw walks steps chain >> 2 + 1
    .. chain where the parse asks for the full budget): its walk rule (stop at limit or where member positions stop
    falling) gives longest_match's full-budget result at every walked position, and the parse over it emits the
    serial deflate_slow's symbols."""
    streams = _streams()
    blob = struct.pack("<I", len(streams)) + struct.pack("<%dI" % len(streams), *map(len, streams)) + b"".join(streams)
    f = tmp_path / "streams.bin"
    f.write_bytes(blob)
    chain, nice, good, lazy = LEVELS_DW[level]
    r = subprocess.run([emu_demand, str(f), str(chain), str(nice), str(good), str(lazy)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "walk mismatches 0, streams with other symbols 0" in r.stdout, r.stdout
