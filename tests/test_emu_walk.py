"""CPU check of zs_k_match's walk logic (tools/emu/emu_match_walk.c): the
two-chains-per-lane lock-step walk with frozen chains, the rare >= 8-byte
path and the chain >> 2 snapshot reproduce a direct longest_match
(deflate.ts:1053-1115) at every position, for the level configurations of
deflate.ts:84-100 (L4..L9).  No GPU needed; the kernel itself is checked
against the oracle by tests/test_gpu_deflate.py."""
import os
import shutil
import struct
import subprocess

import pytest

import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "emu", "emu_match_walk.c")

# (chain, nice) per level, deflate.ts:84-100 configuration_table
LEVELS = {4: (16, 16), 5: (32, 32), 6: (128, 128), 7: (256, 128), 8: (1024, 258), 9: (4096, 258)}


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path_factory.mktemp("emu") / "emu_match_walk")
    subprocess.run(["gcc", "-O2", "-o", exe, SRC], check=True)
    return exe


def _streams():
    specs = [("text", 65536), ("mixed", 65536), ("rand", 40000), ("zeros", 65536), ("ramp", 65536),
             ("text", 3), ("text", 4), ("text", 259), ("mixed", 1000), ("text", 32769), ("text", 65535)]
    return [corpus.make({"kind": k, "n": n, "seed": 7000 + i}) for i, (k, n) in enumerate(specs)]


@pytest.mark.parametrize("level", sorted(LEVELS))
def test_walk_model_matches_longest_match(emu, tmp_path, level):
    streams = _streams() if level <= 7 else _streams()[:4] + _streams()[5:9]
    blob = struct.pack("<I", len(streams)) + struct.pack("<%dI" % len(streams), *map(len, streams)) + b"".join(streams)
    f = tmp_path / "streams.bin"
    f.write_bytes(blob)
    chain, nice = LEVELS[level]
    r = subprocess.run([emu, str(f), str(chain), str(nice)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout, r.stdout
