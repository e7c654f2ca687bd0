"""Loaders for the committed golden fixtures (tests/golden/, made by gen_golden.mjs
from the reference bundle)."""
import json
import os
import struct

import corpus

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def deflate_cases():
    g = json.load(open(os.path.join(GOLDEN, "deflate_small.json")))
    side = json.load(open(os.path.join(GOLDEN, "deflate_small_inputs.json")))
    out = []
    for c in g["cases"]:
        spec = c["spec"]
        data = bytes.fromhex(side[spec["sha256"]]) if spec["kind"] == "hex_sha" else corpus.make(spec)
        out.append((c, data))
    return out


def inflate_cases():
    g = json.load(open(os.path.join(GOLDEN, "inflate_small.json")))
    out = []
    for c in g["cases"]:
        if c.get("in_hex") is not None:
            data = bytes.fromhex(c["in_hex"])
        elif c["name"].startswith("d64_"):
            data = open(os.path.join(GOLDEN, "d64", c["name"][4:]), "rb").read()
        else:
            data = None  # regenerable streams are rebuilt by the test from their spec
        out.append((c, data))
    return out


def batch(name):
    """[(len, sha256[:16] bytes)] per stream for tests/golden/batch_<name>.bin."""
    b = open(os.path.join(GOLDEN, "batch_%s.bin" % name), "rb").read()
    return [(struct.unpack_from("<I", b, 20 * i)[0], b[20 * i + 4: 20 * i + 20]) for i in range(len(b) // 20)]
