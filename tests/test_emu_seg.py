"""CPU check of the segmented decode's call-state plan (tools/emu/emu_seg.py, the
model of inflate_seg.hip's zs_k_seg_plan): for members decoded in pieces, the
reference's inflate() call state at every piece start (streams.ts:78-93,
inflate.ts:282-322) planned from the pieces' counts and events gives the same
window-wrap copy decisions (inffast.ts:127-147) as a serial replay of the whole
member, and the serial expansion equals the oracle's decode with the reference's
defect (reference_bugs = 1).  No GPU needed; the kernels are pinned on the GPU by
tests/test_gpu_seg.py and the reference's own decode of the 256 KiB T-corpus set."""
import os
import random
import sys

import corpus
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "emu"))

import emu_seg  # noqa: E402


def test_piecewise_call_state_equals_serial_replay():
    rng = random.Random(11)
    for kind, size, lv in [("mixed", 120000, 6), ("text", 90000, 9), ("mixed", 70000, 1)]:
        src = corpus.make({"kind": kind, "n": size, "seed": corpus.stream_seed(rng.randrange(4096))})
        c = oracle.compress(src, lv, "deflate-raw")[1]
        ref = oracle.decompress(c, "deflate-raw", cap=size, reference_bugs=True)[1]
        for ps in (40, 700):
            _, npieces, _ = emu_seg.check(c, ref, ps, rng)  # (asserts inside)
            assert npieces > 1


def test_piecewise_call_state_on_the_reference_wrap_defect_member():
    """tests/golden/inffast_wrap_defect.json: a 256 KiB M-corpus member whose reference decode differs from its
    source (the window-wrap copy); the model's serial expansion equals the reference's digest and its pieces make
    the same wrap decisions."""
    import hashlib
    import json

    d = json.load(open(os.path.join(ROOT, "tests", "golden", "inffast_wrap_defect.json")))
    src = corpus.make(d["source"])
    c = oracle.compress(src, 6, "deflate-raw")[1]
    assert hashlib.sha256(c).hexdigest() == d["compressed_sha256"]
    ref = oracle.decompress(c, "deflate-raw", cap=len(src), reference_bugs=True)[1]
    assert hashlib.sha256(ref).hexdigest() == d["ref_out_sha256"] and ref != src
    w, npieces, _ = emu_seg.check(c, ref, 2000, random.Random(3))
    assert w >= 1 and npieces > 1
