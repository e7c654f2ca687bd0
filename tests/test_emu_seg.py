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


def test_piecewise_call_state_with_stored_blocks():
    """Stored blocks (inflate.ts:631-672) among the pieces: the plan replays the COPY state's call ends from each
    stored block's input offset and length (zs_refcalls_t::stored), and the wrap decisions of the pieces after it
    stay the serial replay's -- on hand-built members of stored blocks only (level-0 style; the oracle does not
    restate level 0) and of stored and fixed blocks, on R-corpus bytes at L6 (the encoder's stored blocks), on a
    patchwork member whose reference decode has a window-wrap copy behind its stored blocks, and on stored blocks
    between an encoder's dynamic blocks with an empty one whose header straddles a sub-chunk end."""
    import bitbuild
    from test_gpu_seg import _dyn_stored_member

    rng = random.Random(17)
    src = corpus.text(11, 150000) + corpus.rand(12, 100000) + corpus.make({"kind": "mixed", "n": 100000, "seed": 13})
    cases = [bitbuild.stored_mix(random.Random(1), 262144, src, level0=True)[0],
             bitbuild.stored_mix(random.Random(2), 200000, src)[0],
             oracle.compress(corpus.rand(8, 200000), 6, "deflate-raw")[1],
             oracle.compress(corpus.patchwork(208, 262144), 6, "deflate-raw")[1],
             # an empty stored block whose LEN / NLEN straddle byte 65,536, an encoder's dynamic block after it
             _dyn_stored_member(random.Random(20), 262144, src, 65536)]
    for i, c in enumerate(cases):
        st, ref = oracle.decompress(c, "deflate-raw", cap=1 << 20, reference_bugs=True)[:2]
        assert st == 1
        syms, _, _ = emu_seg.decode(c)
        assert any(x.get("stored") for x in syms), i
        w, npieces, _ = emu_seg.check(c, ref, 300, rng)
        assert npieces > 1
        if i == 3:
            assert w >= 1 and ref != corpus.patchwork(208, 262144)
