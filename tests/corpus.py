"""Deterministic synthetic corpora, SURVEY.md Appendix B.

Same spec as tests/golden/corpus.mjs (used with the reference bundle to make
goldens) and zlib-streams-ts_amd/csrc/corpus.cpp (bulk generation for the
bench).  Pure Python: fine for the small parity cases.
"""
import hashlib

VOCAB = (
    "the of and to in is that for it as was with be by on not he this are or his from at which but have an "
    "they you were her she there been one all we their has would when if so no will more can out said up what "
    "about its into them than only other new some could time these two may then do first any my now such like "
    "our over man me even most made after also did many before must through back years where much your way well "
    "down should because each just those people how too little state good very make world still own see men work "
    "long get here between both life being under never day same another know while last might us great old year "
    "off come since against go came right used take three"
).split(" ")
VOCAB_B = [w.encode() for w in VOCAB]
assert len(VOCAB) == 144


def stream_seed(i):
    return (0x9E3779B9 ^ i) & 0xFFFFFFFF


def _xs(seed):
    s = (seed & 0xFFFFFFFF) or 1
    while True:
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        yield s


def text(seed, n):
    r = _xs(seed)
    out = bytearray()
    w = 0
    while len(out) < n:
        a = next(r)
        idx = min(a % 144, (a >> 12) % 144)
        out += VOCAB_B[idx]
        if len(out) < n:
            w += 1
            out.append(10 if w % 13 == 0 else 32)
    return bytes(out[:n])


def mixed(seed, n):
    out = bytearray(text(seed, n))
    r = _xs((seed ^ 0x85EBCA6B) & 0xFFFFFFFF)
    k = 0
    while k + 8192 <= n:
        for j in range(1024):
            out[k + 4096 + j] = next(r) & 0xFF
        k += 8192
    return bytes(out)


def rand(seed, n):
    r = _xs(seed)
    return bytes(next(r) & 0xFF for _ in range(n))


def make(spec):
    k = spec["kind"]
    if k == "text":
        return text(spec["seed"], spec["n"])
    if k == "mixed":
        return mixed(spec["seed"], spec["n"])
    if k == "rand":
        return rand(spec["seed"], spec["n"])
    if k == "zeros":
        return bytes(spec["n"])
    if k == "ramp":
        return bytes(j % 251 for j in range(spec["n"]))
    if k == "hex":
        return bytes.fromhex(spec["hex"])
    raise ValueError(k)


def sha256(b):
    return hashlib.sha256(b).hexdigest()


def patchwork(seed, n):
    """Test-only (not in corpus.mjs): n bytes of M-, R- and T-corpus stretches of 3,000 .. 40,000 bytes, so that
    an encoder's blocks alternate between coded and stored (the R stretches)."""
    import random

    rng = random.Random(seed)
    parts, k = [], 0
    while k < n:
        kind, m = rng.choice(["mixed", "rand", "text"]), rng.choice([3000, 20000, 40000])
        parts.append(make({"kind": kind, "n": m, "seed": stream_seed(rng.randrange(4096))}))
        k += m
    return b"".join(parts)[:n]
