"""The lane-per-member inflate kernel (csrc/inflate_lane.hip) run on the CPU from
its own source (tools/lane_host: host stand-ins for the few HIP names it uses),
checked against the oracle: every member it finishes (bail = 0) must carry the
oracle's bytes, consumed count and trailer check value, and clean single-call
members must not bail.  Members it bails on go to the exact path on the GPU."""
import os
import random
import struct
import subprocess
import zlib

import pytest

import corpus
import golden_io
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "tools", "lane_host")
W = {"deflate-raw": -15, "deflate": 15, "gzip": 31, "deflate64-raw": -16}


@pytest.fixture(scope="module")
def lane_host():
    subprocess.check_call(["make", "-s", "-C", HOST])
    return os.path.join(HOST, "lane_host")


def cap4(members):
    """the C-ABI's output capacities are multiples of 4 (capi.cpp rejects others)"""
    return [(c, max(4, cap & ~3)) for c, cap in members]


def run(exe, members, fmt, flags=1):
    members = cap4(members)
    data = struct.pack("<I", len(members)) + b"".join(struct.pack("<II", len(c), cap) + c for c, cap in members)
    out = subprocess.run([exe, str(W[fmt]), str(flags)], input=data, capture_output=True, check=True).stdout
    res, p = [], 0
    for _ in members:
        bail, olen, cons, want = struct.unpack_from("<4I", out, p)
        p += 16
        n = 0 if bail else olen
        res.append((bail, olen, cons, want, out[p:p + n]))
        p += n
    return res


def check(exe, members, fmt, flags=1):
    """members: [(compressed, cap)]; returns the bail flags"""
    bails = []
    members = cap4(members)
    for (c, cap), (bail, olen, cons, want, out) in zip(members, run(exe, members, fmt, flags)):
        # the trailer check runs after the lane kernel (zs_k_inflate_lane_verify):
        # a mismatch sends the member to the exact path too
        if not bail and fmt in ("deflate", "gzip"):
            bail = want != (zlib.adler32(out) if fmt == "deflate" else zlib.crc32(out))
        bails.append(bail)
        if bail:
            continue
        ost, oout, ocons, oph, omsg = oracle.decompress(c, fmt, cap=cap, reference_bugs=bool(flags & 1))
        assert ost == 1 and out == oout and cons == ocons, (fmt, len(c), ost, omsg)
    return bails


@pytest.mark.parametrize("fmt", list(W))
def test_lane_kernel_on_host_clean_members(lane_host, fmt):
    rng = random.Random(11)
    members = []
    enc = "deflate-raw" if fmt == "deflate64-raw" else fmt
    for k in range(40):
        kind = rng.choice(["text", "mixed", "ramp", "rand"])
        n = rng.choice([0, 1, 5, 100, 258, 4096, 30000, 65536])
        s = corpus.make({"kind": kind, "n": n, "seed": rng.randrange(1 << 32)})
        members.append((oracle.compress(s, rng.choice([1, 4, 6, 9]), enc)[1], n + 64))
    bails = check(lane_host, members, fmt)
    # every member that decodes cleanly in one inflate() call must finish on the
    # lane (deflate64 over deflate streams: only those without a length-258 match)
    clean = [len(c) <= 32768 and oracle.decompress(c, fmt, cap=cap)[0] == 1 for c, cap in members]
    assert not any(b for b, ok in zip(bails, clean) if ok), bails


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_lane_kernel_on_host_damaged_members(lane_host, fmt):
    """truncations, bit flips, trailing bytes, small capacities: whatever the lane
    finishes must match the oracle exactly"""
    rng = random.Random(12)
    members = []
    for k in range(60):
        s = corpus.make({"kind": rng.choice(["text", "mixed"]), "n": rng.randrange(1, 40000),
                         "seed": rng.randrange(1 << 32)})
        c = oracle.compress(s, rng.choice([1, 6, 9]), fmt)[1]
        cap = len(s) + 64
        v = k % 4
        if v == 0:
            c = c[:rng.randrange(1, len(c))]
        elif v == 1:
            b = bytearray(c)
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            c = bytes(b)
        elif v == 2:
            c = c + bytes(rng.randrange(256) for _ in range(7))
        else:
            cap = max(1, len(s) // 2)
        members.append((c, cap))
    check(lane_host, members, fmt)


def test_lane_kernel_on_host_deflate64_fixtures(lane_host):
    names = sorted(os.listdir(os.path.join(golden_io.GOLDEN, "d64")))
    cases = {c["name"]: c for c, _ in golden_io.inflate_cases()}
    members = [(open(os.path.join(golden_io.GOLDEN, "d64", f), "rb").read(), cases["d64_" + f]["out_len"] + 64)
               for f in names]
    members.append((bytes.fromhex("4b1cfdff07a3e5030000"), 70000))  # test-inflate9-length-code-285.spec.ts:9-15
    res = run(lane_host, members, "deflate64-raw")
    for f, (bail, olen, cons, want, out) in zip(names, res):
        assert not bail and corpus.sha256(out) == cases["d64_" + f]["out_sha256"], f
    assert not res[-1][0] and res[-1][4] == b"a" * 66539


@pytest.mark.parametrize("fmt", ["deflate-raw", "deflate", "gzip"])
def test_lane_kernel_on_host_large_members_reference_calls(lane_host, fmt):
    """The large-member instance (<., true>: more than 32 KiB of input, the
    reference's inflate() calls tracked per lane) against the oracle with the
    reference's window-wrap copy reproduced (inffast.ts:133-147), including the
    256 KiB member whose decode the defect changes (inffast_wrap_defect.json,
    pinned by the reference's own output)."""
    import json
    rng = random.Random(13)
    members = []
    for k in range(10):
        s = corpus.make({"kind": rng.choice(["text", "mixed"]), "n": rng.choice([70000, 150000, 262144, 400000]),
                         "seed": rng.randrange(1 << 32)})
        members.append((oracle.compress(s, rng.choice([1, 6, 9]), fmt)[1], len(s) + 64))
    j = json.load(open(os.path.join(golden_io.GOLDEN, "inffast_wrap_defect.json")))
    wrap_src = corpus.make(j["source"])
    if fmt == "deflate-raw":
        members.append((oracle.compress(wrap_src, 6, fmt)[1], len(wrap_src) + 64))
    bails = check(lane_host, members, fmt, flags=3)
    # members the reference decodes cleanly never leave the lane (with the
    # defect, a zlib / gzip member's trailer can fail: the reference reports
    # "incorrect data check" and so does the exact path the member goes to)
    clean = [oracle.decompress(c, fmt, cap=cap & ~3, reference_bugs=True)[0] == 1 for c, cap in members]
    assert not any(b for b, ok in zip(bails, clean) if ok), (bails, clean)
    if fmt == "deflate-raw":
        out = run(lane_host, members[-1:], fmt, flags=3)[0][4]
        assert corpus.sha256(out) == j["ref_out_sha256"] and out != wrap_src
