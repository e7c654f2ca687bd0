"""Multi-GPU sharding logic (zsamd/shard.py) on CPU: world_size 2 over gloo.
Each rank compresses its shard with the oracle (standing in for its GPU engine),
gathers sizes, and rank 0 gathers the payloads; the result must equal a
single-process run."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import corpus
import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs():
    data = [corpus.text(corpus.stream_seed(i), 3000 + 517 * i) for i in range(7)]
    return data + [b"", b"x" * 5000]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import zsamd.shard as shard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        inputs = _inputs()
        comp = lambda xs: [oracle.compress(x, 6, "deflate-raw")[1] for x in xs]
        outs, sizes, offs, joined = shard.compress_sharded(inputs, comp, gather_to=0)
        q.put((rank, shard.shard_range(len(inputs), world, rank), [len(o) for o in outs], sizes.tolist(),
               offs.tolist(), joined))
    finally:
        dist.destroy_process_group()


def _gz_members():
    return [oracle.compress(x, 6, "gzip")[1] for x in _inputs()]


def _decode_worker(rank, world, port, q):
    """The decode flow of bench.py's C4/C5 lines at world size 3: each rank
    gunzips its shard; one batch of 9 members and one of 2 members (rank 2's
    shard is empty, so it joins the collectives with zero-length tensors)."""
    import torch.distributed as dist
    import zsamd.shard as shard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dec = lambda xs: [oracle.decompress(x, "gzip")[1] for x in xs]
        got = []
        for members in (_gz_members(), _gz_members()[:2]):
            outs, sizes, offs, joined = shard.compress_sharded(members, dec, gather_to=world - 1)
            got.append(([len(o) for o in outs], sizes.tolist(), offs.tolist(), joined))
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_shard_ranges_cover_batch():
    import zsamd.shard as shard

    for n in (0, 1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            rs = [shard.shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_two_rank_gloo_batch_equals_single_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    inputs = _inputs()
    ref = [oracle.compress(x, 6, "deflate-raw")[1] for x in inputs]
    ref_sizes = [len(r) for r in ref]
    ref_offs = [sum(ref_sizes[:i]) for i in range(len(ref))]
    for rank, (lo, hi), local, sizes, offs, joined in res:
        assert local == ref_sizes[lo:hi]
        assert sizes == ref_sizes and offs == ref_offs
        assert joined == (b"".join(ref) if rank == 0 else None)


def test_three_rank_gloo_decode_equals_single_process():
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_decode_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    plain = _inputs()
    for case, n in enumerate((len(plain), 2)):
        ref = plain[:n]
        ref_sizes = [len(r) for r in ref]
        ref_offs = [sum(ref_sizes[:i]) for i in range(n)]
        for rank, got in res:
            local, sizes, offs, joined = got[case]
            lo, hi = rank * n // world, (rank + 1) * n // world
            assert local == ref_sizes[lo:hi]
            assert sizes == ref_sizes and offs == ref_offs
            assert joined == (b"".join(ref) if rank == world - 1 else None)
