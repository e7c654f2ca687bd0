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
