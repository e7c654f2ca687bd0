"""Multi-GPU batches: one process per GPU.

Streams are independent (no shared window or dictionary, deflate.ts:80-84), so
a batch is sharded by contiguous stream-index ranges, [k*n/G, (k+1)*n/G) on
rank k, with no collective on the data path.  The only exchange is the
per-stream size gather at the end of a batch: every rank gets the global
compressed-size array (all_gather over RCCL/xGMI on GPUs, gloo in the CPU
tests) and the exclusive prefix sum of it, i.e. where each stream lands in one
contiguous output.  Payloads can optionally be gathered to one rank.
"""
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Stream indices [lo, hi) owned by `rank` (contiguous, sizes differ by at most one)."""
    return rank * n // world, (rank + 1) * n // world


def gather_sizes(local_sizes: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather the per-stream sizes of every rank's shard into one int64 array
    of length n_total (in global stream order).  Shards may differ in length by
    one, so each rank pads to the largest shard before the collective."""
    world = dist.get_world_size(group)
    shard = max(hi - lo for lo, hi in (shard_range(n_total, world, r) for r in range(world)))
    buf = torch.zeros(shard, dtype=torch.int64, device=local_sizes.device)
    buf[: local_sizes.numel()] = local_sizes.to(torch.int64)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = [parts[r][: hi - lo] for r, (lo, hi) in enumerate(shard_range(n_total, world, r) for r in range(world))]
    return torch.cat(out)


def global_offsets(sizes: torch.Tensor) -> torch.Tensor:
    """Exclusive prefix sum: byte offset of every stream in the concatenated output."""
    off = torch.zeros_like(sizes)
    if sizes.numel() > 1:
        off[1:] = torch.cumsum(sizes[:-1], 0)
    return off


def compress_sharded(inputs: Sequence[bytes], compress: Callable[[List[bytes]], List[bytes]], group=None,
                     device: Optional[torch.device] = None, gather_to: Optional[int] = None):
    """Compress this rank's shard of `inputs` with `compress` (the rank's engine
    call) and return (local_outputs, global_sizes, global_offsets, joined) where
    `joined` is the concatenation of every stream's output on rank `gather_to`
    (None elsewhere, or when gather_to is None)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(len(inputs), world, rank)
    outs = compress(list(inputs[lo:hi]))
    dev = device or torch.device("cpu")
    sizes = gather_sizes(torch.tensor([len(o) for o in outs], dtype=torch.int64, device=dev), len(inputs), group)
    offs = global_offsets(sizes)
    joined = None
    if gather_to is not None:
        # payloads are padded to the largest shard total for the collective
        totals = [int(sizes[a:b].sum()) for a, b in (shard_range(len(inputs), world, r) for r in range(world))]
        cap = max(totals) if totals else 0
        mine = torch.zeros(cap, dtype=torch.uint8, device=dev)
        blob = b"".join(outs)
        if blob:
            mine[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        parts = [torch.empty_like(mine) for _ in range(world)] if rank == gather_to else None
        dist.gather(mine, parts, dst=gather_to, group=group)
        if rank == gather_to:
            joined = b"".join(bytes(parts[r][: totals[r]].cpu().numpy()) for r in range(world))
    return outs, sizes, offs, joined
