"""Multi-GPU plumbing for GOP-sharded coding.

GOPs are independent (each starts from its own I-frame; the only dependency, ``x_prev``, is inside
a GOP, ``models.py:372-376``), so ranks never exchange data while coding. After coding, one
collective round moves the small results: the per-rank elapsed time (MAX), per-rank metrics
(all_gather of a few floats) and every rank's bitstream bytes to rank 0 only (gather of lengths,
then gather of payloads zero-padded to the largest rank's). With the seeded (untrained) weights a
1080p P-frame codes to ~1.3 MB (~5 bpp), so 16 GOPs per rank are ~229 MB per rank and ~1.8 GB
onto rank 0 at 8 ranks; a trained DVC at 0.137 bpp would be ~36 KB per frame. All of it after the
timed region.
Works with ``nccl`` (RCCL on ROCm; device tensors) and ``gloo`` (CPU tensors, tests).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_gops(n_gops: int, rank: int, world: int):
    """GOP g goes to rank g % world (round-robin)."""
    return [g for g in range(n_gops) if g % world == rank]


def shard_views(n_views: int, rank: int, world: int):
    """Camera view v goes to rank v % world (BASELINE configs[4]: 8 views, one per GPU). DVC codes
    each view as an independent stream; the reference's cross-view MCVC coupling is out of scope."""
    return [v for v in range(n_views) if v % world == rank]


def _dev(device):
    return torch.device(device) if device is not None else torch.device("cpu")


def max_over_ranks(value: float, device=None) -> float:
    t = torch.tensor([value], dtype=torch.float64, device=_dev(device))
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_stats(stats, device=None):
    """all_gather a 1-D float64 vector of per-rank statistics -> [world, n] numpy array."""
    t = torch.as_tensor(np.asarray(stats, np.float64), device=_dev(device))
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return t.cpu().numpy()[None]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.stack(out).cpu().numpy()


def gather_bytes(payload: bytes, device=None, dst: int = 0):
    """Every rank contributes one byte string; rank ``dst`` gets the list of all ranks' strings,
    the other ranks get None (the bitstreams go to one writer, not to everyone).
    Two collectives: a gather of the lengths, then a gather of the zero-padded payloads
    (torch.distributed.gather: RCCL send/recv under nccl, gloo on CPU)."""
    dev = _dev(device)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [payload]
    world = dist.get_world_size()
    me = dist.get_rank()
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    lens = [torch.zeros_like(n) for _ in range(world)] if me == dst else None
    dist.gather(n, lens, dst=dst)
    # every rank needs the common padded size: one tiny all_reduce(MAX) of the length
    cap_t = n.clone()
    dist.all_reduce(cap_t, op=dist.ReduceOp.MAX)
    cap = max(int(cap_t.item()), 1)
    buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    if payload:
        buf[: len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)] if me == dst else None
    dist.gather(buf, outs, dst=dst)
    if me != dst:
        return None
    return [bytes(o[: int(L.item())].cpu().numpy().tobytes()) for o, L in zip(outs, lens)]
