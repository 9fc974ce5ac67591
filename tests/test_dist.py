"""CPU: the multi-GPU sharding/gather path with the gloo backend, world_size 2 (the GPU box
runs the same code over RCCL)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fastvideocodec_amd import dist as fd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = fd.shard_gops(7, rank, world)
        t = fd.max_over_ranks(1.0 + rank)
        st = fd.gather_stats([rank, len(mine), 10.0 * rank])
        rng = np.random.default_rng(rank)
        payload = rng.integers(0, 256, 1000 + 37 * rank, dtype=np.uint8).tobytes()
        got = fd.gather_bytes(payload)  # to rank 0 only
        empty = fd.gather_bytes(b"" if rank == 0 else b"x")
        if rank == 0:
            ok = got[1] == np.random.default_rng(1).integers(0, 256, 1037, dtype=np.uint8).tobytes()
            q.put((rank, mine, t, st.tolist(), [len(g) for g in got], ok, empty))
        else:
            q.put((rank, mine, t, st.tolist(), got, True, empty))
    finally:
        dist.destroy_process_group()


def test_gop_sharding_and_gather_gloo_ws2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, t0, st0, l0, ok0, e0), (r1, s1, t1, st1, l1, ok1, e1) = res
    assert sorted(s0 + s1) == list(range(7)) and not set(s0) & set(s1)   # every GOP exactly once
    assert t0 == t1 == 2.0                                               # max over ranks
    assert st0 == st1 == [[0, 4, 0.0], [1, 3, 10.0]]
    assert l0 == [1000, 1037] and ok0 and ok1
    assert l1 is None and e1 is None          # only rank 0 receives the bitstreams
    assert e0 == [b"", b"x"]


def test_single_process_fallbacks():
    assert fd.shard_gops(5, 0, 1) == list(range(5))
    assert fd.max_over_ranks(3.5) == 3.5
    assert fd.gather_bytes(b"abc") == [b"abc"]
    assert fd.gather_stats([1.0, 2.0]).shape == (1, 2)


def test_view_sharding_one_view_per_gpu():
    # BASELINE configs[4]: 8 views on 8 GPUs -> exactly one view per rank, every view once
    shards = [fd.shard_views(8, r, 8) for r in range(8)]
    assert shards == [[r] for r in range(8)]
    shards4 = [fd.shard_views(8, r, 4) for r in range(4)]
    assert sorted(v for s in shards4 for v in s) == list(range(8)) and all(len(s) == 2 for s in shards4)
