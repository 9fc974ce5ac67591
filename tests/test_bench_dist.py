"""CPU: bench.py's per-rank driver (warm-up, barrier-bracketed timed region, max over ranks,
per-rank stats, bitstreams gathered to rank 0, the JSON result) end to end under gloo with
world_size 2 and a CPU stand-in codec. Only RCCL and the HIP codec itself are left to the GPU
box."""
import json
import os
import socket
import time

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from fastvideocodec_amd import dist as fd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class StandInJob:
    """Stands in for bench.GpuGopJob: the same interface, host-side work only."""

    def __init__(self, rank, world, gops_per_gpu):
        self.mine = fd.shard_gops(world * gops_per_gpu, rank, world)
        self.units = len(self.mine)
        self.Hp, self.Wp = 64, 128
        self.rank = rank
        self.steps_done = 0

    def step(self):
        time.sleep(0.01 * (1 + self.rank))  # rank 1 is slower: the max over ranks must see it
        self.steps_done += 1

    def sync(self):
        pass

    def after_timing(self):
        return None

    def verify(self):
        payload = b"".join(bytes([g]) * (100 + g) for g in self.mine)
        return {"bitexact": True, "nbytes": len(payload), "psnr": 30.0 + self.rank, "payload": payload,
                "overflow_recomputes": 0}


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        args = bench.parse_args(["--steps", "3", "--warmup", "1", "--gops-per-gpu", "2", "--height", "64",
                                 "--width", "128", "--gop", "5"])
        job = StandInJob(rank, world, args.gops_per_gpu)
        res = bench.run_rank(job, args, rank, world, None)
        q.put((rank, json.dumps(res) if res is not None else None, job.steps_done))
    finally:
        dist.destroy_process_group()


def test_bench_run_rank_gloo_ws2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, line0, n0), (r1, line1, n1) = out
    assert line1 is None and n0 == n1 == 4           # only rank 0 reports; warm-up + 3 timed steps each
    res = json.loads(line0)
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["scaling"] == "weak"
    # 4 GOPs over both ranks x (gop - 1) P-frames per step, over the slower rank's time
    assert res["config"]["parallelism"] == "gop-shard x2"
    dt = 3 * 4 * 4 / res["value"]
    assert dt >= 3 * 0.02 * 0.9                      # rank 1's 20 ms steps bound the time
    assert abs(res["ms_per_step"] - dt / 3 * 1e3) < 0.05 * res["ms_per_step"] + 0.02
    q_ = res["quality"]
    assert q_["decoder_bitexact"] is True
    assert q_["bitstreams_gathered_to_rank0_bytes"] == sum(100 + g for g in range(4))
    assert q_["psnr_db_mean"] == 30.5
    assert res["metric"].startswith("128x64 ")       # non-1080p runs say so in the metric
