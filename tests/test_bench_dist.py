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


def _run_bench_cli(argv, tmp_path):
    import bench
    out = tmp_path / "line.json"
    rc = bench.main(argv + ["--dry-run", "--json-out", str(out)])
    assert rc == 0
    return json.loads(out.read_text())


def test_bench_gpus2_spawns_two_ranks(tmp_path):
    """`bench.py --gpus 2` with no launcher starts two rank processes itself (gloo host rehearsal
    job): the result line is labelled n_gpus 2 and covers both ranks' GOPs."""
    res = _run_bench_cli(["--gpus", "2", "--steps", "2", "--warmup", "1", "--gops-per-gpu", "3",
                          "--height", "64", "--width", "128", "--gop", "4"], tmp_path)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "gop-shard x2"
    assert res["shards"] == {"unit": "gop", "by_rank": [[0, 2, 4], [1, 3, 5]]}
    assert res["config"]["gops_per_gpu"] == 3
    assert res["quality"]["bitstreams_gathered_to_rank0_bytes"] == sum(100 + g for g in range(6))
    dt = 2 * 6 * 3 / res["value"]                   # 6 GOPs x 3 P-frames per step
    assert dt >= 2 * 0.010 * 0.9                    # rank 1's 10 ms steps bound the time
    # a multi-GPU line carries its own CPU baseline (rank 0, after timing) and every
    # rank's parity block, gathered to rank 0
    cb = res["cpu_baseline"]
    assert cb["n_gpus_in_run"] == 2 and cb["value"] > 0 and cb["cores"] >= 1
    pr = res["quality"]["parity_by_rank"]
    assert [p["rank"] for p in pr] == [0, 1] and [p["unit"] for p in pr] == [0, 1]
    assert all(p["bitstream_t1_byte_exact"] and p["symbols"] == 28800 for p in pr)
    assert res["quality"]["parity_all_ranks"]["ranks_checked"] == 2
    assert res["quality"]["parity"]["frame"].startswith("unit 0 ")


def test_bench_gpus4_gop32_one_gop_per_rank(tmp_path):
    """BASELINE configs[3]'s layout (`--gpus 4 --gop 32 --gops-per-gpu 1`): GOP r on rank r, 31
    P-frames per GOP counted over all four ranks."""
    res = _run_bench_cli(["--gpus", "4", "--gop", "32", "--gops-per-gpu", "1", "--steps", "1", "--warmup", "0",
                          "--height", "64", "--width", "128"], tmp_path)
    assert res["n_gpus"] == 4 and res["config"]["parallelism"] == "gop-shard x4"
    assert res["shards"] == {"unit": "gop", "by_rank": [[0], [1], [2], [3]]}
    assert res["quality"]["bitstreams_gathered_to_rank0_bytes"] == sum(100 + g for g in range(4))
    assert abs(res["value"] * res["ms_per_step"] / 1e3 - 4 * 31) < 1e-3 * 4 * 31  # (rounded fields)


def test_bench_views8_gpus8_view_v_on_rank_v(tmp_path):
    """BASELINE configs[4]: `--views 8 --gpus 8` puts view v on rank v."""
    res = _run_bench_cli(["--gpus", "8", "--views", "8", "--steps", "1", "--warmup", "0",
                          "--height", "64", "--width", "128", "--gop", "3"], tmp_path)
    assert res["n_gpus"] == 8 and res["config"]["parallelism"] == "view-shard x8"
    assert res["shards"] == {"unit": "view", "by_rank": [[v] for v in range(8)]}
    assert res["config"]["views_per_gpu"] == 1
    # at N = 8 only ranks 0..3 (--parity-ranks default) run the oracle parity check
    pa = res["quality"]["parity_all_ranks"]
    assert pa["ranks_checked"] == 4 and pa["parity_ranks_cap"] == 4 and "ranks 0..3" in pa["note"]
    assert pa["ok"] is True
    pr = res["quality"]["parity_by_rank"]
    assert [p.get("checked", True) for p in pr] == [True] * 4 + [False] * 4


def test_bench_parity_ranks_flag_and_strict(tmp_path):
    """--parity-ranks 1 at N = 2 checks rank 0 only; --strict-parity exits 0 when parity holds."""
    res = _run_bench_cli(["--gpus", "2", "--steps", "1", "--warmup", "0", "--gops-per-gpu", "1", "--height", "64",
                          "--width", "128", "--gop", "3", "--parity-ranks", "1", "--strict-parity"], tmp_path)
    pa = res["quality"]["parity_all_ranks"]
    assert pa["ranks_checked"] == 1 and pa["ok"] is True


def test_bench_refuses_gpus_mismatch_under_launcher(monkeypatch):
    """Under torchrun (WORLD_SIZE set) a --gpus that disagrees is refused rather than mislabelled."""
    import pytest
    import bench
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    with pytest.raises(SystemExit, match="--gpus 2 != WORLD_SIZE 1"):
        bench.main(["--gpus", "2", "--dry-run"])


def test_bench_no_cpu_baseline_omits_parity(tmp_path):
    """--cpu-baseline none: no CPU leg and no parity at any N."""
    res = _run_bench_cli(["--gpus", "2", "--steps", "1", "--warmup", "0", "--gops-per-gpu", "1", "--height", "64",
                          "--width", "128", "--gop", "3", "--cpu-baseline", "none"], tmp_path)
    assert "cpu_baseline" not in res and "parity_by_rank" not in res["quality"]


def test_bench_tree_labels_extension(tmp_path):
    """a tree run past the reference's 30-frame graphs says so in its config block."""
    res = _run_bench_cli(["--tree", "--gop", "32", "--gops-per-gpu", "1", "--steps", "1", "--warmup", "0",
                          "--height", "64", "--width", "128", "--cpu-baseline", "none"], tmp_path)
    tr = res["config"]["tree"]
    assert tr["structure"].startswith("EXTENSION") and sum(len(l) for l in tr["layers"]) == 31
    res = _run_bench_cli(["--tree", "--gop", "12", "--gops-per-gpu", "1", "--steps", "1", "--warmup", "0",
                          "--height", "64", "--width", "128", "--cpu-baseline", "none"], tmp_path)
    assert res["config"]["tree"]["layers"] == [[1, 8], [2, 5, 9], [3, 4, 6, 7, 10, 11]]


def test_gops_per_gpu_defaults():
    """16 GOPs per step for the sequential GOP; 4 for --tree (its layers batch up to 6 frames per
    GOP); an explicit value wins either way."""
    import bench
    assert bench.parse_args([]).gops_per_gpu == 16
    assert bench.parse_args(["--tree"]).gops_per_gpu == 4
    assert bench.parse_args(["--tree", "--gops-per-gpu", "8"]).gops_per_gpu == 8
