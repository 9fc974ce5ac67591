"""1080p DVC P-frame encode+decode throughput on MI355X (BASELINE.json metric, configs[2]).

A step = G GOP-12s per GPU batched along dim 0 (G = --gops-per-gpu, default 4; default 2 timed
steps = 8 GOPs per run), one GOP per batch slot, at 1920x1080 (replicate-padded to 1920x1088): frame 0 is
the I-frame (passed through; BPG is out of scope), frames 1..11 are DVC P-frames, each
encoded (full forward incl. reconstruction + bpp path + rANS range coding into a bitstream)
and decoded (rANS decode -> hyperprior -> MV synthesis -> motion compensation -> residual
synthesis) against the previous decoded frame. value = decoded P-frames per second over all
ranks (I-frames are not counted). Inputs are resident in HBM before the timed region.

Consecutive steps are pipelined the way a streaming encoder runs: a GOP's coder/decoder tail
(the last frames' latency-bound rANS decode + reconstruction) overlaps the next GOP's encoder
(encode_decode_gop(join=False)); the timer stops after a device-wide synchronize, so all work of
all K GOPs is inside the timed region.

Multi-GPU: one process per GPU (torchrun), GOPs sharded by rank, no data-path collective;
RCCL is used only after timing (max-time all_reduce, metric/bitstream-size all_gather).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from fastvideocodec_amd import dist as fdist  # noqa: E402
from fastvideocodec_amd import profiling  # noqa: E402
from fastvideocodec_amd.gop import encode_decode_gop  # noqa: E402
from fastvideocodec_amd.models import get_codec_model  # noqa: E402
from fastvideocodec_amd.synthetic import gop_seed, make_gop  # noqa: E402

HBM_PEAK_BPS = 8.0e12           # MI355X_MICROARCH.md: HBM3E peak (spec; ~6.3 TB/s achievable)
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 dense matrix peak (~2.5 PF)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), dense
ENC_TFLOP_PER_PFRAME = 2.931   # SURVEY.md §8(d) algorithmic, 1920x1088
DEC_TFLOP_PER_PFRAME = 1.295


def cpu_baseline(H, W, frames_np):
    """Oracle (CPU PyTorch restatement of the reference forward, validated against the reference's
    golden fixtures) + C oracle coder, one 1080p P-frame encode+decode on the host cores."""
    from oracle import coder_ref as R
    from oracle import dvc_ref
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    from fastvideocodec_amd import entropy_models as EM

    cores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    sd = seeded_torch_state_dict()
    cur = torch.from_numpy(frames_np[1:2].copy())
    ref = torch.from_numpy(frames_np[0:1].copy())
    lt = EM.LaplaceTables()
    t0 = time.perf_counter()
    (clipped, *_), inter = dvc_ref.forward(sd, cur, ref, return_intermediates=True)
    sig = inter["recon_sigma"].numpy()
    feat = inter["compressed_feature"].numpy().astype(np.int32)
    idx = R.build_indexes(sig, lt.scale_table)
    nbytes = 0
    for c in range(feat.shape[1]):
        nbytes += len(R.CRef.encode(feat[0, c].ravel(), idx[0, c].ravel(), lt.cdf, lt.cdf_length, lt.offset))
    dvc_ref.decode(sd, ref, inter["quant_mv"], inter["compressed_z"], inter["compressed_feature"])
    dt = time.perf_counter() - t0
    # also one thread on config 1's 256x256 pair (oracle forward only)
    from fastvideocodec_amd.synthetic import make_gop
    small = make_gop(256, 256, 2, 20261015)
    torch.set_num_threads(1)
    c1, r1 = torch.from_numpy(small[1:2].copy()), torch.from_numpy(small[0:1].copy())
    dvc_ref.forward(sd, c1, r1)  # warm
    t1 = time.perf_counter()
    dvc_ref.forward(sd, c1, r1)
    dt1 = time.perf_counter() - t1
    torch.set_num_threads(cores)
    cpu_model = ""
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": round(1.0 / dt, 4), "unit": "P-frames/s", "cores": cores, "kind": "port",
            "cpu": cpu_model, "one_thread_256x256_forward_s": round(dt1, 3),
            "sample": f"1 P-frame {W}x{H}: oracle forward (encode+recon) + oracle decode + C rANS of the "
                      f"feature latent, torch CPU fp32, {dt:.1f} s",
            "seconds": round(dt, 2)}


def load_pmc_traffic(H, W):
    """HBM bytes per conv_x3_kernel launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes
    over `bench.py --serial` (profiles/r1/x3_traffic.json, written by scripts/rocprof_summary.py;
    FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction). PMC passes serialise every
    dispatch and cannot run inside the timed region, so the figure is the profiled one."""
    path = os.path.join(REPO, "profiles", "r1", "x3_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    if d.get("height") != H or d.get("width") != W:
        return {}
    return {"hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"),
            "source": f"profiles/r1/x3_traffic.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                      f"{d.get('launches')} launches)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--gop", type=int, default=12)
    ap.add_argument("--gops-per-gpu", type=int, default=4,
                    help="GOPs batched per rank per step (SURVEY §8(e)); default 4 x 2 steps = 8 GOPs per run "
                         "(§8(d)). Measured on MI355X: 1 -> 44.5, 2 -> 47.6, 4 -> 49.1 P-frames/s")
    ap.add_argument("--views", type=int, default=0,
                    help="BASELINE configs[4]: V camera views, one GOP stream each, view v -> rank v %% world "
                         "(replaces --gops-per-gpu; the reference's MCVC couples views, DVC views are independent)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--breakdown", action="store_true", help="print per-conv-geometry timing to stderr")
    ap.add_argument("--serial", action="store_true",
                    help="one HIP stream (no encode/code/decode overlap): per-kernel durations are unshared")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    model = get_codec_model("DVC-pretrained", compression_level=2, device=dev)
    model.update()
    if args.views > 0:
        # configs[4]: one GOP stream per camera view, view v -> rank v % world
        if args.views < world:
            raise SystemExit(f"--views {args.views} < world size {world}: a rank would have no view")
        my_views = fdist.shard_views(args.views, rank, world)
        gops = [make_gop(args.height, args.width, args.gop, gop_seed(0, v)) for v in my_views]
        n_units = args.views
    else:
        my_gops = fdist.shard_gops(world * args.gops_per_gpu, rank, world)  # GOP g -> rank g % world
        gops = [make_gop(args.height, args.width, args.gop, gop_seed(g)) for g in my_gops]
        n_units = world * args.gops_per_gpu
    G = len(gops)
    frames = torch.from_numpy(np.stack(gops)).to(dev)  # [G, T, 3, Hp, Wp]
    Hp, Wp = frames.shape[-2:]

    overlap = not args.serial
    for _ in range(args.warmup):
        encode_decode_gop(model, frames, overlap=overlap, join=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        encode_decode_gop(model, frames, overlap=overlap, join=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0

    # ---- roofline pass: one serial GOP (single stream) with HIP events around every conv launch
    # on the launching stream; in the overlapped timed region concurrent kernels would be charged
    # to each other's event windows.
    timer = profiling.KernelTimer()
    with timer:
        encode_decode_gop(model, frames, overlap=False)
    conv_ms, conv_flops, n_launch = timer.collect()
    x3_ms, x3_flops, x3_launch = timer.collect(x3=True)
    x3_bytes = timer.collect_bytes(x3=True)
    hbm = timer.collect_hbm()
    if args.breakdown and rank == 0:
        agg = timer.breakdown()
        for k, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{k:40s} n={n:5d} ms={ms:9.2f} TF/s={fl / (ms * 1e-3) / 1e12:7.2f}", file=sys.stderr)

    # ---- verification + quality, outside the timed region
    from fastvideocodec_amd import kernels as K
    K.x3_overflow(reset=True)
    bss, decoded, sses, encs = encode_decode_gop(model, frames, check=True, overlap=overlap)
    torch.cuda.synchronize()
    x3_overflow = K.x3_overflow(reset=True)
    bitexact = all(torch.equal(a, b) for a, b in zip(decoded, encs))
    nbytes = sum(b.nbytes() for b in bss)
    npx = G * 3 * Hp * Wp
    psnrs = [float(10 * np.log10(1.0 / (float(s[0]) / npx))) for s in sses]

    # one collective round after timing (RCCL over xGMI on the GPU box): max time, per-rank
    # stats, and every rank's bitstream bytes of the verification pass gathered (all ranks)
    dt_max = fdist.max_over_ranks(dt, dev)
    allst = fdist.gather_stats([1.0 if bitexact else 0.0, float(nbytes), float(np.mean(psnrs))], dev)
    payload = b"".join(s for bs in bss for s in bs.mv.to_bytes_list() + bs.z.to_bytes_list()
                       + bs.feature.to_bytes_list())
    gathered = fdist.gather_bytes(payload, dev)
    bitexact_all = bool(np.all(allst[:, 0] == 1.0)) and sum(len(g) for g in gathered) == int(allst[:, 1].sum())
    bytes_all = float(allst[:, 1].sum())
    psnr_all = float(np.mean(allst[:, 2]))

    pmc_traffic = load_pmc_traffic(args.height, args.width)
    pframes = args.steps * n_units * (args.gop - 1)
    value = pframes / dt_max
    nfr = G * (args.gop - 1)
    achieved = x3_flops / (x3_ms * 1e-3) / 1e12 if x3_ms > 0 else 0.0
    result = {
        "metric": "1080p frames/sec encode+decode at λ=1024; bpp/PSNR parity vs CPU ref",
        "value": round(value, 3),
        "unit": "P-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (convs: fp32 operands split into fp16 hi/lo, f32 accumulate)",
        "data": "synthetic (seeded GOP generator, SURVEY.md §8(d)); seeded weights + pretrained SpyNet",
        "config": {"workload": f"DVC P-frame encode+decode with rANS, {args.width}x{args.height} "
                               f"(padded {Wp}x{Hp}) GOP-{args.gop}, lambda=1024 slot",
                   "gops_per_gpu": G, "frames_counted": "P-frames only (I-frame pass-through)",
                   "parallelism": f"gop-shard x{world}"} if args.views <= 0 else
                  {"workload": f"{args.views}-view DVC P-frame encode+decode with rANS, {args.width}x{args.height} "
                               f"(padded {Wp}x{Hp}) GOP-{args.gop} per view, lambda=1024 slot",
                   "views": args.views, "views_per_gpu": G,
                   "frames_counted": "P-frames only (I-frame pass-through)",
                   "parallelism": f"view-shard x{world}"},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": F16_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / F16_MFMA_PEAK_TFLOPS, 4),
                     "traffic": pmc_traffic.get("hbm_bytes_per_launch"),
                     "traffic_source": pmc_traffic.get("source"),
                     "avg_launch_us": round(x3_ms * 1e3 / x3_launch, 2) if x3_launch else None,
                     "algorithmic_bytes_per_launch": round(x3_bytes / x3_launch) if x3_launch else None,
                     "algorithmic_gbps": round(x3_bytes / (x3_ms * 1e-3) / 1e9, 1) if x3_ms else None,
                     "kernel": "conv_x3_kernel (split-precision fp16x3 implicit-GEMM conv/deconv): all its launches",
                     "achieved_is": "algorithmic fp32-conv FLOP (2 x MAC) / kernel time; the kernel issues 3 f16 "
                                    "MFMAs per MAC, so its ceiling in these units is peak/3",
                     "x3_ceiling": round(F16_MFMA_PEAK_TFLOPS / 3, 1),
                     "frac_of_x3_ceiling": round(achieved / (F16_MFMA_PEAK_TFLOPS / 3), 4),
                     "measured": "HIP events on the launching stream around every conv launch of one serial GOP",
                     "launches": x3_launch, "ms_per_pframe": round(x3_ms / nfr, 3),
                     "gflop_per_pframe": round(x3_flops / nfr / 1e9, 1),
                     "all_convs": {"ms_per_pframe": round(conv_ms / nfr, 3),
                                   "gflop_per_pframe": round(conv_flops / nfr / 1e9, 1),
                                   "tflops": round(conv_flops / (conv_ms * 1e-3) / 1e12, 2) if conv_ms else 0.0,
                                   "launches": n_launch}},
        "hbm_kernels": {k: {"gb_per_s": round(b / (ms * 1e-3) / 1e9, 1) if ms else None,
                            "frac_of_8tbps": round(b / (ms * 1e-3) / HBM_PEAK_BPS, 4) if ms else None,
                            "ms_per_pframe": round(ms / nfr, 3), "gb_per_pframe": round(b / nfr / 1e9, 3),
                            "launches": n}
                        for k, (n, ms, b) in sorted(hbm.items(), key=lambda kv: -kv[1][1])},
        "quality": {"decoder_bitexact": bitexact_all, "bytes_per_pframe": round(bytes_all / (n_units * (args.gop - 1)), 1),
                    "bpp_actual": round(bytes_all * 8 / (n_units * (args.gop - 1) * Hp * Wp), 5),
                    "psnr_db_mean": round(psnr_all, 4),
                    "x3_operand_overflow": x3_overflow,
                    "note": "seeded (untrained) codec weights + synthetic GOP: PSNR/bpp are not rate-distortion "
                            "figures; they are the same arithmetic as the oracle (parity in tests/)"},
        "model_tflop_per_pframe": ENC_TFLOP_PER_PFRAME + DEC_TFLOP_PER_PFRAME,
    }
    result["effective_tflops"] = round(value / world * (ENC_TFLOP_PER_PFRAME + DEC_TFLOP_PER_PFRAME), 2)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(Hp, Wp, gops[0])
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
