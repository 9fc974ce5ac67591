"""1080p DVC P-frame encode+decode throughput on MI355X (BASELINE.json metric, configs[2]).

A step = G GOP-12s per GPU batched along dim 0 (G = --gops-per-gpu, default 16; default 2 timed
steps = 32 GOPs per run), one GOP per batch slot, at 1920x1080
(replicate-padded to 1920x1088): frame 0 is the I-frame (passed through; BPG is out of scope),
frames 1..11 are DVC P-frames, each encoded (full encoder forward incl. its reconstruction, then
rANS range coding of mv / z / feature into a bitstream) and decoded (rANS decode -> hyperprior ->
MV synthesis -> motion compensation -> residual synthesis) against the previous decoded frame.
The bits-estimate kernels of forward() are not in the step: the real bitstream replaces the
estimate. value = decoded P-frames per second over all ranks (I-frames are not counted). Inputs
are resident in HBM before the timed region.

Consecutive steps are pipelined the way a streaming encoder runs: a GOP's coder/decoder tail
(the last frames' latency-bound rANS decode + reconstruction) overlaps the next GOP's encoder
(encode_decode_gop(join=False)); the timer stops after a device-wide synchronize, so all work of
all K GOPs is inside the timed region.

Multi-GPU: one process per GPU, either under a launcher (torchrun sets WORLD_SIZE) or spawned
by `bench.py --gpus N` itself (spawn_ranks: N fresh rank processes, rendezvous on 127.0.0.1);
GOPs sharded by rank, no data-path collective; RCCL is used only after timing (max-time
all_reduce, per-rank stats all_gather, bitstreams gathered to rank 0).

After timing, every rank checks its own first GOP's frame 1 against the oracle (BASELINE.md §3's
parity block: symbol / index mismatch counts, dPSNR, dbpp_est and a byte-exact stream check
against the C oracle coder), gathered to rank 0 as `quality.parity_by_rank`; rank 0 then times
the oracle on the host cores (--cpu-baseline quick|full|none) at every N, so every line, single-
or multi-GPU, carries its own CPU baseline and parity.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from fastvideocodec_amd import dist as fdist  # noqa: E402

HBM_PEAK_BPS = 8.0e12           # MI355X_MICROARCH.md: HBM3E peak (spec; ~6.3 TB/s achievable)
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 dense matrix peak (~2.5 PF)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), dense
# SURVEY.md §8(d) algorithmic work at 1920x1088; every layer scales with the frame area
ENC_TFLOP_1088 = 2.931
DEC_TFLOP_1088 = 1.295
AREA_1088 = 1920 * 1088
METRIC_1080 = "1080p frames/sec encode+decode at λ=1024; bpp/PSNR parity vs CPU ref"
ONE_THREAD_1080_BUDGET_S = 240.0  # cap on the CPU leg's 1-thread 1080p run
# T3 parity bounds: the reference's own cross-backend symbol flip rate at 1080p, and
# the north star's PSNR tolerance
SYMBOL_FLIP_BOUND = 1.56e-5
DPSNR_BOUND_DB = 1e-4


def parity_rank_cap(args, world):
    """How many ranks run the per-rank oracle parity check (ranks 0..cap-1). Each check is a 1080p
    oracle forward on the host cores the checking ranks share, so at N = 8 an uncapped run would be
    8 concurrent forwards on 1/8 of the cores each; --parity-ranks bounds that."""
    return max(1, min(world, getattr(args, "parity_ranks", 4)))


def tflop_per_pframe(hp, wp):
    s = hp * wp / AREA_1088
    return ENC_TFLOP_1088 * s, DEC_TFLOP_1088 * s


def metric_name(height, width):
    if (height, width) == (1080, 1920):
        return METRIC_1080
    return f"{width}x{height} frames/sec encode+decode at λ=1024; bpp/PSNR parity vs CPU ref"


# ------------------------------------------------------------------ CPU leg (rank 0, N=1)
def cpu_cores():
    """Host cores this process may use: the affinity mask, capped by the cgroup CPU quota (a GPU
    box shows the whole machine's CPUs in the mask but grants a share of them)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


class _Heartbeat:
    """A progress line on stderr every `every` seconds while a long host-side stage runs (the CPU
    leg's 1080p runs print nothing for minutes otherwise)."""

    def __init__(self, every=30.0):
        import threading
        self.stage, self.every, self.t0 = "start", every, time.perf_counter()
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.wait(self.every):
            print(f"[bench] cpu baseline: {self.stage} ({time.perf_counter() - self.t0:.0f} s)", file=sys.stderr,
                  flush=True)

    def __enter__(self):
        self._th.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._th.join()


def _median_time(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), ts


def cpu_baseline(frames_np, mode="quick", coder=None):
    """The oracle (CPU PyTorch restatement of the reference forward, pinned to the reference's
    golden fixtures) on the host cores, on GOP 0's frame 1 coded against frame 0 (the frame the GPU
    run also codes first, and rank 0's parity frame). `coder`: the C oracle coder's symbols/s from
    the parity block (one core).

    full (default; ~3 min of CPU work): 256x256 forward median of 3 after a warm-up at
    all cores and at 1 thread; 1080p encode+decode median of 3 after a warm-up at all cores, and once
    at 1 thread (skipped, and said so in seconds_1080_1thread_note, if predicted over
    ONE_THREAD_1080_BUDGET_S). quick (~30 s): 1080p once at all cores instead of the 1080p protocol."""
    from oracle import dvc_ref
    from fastvideocodec_amd.synthetic import make_gop
    from fastvideocodec_amd.weights import seeded_torch_state_dict

    cores = cpu_cores()
    torch.set_num_threads(cores)
    sd = seeded_torch_state_dict()
    cur = torch.from_numpy(frames_np[1:2].copy())
    ref = torch.from_numpy(frames_np[0:1].copy())
    Hp, Wp = cur.shape[-2:]

    def enc_dec():
        out, inter = dvc_ref.forward(sd, cur, ref, return_intermediates=True)
        dvc_ref.decode(sd, ref, inter["quant_mv"], inter["compressed_z"], inter["compressed_feature"])

    hb = _Heartbeat()
    with hb:
        hb.stage = "256x256"
        small = make_gop(256, 256, 2, 20261015)
        c1, r1 = torch.from_numpy(small[1:2].copy()), torch.from_numpy(small[0:1].copy())
        f256 = lambda: dvc_ref.forward(sd, c1, r1)
        f256()
        t_256 = _median_time(f256, 3)[0]
        torch.set_num_threads(1)
        f256()
        t_256_1 = _median_time(f256, 3)[0]
        torch.set_num_threads(cores)

        full = mode == "full"
        hb.stage = f"1080p on {cores} threads"
        if full:
            enc_dec()  # warm-up
        t_1080, runs_1080 = _median_time(enc_dec, 3 if full else 1)
        one_thread_1080 = None
        one_thread_note = None
        if full:
            # the 1-thread 1080p run is bounded so the default bench stays within a few minutes: its
            # length is predicted from the all-core 1080p median and the 256x256 thread-scaling ratio
            est = t_1080 * t_256_1 / max(t_256, 1e-9)
            if est <= ONE_THREAD_1080_BUDGET_S:
                hb.stage = f"1080p on 1 thread (predicted {est:.0f} s)"
                torch.set_num_threads(1)
                one_thread_1080 = _median_time(enc_dec, 1)[0]
                torch.set_num_threads(cores)
            else:
                one_thread_note = f"skipped: predicted {est:.0f} s > {ONE_THREAD_1080_BUDGET_S:.0f} s budget"
    cpu_model = ""
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    res = {"value": round(1.0 / t_1080, 4), "unit": "P-frames/s", "cores": cores, "kind": "port",
           "cpu": cpu_model, "mode": mode,
           "sample": f"1 P-frame {Wp}x{Hp} (GOP 0 frame 1): oracle forward (encode + reconstruction) + oracle "
                     f"decode, torch CPU fp32 on {cores} threads, {'median of 3 after a warm-up' if full else 'one run'}"
                     f" = {t_1080:.2f} s",
           "seconds_1080": round(t_1080, 3), "runs_1080": [round(x, 3) for x in runs_1080],
           "forward_256x256_s": {"threads": cores, "median_of_3": round(t_256, 4)},
           "forward_256x256_1thread_s": round(t_256_1, 4),
           "coder_1core": coder}
    res["seconds_1080_1thread"] = round(one_thread_1080, 2) if one_thread_1080 is not None else None
    if one_thread_note:
        res["seconds_1080_1thread_note"] = one_thread_note
    return res


def dry_cpu_baseline():
    """--dry-run stand-in for the CPU leg (no GPU anywhere): the oracle forward on one 64x64 frame
    pair on the host cores, so the multi-rank result line carries the field it would carry."""
    from oracle import dvc_ref
    from fastvideocodec_amd.synthetic import make_gop
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    cores = cpu_cores()
    torch.set_num_threads(cores)
    sd = seeded_torch_state_dict()
    g = make_gop(64, 64, 2, 7)
    c1, r1 = torch.from_numpy(g[1:2].copy()), torch.from_numpy(g[0:1].copy())
    t = _median_time(lambda: dvc_ref.forward(sd, c1, r1), 1)[0]
    return {"value": round(1.0 / t, 4), "unit": "P-frames/s", "cores": cores, "kind": "port", "mode": "dry-run",
            "sample": f"dry run: 1 P-frame 64x64 oracle forward on {cores} threads = {t:.3f} s"}


def rank_parity(model, dev, frames_np, unit, threads):
    """BASELINE.md §3's parity block of this rank's first GOP (or view) `unit`: its frame 1 coded
    against frame 0 by the oracle on `threads` host threads and by the GPU path (not timed)."""
    from oracle import coder_ref as R
    from oracle import dvc_ref
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    old = torch.get_num_threads()
    torch.set_num_threads(max(1, threads))
    try:
        cur = torch.from_numpy(frames_np[1:2].copy())
        ref = torch.from_numpy(frames_np[0:1].copy())
        out, inter = dvc_ref.forward(seeded_torch_state_dict(), cur, ref, return_intermediates=True)
        par, coder = parity_block(model, dev, cur, ref, out, inter, R)
    finally:
        torch.set_num_threads(old)
    par["frame"] = f"unit {unit} frame 1 vs frame 0"
    return par, coder


# ------------------------------------------------------------------ reference-comparable figures
def reference_metrics(model, frames, reps=5):
    """The figures the reference publishes for this path, measured here at
    batch 1 on one GOP of this run's workload (frames: [T, 3, H, W] device tensor), after the timed
    region. Secondary fields beside the headline:
    * stage split (plot_hermes.py:547-554: SpyNet ME / MC / MV codec / residual codec): HIP
      events on the launching stream around each stage of one encoder forward, median of `reps`;
    * per-frame decode time (plot_hermes.py:735-737, simulation.py:133-137): the P-frames of the
      GOP range-coded first, then each decoded (rANS decode -> hyperprior -> MV synthesis -> MC ->
      residual synthesis) against the previous decoded frame with a host sync per frame;
    * the drop-in path: models.parallel_compression (the reference's eval loop, models.py:368-383:
      forward + bits estimate per P-frame at batch 1, the result of each frame feeding the next),
      end to end including its host waits (the per-frame overflow probe, net.py:_run_checked)."""
    from fastvideocodec_amd import kernels as K
    from fastvideocodec_amd.models import parallel_compression

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    T = frames.shape[0]
    cur, ref = frames[1:2].contiguous(), frames[0:1].contiguous()
    names = ("me_spynet", "mv_codec", "mc", "residual_codec", "rans_encode")
    stages = {n: [] for n in names}
    with torch.no_grad():
        for _ in range(reps + 1):
            e = [ev() for _ in range(len(names) + 1)]
            e[0].record()
            cur4 = K.nchw_to_nhwc(cur.float(), 4)
            ref4 = K.nchw_to_nhwc(ref.float(), 4)
            estmv = model.opticFlow.run(cur4, ref4)
            e[1].record()
            mvfeature = model.mvEncoder.run(estmv)
            mv_up = model.mvDecoder.run(mvfeature)
            e[2].record()
            prediction, _ = model.motioncompensation(ref4, mv_up)
            e[3].record()
            feature = model.resEncoder.run(K.sub(cur4, prediction))
            z = model.respriorEncoder.run(feature)
            sigma = model.respriorDecoder.run(z)
            model.resDecoder.run(feature, prediction)
            e[4].record()
            model.compress_tensors({"mvfeature": mvfeature, "z": z, "feature": feature, "sigma": sigma})
            e[5].record()
            torch.cuda.synchronize()
            for i, n in enumerate(names):
                stages[n].append(e[i].elapsed_time(e[i + 1]))
    split = {n: round(statistics.median(v[1:]), 3) for n, v in stages.items()}

    # per-frame decode at batch 1: encode the GOP's P-frames first (the encoder's own chain)
    bss, x = [], frames[0:1]
    with torch.no_grad():
        for t in range(1, T):
            bs, x = model.compress(frames[t:t + 1], x)
            bss.append(bs)
        torch.cuda.synchronize()
        dec_ms, x = [], frames[0:1]
        for _ in range(2):  # a warm pass, then the timed one
            dec_ms, x = [], frames[0:1]
            for bs in bss:
                t0 = time.perf_counter()
                x = model.decompress(bs, x)
                torch.cuda.synchronize()
                dec_ms.append((time.perf_counter() - t0) * 1e3)
        enc_ms, x = [], frames[0:1]
        for t in range(1, T):
            t0 = time.perf_counter()
            _, x = model.compress(frames[t:t + 1], x)
            torch.cuda.synchronize()
            enc_ms.append((time.perf_counter() - t0) * 1e3)

    # the drop-in eval path (reference semantics: bits estimated, not coded)
    data = frames.clone()
    parallel_compression(None, model, data.clone(), False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    parallel_compression(None, model, data, False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    H, W = frames.shape[-2:]
    return {
        "resolution": f"{W}x{H}", "batch": 1,
        "stage_ms_b1": split,
        "stage_note": "one encoder forward at batch 1 on one stream, HIP events between stages (median of "
                      f"{reps}); reference (BASELINE.md §1, plot_hermes.py:547-554, trained weights, NVIDIA, "
                      "resolution not recorded): ME / MC / MV codec / residual codec = 14.3 / 6.6 / 9.8 / 2.4 ms "
                      "(GTX 1080 Ti), 9.2 / 4.0 / 3.7 / 1.6 ms (RTX 2080 Ti); their MV / residual codec "
                      "excludes range coding (estimated bits), reported here separately as rans_encode",
        "decode_ms_per_frame_b1": {"median": round(statistics.median(dec_ms), 3), "min": round(min(dec_ms), 3),
                                   "frames": len(dec_ms)},
        "decode_fps_b1": round(1e3 / statistics.median(dec_ms), 2),
        "decode_note": "bitstream -> rANS decode -> hyperprior -> MV synthesis -> MC -> residual synthesis per "
                       "P-frame, host sync per frame; reference per-frame decode time 38.2 / 28.0 / 10.0 ms on "
                       "GTX 1080 Ti / RTX 2080 Ti / RTX 3090 Ti (plot_hermes.py:735-737, simulation.py:133-137)",
        "encode_ms_per_frame_b1": {"median": round(statistics.median(enc_ms), 3), "frames": len(enc_ms)},
        "dropin_parallel_compression": {"pframes_per_s": round((T - 1) / dt, 2), "seconds": round(dt, 4),
                                        "pframes": T - 1,
                                        "note": "models.parallel_compression on one GOP at batch 1 (forward + "
                                                "bits estimate, each frame's recon feeding the next), including "
                                                "the per-frame host wait of the overflow probe (net.py:_run_checked)"},
    }


# per-rank parity summary gathered to rank 0 (fixed order of floats)
PARITY_FIELDS = ("checked", "symbols", "symbol_mismatches", "index_mismatches", "dpsnr_db", "dbpp_est_rel",
                 "streams", "streams_t1_equal", "streams_equal_on_oracle_symbols")


def parity_vector(par):
    if par is None:
        return [0.0] * len(PARITY_FIELDS)
    lat = par["latents"].values()
    return [1.0, float(sum(v["symbols"] for v in lat)), float(sum(v["symbol_mismatches"] for v in lat)),
            float(sum(v["index_mismatches"] for v in lat)), float(par["dpsnr_db"]), float(par["dbpp_est_rel"]),
            float(sum(v["streams"] for v in lat)),
            float(sum(v["streams_bytes_equal_c_oracle_same_symbols"] for v in lat)),
            float(sum(v["streams_bytes_equal_c_oracle_on_oracle_symbols"] for v in lat))]


def parity_block(model, dev, cur, ref, oracle_out, inter, R):
    """BASELINE.md §3 parity of the GPU path against the oracle on one frame: symbol and index
    mismatch counts per latent, dPSNR, dbpp_est, and every device stream vs the C oracle coder
    (T1: same symbols / indexes / tables -> same bytes; T3: streams of the oracle's own symbols
    that come out byte-identical). Also times the C coder on one core (symbols/s)."""
    from fastvideocodec_amd import kernels as K

    with torch.no_grad():
        out = model(cur.to(dev), ref.to(dev))
        t = model._encode_graph(cur.to(dev), ref.to(dev))
        bs = model.compress_tensors(t)
    c = model._coders
    tz, tmv, tf = c["tables"]
    tabs = {"mv": tmv, "z": tz, "feature": tf}
    keys = {"mv": ("mvfeature", "quant_mv", 128), "z": ("z", "compressed_z", 64),
            "feature": ("feature", "compressed_feature", 96)}
    st = c["scale_table"].cpu().numpy()
    from fastvideocodec_amd.net import stream_rows
    par = {"frame": "GOP 0 frame 1 vs frame 0", "framing": bs.framing, "latents": {}}
    total_sym = total_flip = 0
    t_enc = t_dec = 0.0
    nsym = 0
    for name, (key, gkey, C) in keys.items():
        gsym = K.latent_to_symbols(t[key], C).cpu().numpy().reshape(C, -1)
        osym = inter[gkey].numpy().reshape(C, -1).astype(np.int32)
        if name == "feature":
            gidx = K.build_indexes(t["sigma"], c["scale_table"], C).cpu().numpy().reshape(C, -1)
            oidx = R.build_indexes(inter["recon_sigma"].numpy().reshape(C, -1), st)
        else:
            gidx = oidx = np.repeat(np.arange(C, dtype=np.int32)[:, None], gsym.shape[1], 1)
        tb = tabs[name]
        strings = getattr(bs, name).to_bytes_list()
        # one row per stream of the bitstream's framing (segments of a channel row are contiguous)
        shape = stream_rows(bs.framing, 1, C, gsym.shape[1])
        gsym, gidx, osym, oidx = (a.reshape(shape) for a in (gsym, gidx, osym, oidx))
        assert len(strings) == shape[0]
        t1_equal = oracle_equal = 0
        for ch in range(shape[0]):
            t0 = time.perf_counter()
            s_gpu_syms = R.CRef.encode(gsym[ch], gidx[ch], tb.cdf, tb.cdf_length, tb.offset)
            t_enc += time.perf_counter() - t0
            t0 = time.perf_counter()
            R.CRef.decode(s_gpu_syms, gidx[ch], tb.cdf, tb.cdf_length, tb.offset)
            t_dec += time.perf_counter() - t0
            nsym += gsym.shape[1]
            t1_equal += strings[ch] == s_gpu_syms
            oracle_equal += strings[ch] == R.CRef.encode(osym[ch], oidx[ch], tb.cdf, tb.cdf_length, tb.offset)
        flips = int((gsym != osym).sum())
        total_flip += flips
        total_sym += gsym.size
        par["latents"][name] = {"symbols": int(gsym.size), "symbol_mismatches": flips,
                                "index_mismatches": int((gidx != oidx).sum()), "streams": shape[0],
                                "streams_bytes_equal_c_oracle_same_symbols": int(t1_equal),
                                "streams_bytes_equal_c_oracle_on_oracle_symbols": int(oracle_equal)}
    npx = cur.shape[-1] * cur.shape[-2]
    psnr_gpu = 10 * math.log10(1.0 / float(out[1]))
    psnr_cpu = 10 * math.log10(1.0 / float(oracle_out[1]))
    par.update({
        "symbol_mismatch_rate": total_flip / total_sym,
        "symbol_mismatch_bound": SYMBOL_FLIP_BOUND,
        "dpsnr_db": abs(psnr_gpu - psnr_cpu), "dpsnr_bound_db": DPSNR_BOUND_DB,
        "psnr_gpu_db": round(psnr_gpu, 6), "psnr_cpu_db": round(psnr_cpu, 6),
        "bpp_est_gpu": float(out[7]), "bpp_est_cpu": float(oracle_out[7]),
        "dbpp_est_rel": abs(float(out[7]) - float(oracle_out[7])) / float(oracle_out[7]),
        "bpp_actual_gpu": bs.nbytes() * 8 / npx,
        "bitstream_t1_byte_exact": all(v["streams_bytes_equal_c_oracle_same_symbols"] == v["streams"]
                                      for v in par["latents"].values()),
    })
    coder = {"encode_symbols_per_s": round(nsym / t_enc), "decode_symbols_per_s": round(nsym / t_dec),
             "symbols": nsym, "note": f"oracle/rans_ref.c (-O2), all streams of the frame ({bs.framing} framing), "
                                      f"one core"}
    return par, coder


# ------------------------------------------------------------------ per-rank workload
class GpuGopJob:
    """One rank's share of the benchmark: G GOPs resident in HBM, pipelined encode+decode."""

    def __init__(self, args, rank, world, dev):
        from fastvideocodec_amd.models import get_codec_model
        from fastvideocodec_amd.synthetic import gop_seed, make_gop
        self.args, self.dev = args, dev
        self.model = get_codec_model("DVC-pretrained", compression_level=2, device=dev)
        self.model.update()
        if args.views > 0:
            if args.views < world:
                raise SystemExit(f"--views {args.views} < world size {world}: a rank would have no view")
            mine = fdist.shard_views(args.views, rank, world)
            gops = [make_gop(args.height, args.width, args.gop, gop_seed(0, v)) for v in mine]
        else:
            mine = fdist.shard_gops(world * args.gops_per_gpu, rank, world)  # GOP g -> rank g % world
            gops = [make_gop(args.height, args.width, args.gop, gop_seed(g)) for g in mine]
        self.shard = mine  # GOP (or view) ids this rank codes
        self.gops_np = gops
        self.units = len(gops)
        self.frames = torch.from_numpy(np.stack(gops)).to(dev)  # [G, T, 3, Hp, Wp]
        self.Hp, self.Wp = self.frames.shape[-2:]

    def step(self):
        if self.args.tree:
            from fastvideocodec_amd.tree_gop import encode_decode_tree_gop
            # streamed like the linear GOP: no per-step host wait, overflow probes resolved in
            # after_timing (gop.check_overflow); past 31 P-frames the 62-frame binary tree
            encode_decode_tree_gop(self.model, self.frames, overlap=not self.args.serial, join=False,
                                   extend=True)
            return
        from fastvideocodec_amd.gop import encode_decode_gop
        encode_decode_gop(self.model, self.frames, overlap=not self.args.serial, join=False)

    def sync(self):
        torch.cuda.synchronize()

    def _tree_layers(self):
        from fastvideocodec_amd.tree_gop import coding_layers
        return coding_layers(self.args.gop - 1, extend=True)

    def after_timing(self):
        """Roofline pass: one serial GOP (single stream) with HIP events around every launch on
        the launching stream (in the overlapped timed region concurrent kernels would be charged
        to each other's event windows); plus the streamed GOPs' overflow probes."""
        from fastvideocodec_amd import gop, profiling
        from fastvideocodec_amd.gop import encode_decode_gop
        gop.check_overflow(self.model)  # raises if a timed GOP left the split-precision range
        timer = profiling.KernelTimer()
        with timer:
            encode_decode_gop(self.model, self.frames, overlap=False)
        r = {"conv": timer.collect(), "x3": timer.collect(x3=True), "x3_bytes": timer.collect_bytes(x3=True),
             "hbm": timer.collect_hbm(),
             "family": {f: (timer.collect(x3=True, family=f), timer.collect_bytes(x3=True, family=f))
                        for f in ("x3", "dx", "wino", "wr7", "stem")}}
        if self.args.breakdown:
            for k, (n, ms, fl) in sorted(timer.breakdown().items(), key=lambda kv: -kv[1][1]):
                print(f"{k:40s} n={n:5d} ms={ms:9.2f} TF/s={fl / (ms * 1e-3) / 1e12:7.2f}", file=sys.stderr)
        return r

    def parity(self, threads):
        """Parity block of this rank's first unit, frame 1 (rank_parity)."""
        return rank_parity(self.model, self.dev, self.gops_np[0], self.shard[0], threads)

    def verify(self):
        from fastvideocodec_amd.gop import encode_decode_gop
        overflow_before = getattr(self.model, "overflow_events", 0)
        if self.args.tree:
            from fastvideocodec_amd.tree_gop import encode_decode_tree_gop
            bss, dd, sses, ee = encode_decode_tree_gop(self.model, self.frames, check=True,
                                                       overlap=not self.args.serial, extend=True)
            decoded, encs = [dd[t] for t in sorted(dd)], [ee[t] for t in sorted(ee)]
            sses = [s / len(lay) for s, lay in zip(sses, self._tree_layers())]  # per-frame mean SSE
        else:
            bss, decoded, sses, encs = encode_decode_gop(self.model, self.frames, check=True,
                                                         overlap=not self.args.serial)
        torch.cuda.synchronize()
        npx = self.units * 3 * self.Hp * self.Wp
        psnrs = [float(10 * np.log10(1.0 / (float(s[0]) / npx))) for s in sses]
        payload = b"".join(s for bs in bss for s in bs.mv.to_bytes_list() + bs.z.to_bytes_list()
                           + bs.feature.to_bytes_list())
        return {"bitexact": all(torch.equal(a, b) for a, b in zip(decoded, encs)),
                "nbytes": sum(b.nbytes() for b in bss), "psnr": float(np.mean(psnrs)), "payload": payload,
                "overflow_recomputes": getattr(self.model, "overflow_events", 0) - overflow_before}


class HostRehearsalJob:
    """`--dry-run`: the per-rank job's interface with host-only work (no GPU, no codec), so the
    launcher, the rank partitioning and the collectives can be rehearsed under gloo on CPU
    (tests/test_bench_dist.py). Its numbers measure nothing."""

    def __init__(self, args, rank, world):
        self.args = args
        if args.views > 0:
            if args.views < world:
                raise SystemExit(f"--views {args.views} < world size {world}: a rank would have no view")
            self.shard = fdist.shard_views(args.views, rank, world)
        else:
            self.shard = fdist.shard_gops(world * args.gops_per_gpu, rank, world)
        self.units = len(self.shard)
        self.Hp, self.Wp = (args.height + 63) // 64 * 64, (args.width + 63) // 64 * 64
        self.rank = rank

    def step(self):
        time.sleep(0.005 * (1 + self.rank))

    def sync(self):
        pass

    def after_timing(self):
        return None

    def parity(self, threads):
        """Stand-in parity block (no GPU): the fields a real rank reports, all zero mismatches."""
        lat = {"mv": (128, 2), "z": (64, 0), "feature": (96, 0)}
        par = {"frame": f"unit {self.shard[0]} frame 1 vs frame 0 (dry run)", "dpsnr_db": 0.0, "dbpp_est_rel": 0.0,
               "latents": {k: {"symbols": c * 100, "symbol_mismatches": 0, "index_mismatches": 0, "streams": c,
                               "streams_bytes_equal_c_oracle_same_symbols": c,
                               "streams_bytes_equal_c_oracle_on_oracle_symbols": c} for k, (c, _) in lat.items()}}
        return par, None

    def verify(self):
        payload = b"".join(bytes([u % 256]) * (100 + u) for u in self.shard)
        return {"bitexact": True, "nbytes": len(payload), "psnr": 30.0, "payload": payload,
                "overflow_recomputes": 0}


def run_rank(job, args, rank, world, device):
    """Warm-up, the timed region (barrier + device sync on both sides, max over ranks), then one
    collective round after timing. Returns the result dict on rank 0, None elsewhere."""
    for _ in range(args.warmup):
        job.step()
    job.sync()
    if world > 1:
        dist.barrier()
    job.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.step()
    job.sync()
    if world > 1:
        dist.barrier()
    job.sync()
    dt = time.perf_counter() - t0

    prof = job.after_timing()
    ver = job.verify()
    # every rank checks its own first unit against the oracle (host threads shared among the
    # node's ranks), before the collectives so the ranks do it concurrently
    par = coder = None
    cap = parity_rank_cap(args, world)
    if getattr(args, "cpu_baseline", "none") != "none" and hasattr(job, "parity") and rank < cap:
        par, coder = job.parity(max(1, cpu_cores() // cap))
    pvec = fdist.gather_stats(parity_vector(par), device)
    dt_max = fdist.max_over_ranks(dt, device)
    allst = fdist.gather_stats([1.0 if ver["bitexact"] else 0.0, float(ver["nbytes"]), ver["psnr"],
                                float(job.units), float(ver["overflow_recomputes"])], device)
    gathered = fdist.gather_bytes(ver["payload"], device, dst=0)
    shards = fdist.gather_bytes(json.dumps(list(getattr(job, "shard", []))).encode(), device, dst=0)
    if rank != 0:
        return None
    units = int(allst[:, 3].sum())
    pframes_per_step = units * (args.gop - 1)
    value = args.steps * pframes_per_step / dt_max
    bitexact_all = bool(np.all(allst[:, 0] == 1.0)) and sum(len(g) for g in gathered) == int(allst[:, 1].sum())
    bytes_all = float(allst[:, 1].sum())
    enc_tf, dec_tf = tflop_per_pframe(job.Hp, job.Wp)
    res_label = f"{args.width}x{args.height} (padded {job.Wp}x{job.Hp})"
    tree_info = None
    if getattr(args, "tree", False):
        from fastvideocodec_amd.tree_gop import coding_layers
        lay = coding_layers(args.gop - 1, extend=True)
        tree_info = {"layers": [[t for t, _ in l] for l in lay], "depth": len(lay),
                     "structure": ("the reference's graph_from_batch tree (models.py:683-728)" if args.gop - 1 <= 30
                                   else "EXTENSION (not a reference structure): prefix of the 62-frame binary tree "
                                        "(binary_tree_graph), the reference's graphs stop at 30 P-frames")}
    result = {
        "metric": metric_name(args.height, args.width),
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
        "config": ({"workload": f"DVC P-frame encode+decode with rANS, {res_label} GOP-{args.gop}"
                                f"{' as an LSVC reference tree (models.py:683-728), one batch per tree layer' if args.tree else ''}"
                                f", lambda=1024 slot",
                    "gops_per_gpu": job.units, "frames_counted": "P-frames only (I-frame pass-through)",
                    "parallelism": f"gop-shard x{world}", **({"tree": tree_info} if tree_info else {})}
                   if args.views <= 0 else
                   {"workload": f"{args.views}-view DVC P-frame encode+decode with rANS, {res_label} GOP-{args.gop} "
                                f"per view, lambda=1024 slot",
                    "views": args.views, "views_per_gpu": job.units,
                    "frames_counted": "P-frames only (I-frame pass-through)",
                    "parallelism": f"view-shard x{world}"}),
        "shards": {"unit": "view" if args.views > 0 else "gop",
                   "by_rank": [json.loads(s.decode()) for s in shards]},
        "model_tflop_per_pframe": round(enc_tf + dec_tf, 3),
        "effective_tflops": round(value / world * (enc_tf + dec_tf), 2),
        "quality": {"decoder_bitexact": bitexact_all,
                    "bytes_per_pframe": round(bytes_all / pframes_per_step, 1),
                    "bpp_actual": round(bytes_all * 8 / (pframes_per_step * job.Hp * job.Wp), 5),
                    "psnr_db_mean": round(float(np.mean(allst[:, 2])), 4),
                    "overflow_recomputes": int(allst[:, 4].sum()),
                    "bitstreams_gathered_to_rank0_bytes": sum(len(g) for g in gathered),
                    "note": "seeded (untrained) codec weights + synthetic GOP: PSNR/bpp are not rate-distortion "
                            "figures; the coder's symbol statistics (and so its timing) are those of untrained "
                            "weights (~5 bpp vs DVC's 0.137 bpp at lambda=1024)"},
    }
    if par is not None:
        by_rank = []
        for r, v in enumerate(pvec):
            d = dict(zip(PARITY_FIELDS, (float(x) for x in v)))
            if not d["checked"]:
                by_rank.append({"rank": r, "checked": False})
                continue
            by_rank.append({"rank": r, "unit": result["shards"]["by_rank"][r][0],
                            "symbol_mismatch_rate": d["symbol_mismatches"] / max(d["symbols"], 1.0),
                            "symbol_mismatches": int(d["symbol_mismatches"]), "symbols": int(d["symbols"]),
                            "index_mismatches": int(d["index_mismatches"]), "dpsnr_db": d["dpsnr_db"],
                            "dbpp_est_rel": d["dbpp_est_rel"],
                            "bitstream_t1_byte_exact": d["streams_t1_equal"] == d["streams"],
                            "streams_bytes_equal_on_oracle_symbols": int(d["streams_equal_on_oracle_symbols"]),
                            "streams": int(d["streams"])})
        checked = [b for b in by_rank if b.get("checked", True)]
        result["quality"]["parity"] = par  # rank 0's full block
        result["quality"]["parity_by_rank"] = by_rank
        pa = {"ranks_checked": len(checked), "parity_ranks_cap": cap,
              "max_symbol_mismatch_rate": max(b["symbol_mismatch_rate"] for b in checked),
              "symbol_mismatch_bound": SYMBOL_FLIP_BOUND,
              "max_dpsnr_db": max(b["dpsnr_db"] for b in checked), "dpsnr_bound_db": DPSNR_BOUND_DB,
              "bitstream_t1_byte_exact": all(b["bitstream_t1_byte_exact"] for b in checked)}
        if cap < world:
            pa["note"] = (f"ranks 0..{cap - 1} checked (--parity-ranks {cap}): each check is one 1080p oracle "
                          f"forward on the host cores shared by the checking ranks")
        pa["ok"] = bool(pa["max_symbol_mismatch_rate"] <= SYMBOL_FLIP_BOUND and pa["max_dpsnr_db"] <= DPSNR_BOUND_DB
                        and pa["bitstream_t1_byte_exact"] and bitexact_all)
        result["quality"]["parity_all_ranks"] = pa
        if coder is not None:
            result["_coder"] = coder
    if prof is not None:
        result.update(roofline_fields(prof, job, args))
    return result


def roofline_fields(prof, job, args):
    conv_ms, conv_flops, n_launch = prof["conv"]
    x3_ms, x3_flops, x3_launch = prof["x3"]
    x3_bytes = prof["x3_bytes"]
    nfr = job.units * (args.gop - 1)
    achieved = x3_flops / (x3_ms * 1e-3) / 1e12 if x3_ms > 0 else 0.0
    pmc = load_pmc_traffic(args.height, args.width, job.units)
    return {
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": F16_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / F16_MFMA_PEAK_TFLOPS, 4),
                     "traffic": pmc.get("hbm_bytes_per_launch"),
                     "traffic_source": pmc.get("source"),
                     "avg_launch_us": round(x3_ms * 1e3 / x3_launch, 2) if x3_launch else None,
                     "algorithmic_bytes_per_launch": round(x3_bytes / x3_launch) if x3_launch else None,
                     "algorithmic_gbps": round(x3_bytes / (x3_ms * 1e-3) / 1e9, 1) if x3_ms else None,
                     "kernel": "split-precision conv kernels (every conv launch but 4 small-cin layers): "
                               "conv_x3_kernel (fp16x3 implicit-GEMM conv/deconv) + conv_dx_kernel (stride-2 "
                               "transposed convs, all parity classes per staged tile) + conv_wino_kernel (Winograd "
                               "F(2x2,3x3) for the 64->64 3x3 layers, and the 544x960 128->128 ones as four 64->64 "
                               "quarters) + conv_wr7_kernel (Winograd-rows F(2,7) for SpyNet's 7x7 32->64, 64->32 "
                               "and 32->16 layers) + conv_stem_kernel (the cin <= 8 stems: Warp_net feature_ext, "
                               "mvEncoder conv1, resEncoder conv1), all their dispatches",
                     "achieved_is": "algorithmic fp32-conv FLOP (2 x MAC of the direct convolution) / kernel time; "
                                    "the direct kernel issues 3 f16 MFMAs per MAC (ceiling peak/3), the Winograd "
                                    "kernel 3 per 16/36 MAC (ceiling peak/3 x 36/16), the Winograd-rows kernel 3 per "
                                    "28/49 MAC (ceiling peak/3 x 49/28); frac_issued / issued_tflops count the f16 "
                                    "MFMA FLOP each family issues per algorithmic FLOP as measured by SQ_INSTS_MFMA "
                                    "(bench.ISSUED_PER_FLOP, profiles/r6/pmc_families.txt: padding included)",
                     "x3_ceiling": round(F16_MFMA_PEAK_TFLOPS / 3, 1),
                     "frac_of_x3_ceiling": round(achieved / (F16_MFMA_PEAK_TFLOPS / 3), 4),
                     **issued_fields(prof, x3_ms),
                     "per_kernel": per_kernel_fields(prof, nfr),
                     "dominant_kernel": dominant_kernel_fields(per_kernel_fields(prof, nfr)),
                     "fused_hbm_work": "since r6 the Warp_net upsample-adds (c3_u = c1 + up(c3), c4_u = c0 + "
                                       "up(c4), endecoder.py:288-293; 0.63 ms per P-frame as a standalone HBM kernel "
                                       "in r5) are formed inside the ResBlock conv1 Winograd launches that read them: "
                                       "their time is in this family's and their bytes in algorithmic_bytes_per_launch",
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
                        for k, (n, ms, b) in sorted(prof["hbm"].items(), key=lambda kv: -kv[1][1])},
    }


# f16 MFMA FLOP issued per algorithmic fp32-conv FLOP, per kernel family: 3 split products (hi*hi,
# hi*lo, lo*hi) per MAC; Winograd F(2x2,3x3) computes 16 products per 36 direct MACs, the
# Winograd-rows F(2,7) 28 per 49
# f16 MFMA FLOP issued per algorithmic FLOP, per family: SQ_INSTS_MFMA x FLOP per instruction over
# the bench's serial pass / the pass's algorithmic FLOP (profiles/r6/pmc_families.txt, r6). The
# models they replace (direct 3, Winograd 3 x 16/36, Winograd-rows 3 x 28/49) miss the K padding
# of the small-cin stems (3 -> 4.68: K rounded up to whole 16-deep k-steps), the x3 / dx tile
# padding (3.16 / 3.10) and the tap-partial epilogues' MFMAs (Winograd 1.348)
ISSUED_PER_FLOP = {"x3": 3.156, "dx": 3.101, "wino": 1.348, "wr7": 1.716, "stem": 4.685}


def issued_fields(prof, fam_ms):
    """the family against what its own arithmetic could reach. frac_issued = f16 MFMA
    FLOP actually issued / family time / f16 peak; frac_of_blended_ceiling = the time the family's
    algorithmic FLOP would take at each kernel's own ceiling (direct: peak/3; Winograd: peak/3 x
    36/16) / the measured time. The two are the same quantity computed two ways."""
    issued = ceil_s = 0.0
    for fam, k in ISSUED_PER_FLOP.items():
        (ms, fl, n), _ = prof["family"][fam]
        issued += k * fl
        ceil_s += fl / (F16_MFMA_PEAK_TFLOPS * 1e12 / k)
    if fam_ms <= 0:
        return {}
    return {"frac_issued": round(issued / (fam_ms * 1e-3) / (F16_MFMA_PEAK_TFLOPS * 1e12), 4),
            "issued_tflops": round(issued / (fam_ms * 1e-3) / 1e12, 1),
            "frac_of_blended_ceiling": round(ceil_s / (fam_ms * 1e-3), 4),
            "blended_ceiling_tflops": round(sum(prof["family"][f][0][1] for f in ISSUED_PER_FLOP) / ceil_s / 1e12, 1)
            if ceil_s else None}


def per_kernel_fields(prof, nfr):
    """The roofline object split by kernel: algorithmic TF/s, launches and time of conv_x3_kernel,
    conv_dx_kernel and conv_wino_kernel, and for Winograd the f16 matrix rate it actually issues (3 MFMAs per
    16/36 of a direct MAC)."""
    out = {}
    for fam, name in (("x3", "conv_x3_kernel"), ("dx", "conv_dx_kernel"), ("wino", "conv_wino_kernel"),
                      ("wr7", "conv_wr7_kernel"), ("stem", "conv_stem_kernel")):
        (ms, fl, n), nbytes = prof["family"][fam]
        if not n:
            continue
        tf = fl / (ms * 1e-3) / 1e12
        out[name] = {"achieved": round(tf, 2), "launches": n, "avg_launch_us": round(ms * 1e3 / n, 2),
                     "ms_per_pframe": round(ms / nfr, 3), "gflop_per_pframe": round(fl / nfr / 1e9, 1),
                     "algorithmic_gbps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                     "f16_mfma_tflops_issued": round(ISSUED_PER_FLOP[fam] * tf, 1),
                     "frac_of_f16_peak_issued": round(ISSUED_PER_FLOP[fam] * tf / F16_MFMA_PEAK_TFLOPS, 4),
                     **attainable_fields(tf, nbytes / (ms * 1e-3), fam)}
    return out


def dominant_kernel_fields(pk):
    """The family member with the most time per P-frame, on the roofline its own arithmetic
    intensity puts it on (attainable_fields): for the Winograd kernel HBM, so achieved / peak are
    algorithmic GB/s / 8 TB/s. The family's `frac` above stays the MFMA-peak framing."""
    if not pk:
        return None
    name, v = max(pk.items(), key=lambda kv: kv[1]["ms_per_pframe"])
    if v.get("attainable_bound") == "hbm":
        achieved, peak, unit = v["algorithmic_gbps"], HBM_PEAK_BPS / 1e9, "GB/s"
    else:
        achieved, peak, unit = v["achieved"], F16_MFMA_PEAK_TFLOPS / ISSUED_PER_FLOP[FAMILY_OF[name]], "TFLOP/s"
    return {"kernel": name, "bound": v.get("attainable_bound"), "achieved": achieved, "peak": round(peak, 1),
            "unit": unit, "frac": round(achieved / peak, 4) if peak else None,
            "flop_per_byte": v.get("flop_per_byte"), "ms_per_pframe": v["ms_per_pframe"]}


FAMILY_OF = {"conv_x3_kernel": "x3", "conv_dx_kernel": "dx", "conv_wino_kernel": "wino", "conv_wr7_kernel": "wr7",
             "conv_stem_kernel": "stem"}


def attainable_fields(tflops, bytes_per_s, fam):
    """The roofline model for one kernel family: attainable = min(its MFMA ceiling (f16 peak / the
    f16 FLOP it issues per algorithmic FLOP), arithmetic intensity (algorithmic FLOP per algorithmic
    byte) x 8 TB/s); `bound` names the smaller. The Winograd family's intensity is low enough
    (~120-140 FLOP per byte against a ~230 ridge for its ceiling) that HBM bounds it."""
    if bytes_per_s <= 0:
        return {}
    ai = tflops * 1e12 / bytes_per_s
    mfma_ceiling = F16_MFMA_PEAK_TFLOPS / ISSUED_PER_FLOP[fam]
    hbm_ceiling = ai * HBM_PEAK_BPS / 1e12
    att = min(mfma_ceiling, hbm_ceiling)
    return {"flop_per_byte": round(ai, 1), "frac_of_8tbps": round(bytes_per_s / HBM_PEAK_BPS, 4),
            "attainable_tflops": round(att, 1), "attainable_bound": "hbm" if hbm_ceiling < mfma_ceiling else "mfma",
            "frac_of_attainable": round(tflops / att, 4)}


def load_pmc_traffic(H, W, gops):
    """HBM bytes per conv_x3_kernel launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes
    over `bench.py --serial` (profiles/<round>/x3_traffic.json, written by scripts/rocprof_summary.py;
    FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction). PMC passes serialise every
    dispatch and cannot run inside the timed region, so the figure is the profiled one."""
    for rnd in ("r6", "r5", "r4", "r3", "r2", "r1"):
        path = os.path.join(REPO, "profiles", rnd, "x3_traffic.json")
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        # per-dispatch bytes depend on the batch: only a file profiled at this GOP count counts
        # (files without the field were profiled at 8)
        if d.get("height") != H or d.get("width") != W or d.get("gops_per_gpu", 8) != gops:
            continue
        return {"hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"),
                "source": f"profiles/{rnd}/x3_traffic.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                          f"{d.get('launches')} dispatches at {gops} GOPs per step)"}
    return {}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--gop", type=int, default=12)
    ap.add_argument("--gops-per-gpu", type=int, default=None,
                    help="GOPs batched per rank per step (SURVEY §8(e)); default 16 x 2 steps = 32 GOPs per run "
                         "(§8(d)), 4 with --tree (a tree layer batches up to 6 frames per GOP: 16 GOPs would "
                         "need ~50 GB per 1080p activation). Measured on MI355X: r3 8 -> 68.92/68.84, 16 -> "
                         "69.92/69.95/69.91, 24 -> 68.13, 32 -> 68.22 P-frames/s (profiles/r3/gops_sweep); r4 "
                         "12 -> 71.27/71.30, 16 -> 73.34/73.23, 24 -> 70.06/69.94 (profiles/r4/gops_sweep)")
    ap.add_argument("--views", type=int, default=0,
                    help="BASELINE configs[4]: V camera views, one GOP stream each, view v -> rank v %% world "
                         "(replaces --gops-per-gpu; the reference's MCVC couples views, DVC views are independent)")
    ap.add_argument("--cpu-baseline", choices=("quick", "full", "none"), default="full",
                    help="CPU leg + parity block on rank 0 at N=1: full (default; BASELINE.md §3 protocol, "
                         "~3 min), quick (~30 s), none")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="same as --cpu-baseline none")
    ap.add_argument("--no-ref-metrics", dest="ref_metrics", action="store_false",
                    help="skip the reference-comparable batch-1 figures (stage split, per-frame decode time, "
                         "drop-in parallel_compression throughput) rank 0 measures after timing")
    ap.add_argument("--parity-ranks", type=int, default=4,
                    help="ranks 0..K-1 run the per-rank oracle parity check after timing (default 4: at N = 8 "
                         "the other ranks skip it, so the CPU work stays bounded; the line says which ranks)")
    ap.add_argument("--strict-parity", action="store_true",
                    help="exit with status 3 when quality.parity_all_ranks.ok is false (the line is printed "
                         "either way)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--breakdown", action="store_true", help="print per-conv-geometry timing to stderr")
    ap.add_argument("--tree", action="store_true",
                    help="code each GOP as the LSVC reference tree (SURVEY §8(f)#4): one batched forward per "
                         "tree layer instead of one per frame (a different coding structure from the headline's "
                         "sequential DVC GOP; reported separately)")
    ap.add_argument("--serial", action="store_true",
                    help="one HIP stream (no encode/code/decode overlap): per-kernel durations are unshared")
    ap.add_argument("--dry-run", action="store_true",
                    help="rehearse the launcher, sharding and collectives on CPU (gloo) with a host job: "
                         "no GPU work, the numbers measure nothing")
    args = ap.parse_args(argv)
    if args.no_cpu_baseline:
        args.cpu_baseline = "none"
    if args.gops_per_gpu is None:
        args.gops_per_gpu = 4 if args.tree else 16
    return args


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """`python bench.py --gpus N` outside a launcher: start N fresh rank processes (this parent
    never touches the GPU, so no process that has initialised HIP is replaced), one per GPU,
    with the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, rendezvous on
    127.0.0.1). Only rank 0 prints. If a rank fails, the others are stopped (their exact PIDs).
    Returns the first non-zero exit status, or 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    try:
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
    finally:
        # interrupted (KeyboardInterrupt / SIGTERM turned into an exception): stop the exact rank
        # processes this parent started, then kill what is still alive, and report a failure
        if live:
            rc = rc or 1
            for q in live:
                if q.poll() is None:
                    q.terminate()
            deadline = time.time() + 10
            for q in live:
                try:
                    q.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    q.kill()
                    q.wait()
    return rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a result must never mislabel its rank count
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world} set by the launcher")
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        job, dev = HostRehearsalJob(args, rank, world), None
    else:
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        job = GpuGopJob(args, rank, world, dev)
    result = run_rank(job, args, rank, world, dev)
    if args.dry_run and rank == 0:
        result["data"] = "dry run: host rehearsal job, no GPU work (launcher / sharding / collectives only)"
    if rank == 0 and not args.dry_run and args.ref_metrics:
        result["reference_comparable"] = reference_metrics(job.model, job.frames[0])
    # the CPU leg on rank 0 at every N, after the timed region and the collectives
    if rank == 0 and args.cpu_baseline != "none":
        coder = result.pop("_coder", None)
        if args.dry_run:
            result["cpu_baseline"] = dry_cpu_baseline()
        else:
            result["cpu_baseline"] = cpu_baseline(job.gops_np[0], args.cpu_baseline, coder)
        result["cpu_baseline"]["n_gpus_in_run"] = world
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()
    if rank == 0 and args.strict_parity:
        pa = result.get("quality", {}).get("parity_all_ranks")
        if pa is not None and not pa["ok"]:
            print("[bench] parity FAILED: " + json.dumps(pa), file=sys.stderr, flush=True)
            return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
