"""BASELINE.json configs exercised through the bench's own per-rank job on one GPU (small frames,
so the checks run in seconds): configs[4] (8 camera views, one GOP stream per view, view v on rank
v % world) and the default GOP sharding. The properties are size-independent: decoder recon ==
encoder recon bit for bit, every view coded in the batch == that view coded alone (views are
independent streams), and the rank job's verify() agrees."""
import argparse

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _args(**kw):
    a = argparse.Namespace(gpus=1, steps=1, warmup=0, height=96, width=128, gop=3, gops_per_gpu=2, views=0,
                           cpu_baseline="none", json_out=None, breakdown=False, tree=False, serial=False)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_views_config_one_gpu(dev):
    """configs[4] on one GPU (bench --views 8): all 8 views batch into one rank's job; each view's
    decoded frames equal the same view coded alone, and the decoder is bit-exact."""
    import bench
    from fastvideocodec_amd.gop import encode_decode_gop

    job = bench.GpuGopJob(_args(views=8), 0, 1, dev)
    assert job.units == 8 and tuple(job.frames.shape[:2]) == (8, 3)
    job.step()
    job.sync()
    v = job.verify()
    assert v["bitexact"] and v["nbytes"] > 0 and v["overflow_recomputes"] == 0
    _, dec_all, _, _ = encode_decode_gop(job.model, job.frames, check=True, overlap=True)
    for view in (0, 5):
        _, dec_one, _, enc_one = encode_decode_gop(job.model, job.frames[view:view + 1], check=True, overlap=False)
        torch.cuda.synchronize()
        for a, b, c in zip(dec_all, dec_one, enc_one):
            assert torch.equal(a[view:view + 1], b) and torch.equal(b, c)


def test_views_shard_over_ranks_match_one_rank(dev):
    """configs[4] over 2 ranks (run here one after the other on the same GPU): rank r codes views
    r, r+2, ...; the union of the two ranks' payloads has the same size as the one-rank run."""
    import bench

    one = bench.GpuGopJob(_args(views=4), 0, 1, dev)
    r0 = bench.GpuGopJob(_args(views=4), 0, 2, dev)
    r1 = bench.GpuGopJob(_args(views=4), 1, 2, dev)
    assert (one.units, r0.units, r1.units) == (4, 2, 2)
    np.testing.assert_array_equal(r0.gops_np[1], one.gops_np[2])  # rank 0 holds views 0 and 2
    np.testing.assert_array_equal(r1.gops_np[0], one.gops_np[1])  # rank 1 holds views 1 and 3
    v_one, v0, v1 = one.verify(), r0.verify(), r1.verify()
    assert v_one["bitexact"] and v0["bitexact"] and v1["bitexact"]
    assert v0["nbytes"] + v1["nbytes"] == v_one["nbytes"]


def test_run_rank_default_config(dev):
    """bench.run_rank on one rank with the real GPU job: the result line carries the headline
    fields and the decoder bit-exactness check."""
    import bench

    job = bench.GpuGopJob(_args(steps=2, warmup=1), 0, 1, dev)
    res = bench.run_rank(job, job.args, 0, 1, dev)
    assert res["n_gpus"] == 1 and res["steps"] == 2 and res["value"] > 0
    assert res["quality"]["decoder_bitexact"] is True


def test_4k_gop_batch_split_pipeline(dev):
    """configs[3] shape on one GPU: three 4K GOPs (3840x2160 -> 2176) through the overlapped GOP
    pipeline. Their 64-channel full-resolution activations are 6.4 GB per launch, so every such
    conv runs as launches over sub-batches (the 32-bit buffer-offset split); the decoder must still
    match the encoder bit for bit and each GOP must equal that GOP coded alone."""
    from fastvideocodec_amd.gop import encode_decode_gop
    from fastvideocodec_amd.models import get_codec_model
    from fastvideocodec_amd.synthetic import gop_seed, make_gop

    model = get_codec_model("DVC-pretrained", compression_level=2, device=dev)
    frames = torch.from_numpy(np.stack([make_gop(2160, 3840, 2, gop_seed(g)) for g in (3, 4, 5)])).to(dev)
    assert 3 * 2176 * 3840 * 64 * 4 >= (1 << 32) - 4096  # the split path is taken
    _, dec, _, enc = encode_decode_gop(model, frames, check=True, overlap=True)
    _, dec1, _, enc1 = encode_decode_gop(model, frames[1:2], check=True, overlap=False)
    torch.cuda.synchronize()
    for a, b, c in zip(dec, enc, dec1):
        assert torch.equal(a, b) and torch.equal(a[1:2], c)


def test_views8_1080p_config4(dev):
    """BASELINE configs[4] at its own size: 8 camera views of 1920x1080 (padded to 1088) batched
    through the bench's rank job (GOP-3 per view). Decoder recon == encoder recon bit for bit,
    views 0 and 7 coded alone equal their batch slots, no split-precision overflow, and view 0's
    frame-1 latents from the 8-view batched forward match the CPU oracle within the 1080p T3
    bounds (test_gpu_forward.py: aggregate flips <= 1.56e-5 of 1.86 M symbols, dPSNR <= 1e-4 dB)."""
    import os

    import bench
    from fastvideocodec_amd import kernels as K
    from fastvideocodec_amd.gop import encode_decode_gop
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    from oracle import dvc_ref

    job = bench.GpuGopJob(_args(views=8, height=1080, width=1920, gop=3), 0, 1, dev)
    assert job.units == 8 and tuple(job.frames.shape) == (8, 3, 3, 1088, 1920)
    assert job.shard == list(range(8))
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(job.model, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    for a, b in zip(dec, enc):
        assert torch.equal(a, b)
    for view in (0, 7):
        _, dec1, _, enc1 = encode_decode_gop(job.model, job.frames[view:view + 1], check=True, overlap=False)
        torch.cuda.synchronize()
        for a, b, c in zip(dec, dec1, enc1):
            assert torch.equal(a[view:view + 1], b) and torch.equal(b, c)
    v = job.verify()
    assert v["bitexact"] and v["overflow_recomputes"] == 0
    assert not K.x3_overflow(reset=True)

    # view 0, frame 1 (against the I-frame) out of the batched 8-view forward vs the oracle
    out, t = job.model(job.frames[:, 1].contiguous(), job.frames[:, 0].contiguous(), return_intermediates=True)
    torch.cuda.synchronize()
    cur, ref = job.frames[0:1, 1].cpu(), job.frames[0:1, 0].cpu()
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    (o_clip, o_mse, *_), inter = dvc_ref.forward(seeded_torch_state_dict(), cur, ref, return_intermediates=True)
    nflip = ntot = 0
    for name, gname, c in (("mvfeature", "quant_mv", 128), ("feature", "compressed_feature", 96),
                           ("z", "compressed_z", 64)):
        got = np.round(t[name][0:1, ..., :c].permute(0, 3, 1, 2).cpu().numpy())
        d = got != inter[gname].numpy()
        nflip += int(d.sum())
        ntot += d.size
    assert nflip / ntot <= 1.56e-5, (nflip, ntot)
    sse_gpu = float(((out[0][0:1].cpu() - cur) ** 2).sum())
    sse_cpu = float(((o_clip - cur) ** 2).sum())
    dpsnr = abs(10 * np.log10(sse_cpu / sse_gpu))
    assert dpsnr <= 1e-4, dpsnr


@pytest.mark.timeout(420)
def test_4k_gop32_one_rank_share(dev):
    """BASELINE configs[3] at its own workload: one rank's share of the 4-GPU split, i.e. one
    3840x2160 (padded to 2176) GOP-32 = 31 chained P-frames through the bench's rank job
    (models.py:372-376's sequential loop, encode + rANS + decode). Checks: decoder recon == encoder
    recon bit for bit over all 31 P-frames, no split-precision overflow anywhere in the chain (31
    chained reconstructions at 4K, flag clear after frame 31), and frame 1's latents / PSNR vs the
    CPU oracle: dPSNR <= 1e-4 dB, and symbol flips no more than the reference's own flips on this
    frame between its CPU backends / its fp32 and float64 runs (committed fixture, measured r5:
    native 48, channels-last 30, 1 thread 2, float64 193 of 7.44 M) or the fp32-MFMA path's
    (measured r4: split path 154, fp32 159)."""
    import os

    import bench
    from fastvideocodec_amd import kernels as K
    from fastvideocodec_amd.gop import encode_decode_gop
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    from oracle import dvc_ref

    job = bench.GpuGopJob(_args(gop=32, gops_per_gpu=1, height=2160, width=3840), 2, 4, dev)
    assert job.units == 1 and job.shard == [2] and tuple(job.frames.shape) == (1, 32, 3, 2176, 3840)
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(job.model, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    assert len(dec) == 31 and len(bss) == 31
    for t, (a, b) in enumerate(zip(dec, enc), 1):
        assert torch.equal(a, b), f"P-frame {t}: decoder recon != encoder recon"
    assert getattr(job.model, "overflow_events", 0) == 0
    assert not K.x3_overflow(reset=True)
    assert all(bs.precision == "x3" for bs in bss)
    del dec, enc, bss

    cur, ref = job.frames[0:1, 1].cpu(), job.frames[0:1, 0].cpu()
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    (o_clip, o_mse, *_), inter = dvc_ref.forward(seeded_torch_state_dict(), cur, ref, return_intermediates=True)

    def flips(t):
        n = tot = 0
        per = {}
        for name, gname, c in (("mvfeature", "quant_mv", 128), ("feature", "compressed_feature", 96),
                               ("z", "compressed_z", 64)):
            got = np.round(t[name][..., :c].permute(0, 3, 1, 2).cpu().numpy())
            d = got != inter[gname].numpy()
            per[gname] = int(d.sum())
            n += int(d.sum())
            tot += d.size
        return n, tot, per

    with K.precision("f32"):
        _, t32 = job.model(job.frames[:, 1].contiguous(), job.frames[:, 0].contiguous(), return_intermediates=True)
        n32, _, per32 = flips(t32)
    del t32
    out, t = job.model(job.frames[:, 1].contiguous(), job.frames[:, 0].contiguous(), return_intermediates=True)
    torch.cuda.synchronize()
    nflip, ntot, per = flips(t)
    # the bound is the reference's own flips on this frame, measured in the build
    # container by tests/golden/gen_fullsize_parity.py (tests/golden/ref_fullsize_parity.json): the
    # reference forward run under ATen's native convs, oneDNN on one thread, oneDNN channels-last
    # and in float64, each against its default oneDNN run (which the oracle equals here: 0 flips).
    # The largest, fp32 vs float64, is how far the reference's own fp32 arithmetic lands from the
    # exact result; the fp32-MFMA path on the same frame is kept as the second anchor.
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "ref_fullsize_parity.json")) as f:
        k4 = json.load(f)["k4_frame1"]
    assert k4["oracle_vs_onednn8"]["flips"]["total"] == 0 and ntot == k4["variants"]["native"]["n_symbols"]
    ref_flips = {v: r["flips"]["total"] for v, r in k4["variants"].items()}
    print(f"4K frame 1 vs oracle: x3 {nflip} flips {per}, f32 {n32} flips {per32} of {ntot} symbols; "
          f"reference cross-backend {ref_flips}")
    assert nflip <= max(max(ref_flips.values()), n32), (nflip, n32, ref_flips)
    sse_gpu = float(((out[0].cpu() - cur) ** 2).sum())
    sse_cpu = float(((o_clip - cur) ** 2).sum())
    dpsnr = abs(10 * np.log10(sse_cpu / sse_gpu))
    assert dpsnr <= 1e-4, dpsnr


def test_gop32_four_rank_split(dev):
    """BASELINE configs[3]'s GOP structure (GOP-32: 31 P-frames per I-frame, one GOP per rank over
    4 ranks), at a small frame size, with the ranks' jobs run one after the other on this GPU: rank r
    codes GOP r (the same frames as GOP r of a one-rank job with 4 GOPs), every rank's decoder is
    bit-exact over all 31 P-frames without split-precision overflow, and the four ranks' payloads
    add up to the one-rank job's."""
    import bench
    from fastvideocodec_amd import kernels as K

    one = bench.GpuGopJob(_args(gop=32, gops_per_gpu=4, height=64, width=96), 0, 1, dev)
    assert one.units == 4 and tuple(one.frames.shape[:2]) == (4, 32)
    v_one = one.verify()
    assert v_one["bitexact"] and v_one["overflow_recomputes"] == 0
    total = 0
    for r in range(4):
        job = bench.GpuGopJob(_args(gop=32, gops_per_gpu=1, height=64, width=96), r, 4, dev)
        assert job.shard == [r] and job.units == 1
        np.testing.assert_array_equal(job.gops_np[0], one.gops_np[r])
        K.x3_overflow(reset=True)
        v = job.verify()
        assert v["bitexact"] and v["overflow_recomputes"] == 0 and not K.x3_overflow(reset=True)
        total += v["nbytes"]
    assert total == v_one["nbytes"]
