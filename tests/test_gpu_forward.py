"""End-to-end parity of the HIP VideoCompressor against the reference golden fixtures
(produced by the reference DVC forward, tests/golden/gen_golden.py) and the CPU oracle."""
import os

import numpy as np
import pytest
import torch

from fastvideocodec_amd.models import get_codec_model, parallel_compression, PSNR
from oracle import dvc_ref

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

# fp32 tolerances (north star: recon within 1e-4 dB PSNR; symbols per SURVEY §7 tiers)
TOL_TENSOR = 2e-4      # relative to tensor max-abs (GOP chain / 1080p stage checks)
# per-stage max deviation from the reference's golden tensors, relative to the tensor's max-abs
# (measured r2 on MI355X over the three fixture sizes: estmv 5.1e-5 -- SpyNet's warp-and-refine
# iterations amplify ulp differences --, mvfeature 7.3e-6, others <= 5.5e-6), and the clipped
# reconstruction's absolute deviation (measured <= 8.1e-6; SURVEY §8(c) asks <= 1e-5)
TOL_STAGE = {"estmv": 1e-4, "mvfeature": 2e-5, "mv_up": 1e-5, "warpframe": 2e-5, "prediction": 1e-5,
             "feature": 1e-5, "z": 1e-5, "sigma": 1e-5}
TOL_CLIPPED_ABS = 1e-5
TOL_PSNR_DB = 1e-4
TOL_SYMBOL_FLIP = 1e-3  # fraction of symbols allowed to differ at these tiny sizes (0 observed)


@pytest.fixture(scope="module")
def model(dev):
    return get_codec_model("DVC-pretrained", compression_level=2, device=dev)


def nhwc_to_nchw(t, c):
    return t[..., :c].permute(0, 3, 1, 2).cpu()


STAGES = {"estmv": 2, "mvfeature": 128, "mv_up": 2, "warpframe": 3, "prediction": 3, "feature": 96,
          "z": 64, "sigma": 96}
GOLD_NAME = {"mv_up": "quant_mv_upsample", "sigma": "recon_sigma"}


@pytest.mark.parametrize("size", ["64x64", "128x192", "256x256"])
def test_forward_vs_golden(model, dev, size):
    g = np.load(os.path.join(GOLD, f"dvc_{size}.npz"))
    cur = torch.from_numpy(g["input_image"]).to(dev)
    ref = torch.from_numpy(g["referframe"]).to(dev)
    out, t = model(cur, ref, return_intermediates=True)
    torch.cuda.synchronize()
    measured = {}
    for name, c in STAGES.items():
        got = nhwc_to_nchw(t[name], c).numpy()
        exp = g[GOLD_NAME.get(name, name)]
        scale = np.abs(exp).max() + 1e-6
        err = np.abs(got - exp).max()
        measured[name] = float(err / scale)
    measured["clipped_abs"] = float(np.abs(out[0].cpu().numpy() - g["clipped"]).max())
    print(f"golden {size} max rel dev per stage:", measured)
    for name in STAGES:
        assert measured[name] <= TOL_STAGE[name], (name, measured)
    assert measured["clipped_abs"] <= TOL_CLIPPED_ABS, measured
    for name, gname in (("mvfeature", "quant_mv"), ("feature", "compressed_feature"), ("z", "compressed_z")):
        got = np.round(nhwc_to_nchw(t[name], STAGES[name]).numpy())
        flips = float((got != g[gname]).mean())
        assert flips <= TOL_SYMBOL_FLIP, f"{gname}: flip rate {flips}"
    names = ["clipped", "mse_loss", "warploss", "interloss", "bpp_feature", "bpp_z", "bpp_mv", "bpp"]
    for n, o in zip(names, out):
        o = o.cpu().numpy()
        exp = g[n]
        if n == "clipped":
            continue  # checked above against TOL_CLIPPED_ABS
        else:
            assert abs(float(o) - float(exp)) <= 2e-4 * abs(float(exp)) + 1e-7, (n, float(o), float(exp))
    psnr_got = 10 * np.log10(1.0 / float(out[1]))
    psnr_exp = 10 * np.log10(1.0 / float(g["mse_loss"]))
    assert abs(psnr_got - psnr_exp) <= TOL_PSNR_DB


def _flip_rate(t, g, i=None):
    pre = "" if i is None else f"f{i}_"
    flips = []
    for name, gname in (("mvfeature", "quant_mv"), ("feature", "compressed_feature"), ("z", "compressed_z")):
        got = np.round(nhwc_to_nchw(t[name], STAGES[name]).numpy())
        flips.append(float((got != g[pre + gname]).mean()))
    return max(flips)


def test_gop_chain_vs_golden(model, dev):
    """parallel_compression loop (models.py:368-383) over a 4-frame GOP.

    Open loop (each P-frame coded against the reference's own previous recon): symbols match
    (flip rate <= TOL_SYMBOL_FLIP) and PSNR within 5e-4 dB (one flipped symbol of a 256x256
    frame moves PSNR by ~1e-4 dB; the 1e-4 dB bar is checked exactly on identical symbols in
    test_decode_from_golden_symbols). Closed loop (our own previous recon) the chain drifts the
    way the reference drifts across CPU backends, so the closed-loop bound is looser."""
    g = np.load(os.path.join(GOLD, "dvc_chain_256x256.npz"))
    gop = torch.from_numpy(g["gop"]).to(dev)
    exp_psnr = np.array([10 * np.log10(1 / float(g[f"f{i}_mse_loss"])) for i in range(1, 4)])
    for i in range(1, 4):
        ref = gop[0:1] if i == 1 else torch.from_numpy(g[f"f{i-1}_clipped"]).to(dev)
        out, t = model(gop[i:i + 1], ref, return_intermediates=True)
        assert _flip_rate(t, g, i) <= TOL_SYMBOL_FLIP
        assert abs(10 * np.log10(1 / float(out[1])) - exp_psnr[i - 1]) <= 5 * TOL_PSNR_DB
        assert abs(float(out[7]) - float(g[f"f{i}_bpp"])) <= 1e-3 * float(g[f"f{i}_bpp"])
    data = gop.clone()
    x_hat, loss, img_loss, be_loss, _, psnr, psnr_list, aux, aux2, _, _ = parallel_compression(None, model, data, False)
    assert x_hat.shape == (3, 3, 256, 256)
    drift = np.abs(np.array(psnr_list) - exp_psnr)
    # the closed-loop bound is anchored to the measured floor of the fp32-MFMA convs on the same
    # chain (the split-precision path must not drift more than twice what plain fp32 does)
    from fastvideocodec_amd import kernels as K
    with K.precision("f32"):
        psnr_f32 = parallel_compression(None, model, gop.clone(), False)[6]
    drift_f32 = np.abs(np.array(psnr_f32) - exp_psnr)
    print("closed-loop PSNR drift per frame (dB): x3", drift, "f32", drift_f32)
    assert drift[0] <= TOL_PSNR_DB, drift
    # the old fixed cap (2e-2 dB) stays as a ceiling on both drifts
    assert drift_f32.max() <= 2e-2, drift_f32
    assert drift.max() <= min(max(2 * drift_f32.max(), 1e-4), 2e-2), (drift, drift_f32)
    exp_bpp = np.mean([float(g[f"f{i}_bpp"]) for i in range(1, 4)])
    assert abs(be_loss - exp_bpp) <= 1e-2 * exp_bpp


@pytest.mark.parametrize("case", ["64x64", "128x192", "256x256", "chain2", "chain3"])
def test_decode_from_golden_symbols(model, dev, case):
    """T3 on identical decisions: the reference's own quantised latents, entropy-coded by the
    device rANS and decoded by the HIP decoder, reconstruct the reference's frame within 1e-4 dB."""
    from fastvideocodec_amd import kernels as K
    if case.startswith("chain"):
        i = int(case[-1])
        g = np.load(os.path.join(GOLD, "dvc_chain_256x256.npz"))
        cur, ref = g["gop"][i:i + 1], g[f"f{i-1}_clipped"]
        qmv, qz, qf, clipped = g[f"f{i}_quant_mv"], g[f"f{i}_compressed_z"], g[f"f{i}_compressed_feature"], g[f"f{i}_clipped"]
    else:
        g = np.load(os.path.join(GOLD, f"dvc_{case}.npz"))
        cur, ref = g["input_image"], g["referframe"]
        qmv, qz, qf, clipped = g["quant_mv"], g["compressed_z"], g["compressed_feature"], g["clipped"]
    to_nhwc = lambda a: K.nchw_to_nhwc(torch.from_numpy(np.ascontiguousarray(a)).to(dev))
    sigma = model.respriorDecoder.run(to_nhwc(qz))
    bs = model.compress_tensors({"mvfeature": to_nhwc(qmv), "z": to_nhwc(qz), "feature": to_nhwc(qf), "sigma": sigma})
    rec = model.decompress(bs, torch.from_numpy(np.ascontiguousarray(ref)).to(dev)).cpu().numpy()
    assert np.abs(rec - clipped).max() <= 1e-4
    p_got = 10 * np.log10(1 / np.mean((rec.astype(np.float64) - cur) ** 2))
    p_exp = 10 * np.log10(1 / np.mean((clipped.astype(np.float64) - cur) ** 2))
    assert abs(p_got - p_exp) <= TOL_PSNR_DB


def test_compress_decompress_bitexact(model, dev):
    g = np.load(os.path.join(GOLD, "dvc_128x192.npz"))
    cur = torch.from_numpy(g["input_image"]).to(dev)
    ref = torch.from_numpy(g["referframe"]).to(dev)
    bs, rec_enc = model.compress(cur, ref)
    rec_dec = model.decompress(bs, ref)
    torch.cuda.synchronize()
    assert torch.equal(rec_enc, rec_dec)
    assert bs.nbytes() > 0
    # forward's clipped recon is the same tensor the encoder reconstructs
    out = model(cur, ref)
    assert torch.equal(out[0], rec_enc)


def test_compress_deterministic_and_portable(model, dev):
    """Determinism check (SURVEY §5 race detection): encoding the same frame twice gives the same
    bytes, and a separately constructed decoder instance reproduces the encoder's recon."""
    g = np.load(os.path.join(GOLD, "dvc_128x192.npz"))
    cur = torch.from_numpy(g["input_image"]).to(dev)
    ref = torch.from_numpy(g["referframe"]).to(dev)
    bs1, rec1 = model.compress(cur, ref)
    bs2, rec2 = model.compress(cur, ref)
    torch.cuda.synchronize()
    assert torch.equal(rec1, rec2)
    for part in ("z", "mv", "feature"):
        assert getattr(bs1, part).to_bytes_list() == getattr(bs2, part).to_bytes_list(), part
    other = get_codec_model("DVC-pretrained", compression_level=2, device=dev)
    rec_dec = other.decompress(bs1, ref)
    torch.cuda.synchronize()
    assert torch.equal(rec_dec, rec1)


def test_compress_streams_vs_oracle_coder(model, dev):
    """Device bitstream == C oracle coder fed the same symbols/indexes/tables."""
    from oracle import coder_ref as R
    from fastvideocodec_amd import kernels as K
    g = np.load(os.path.join(GOLD, "dvc_64x64.npz"))
    cur = torch.from_numpy(g["input_image"]).to(dev)
    ref = torch.from_numpy(g["referframe"]).to(dev)
    with torch.no_grad():
        t = model._encode_graph(cur, ref)
    bs = model.compress_tensors(t)
    tz, tmv, tf = model._coders["tables"]
    sym_f = K.latent_to_symbols(t["feature"], 96).cpu().numpy().reshape(96, -1)
    idx_f = K.build_indexes(t["sigma"], model._coders["scale_table"], 96).cpu().numpy().reshape(96, -1)
    strings = bs.feature.to_bytes_list()
    for c in range(96):
        assert strings[c] == R.CRef.encode(sym_f[c], idx_f[c], tf.cdf, tf.cdf_length, tf.offset)
    sym_mv = K.latent_to_symbols(t["mvfeature"], 128).cpu().numpy().reshape(128, -1)
    strings = bs.mv.to_bytes_list()
    for c in range(128):
        idx = np.full(sym_mv.shape[1], c, np.int32)
        assert strings[c] == R.CRef.encode(sym_mv[c], idx, tmv.cdf, tmv.cdf_length, tmv.offset)


def test_calrealbits(model, dev):
    g = np.load(os.path.join(GOLD, "dvc_64x64.npz"))
    cur = torch.from_numpy(g["input_image"]).to(dev)
    ref = torch.from_numpy(g["referframe"]).to(dev)
    est = model(cur, ref)
    model.calrealbits = True
    try:
        real = model(cur, ref)
    finally:
        model.calrealbits = False
    # torchac-compatible real bits (tests/test_gpu_torchac.py pins them): near the estimate
    assert float(real[7]) > 0.5 * float(est[7])
    assert torch.equal(real[0], est[0])


def test_batch_matches_single(model, dev):
    g = np.load(os.path.join(GOLD, "dvc_64x64.npz"))
    cur = torch.from_numpy(g["input_image"]).to(dev)
    ref = torch.from_numpy(g["referframe"]).to(dev)
    one = model(cur, ref)[0]
    two = model(torch.cat([cur, cur]), torch.cat([ref, ref]))[0]
    assert torch.equal(two[0:1], one) and torch.equal(two[1:2], one)


def test_fused_upsample_add_leaves_forward_bitexact(model, dev, monkeypatch):
    """Warp_net's upsample-adds formed inside ResBlock conv1 (fvc_conv2d_nhwc_wino_up, the default)
    against the standalone upsample-add kernel then conv1 (FVC_UP_FUSE=0): the whole 8-tuple of
    VideoCompressor.forward (net.py:70-220) and the prediction are bit-identical, at 256x256 and at
    192x320 x 2 frames (the quarter-resolution ResBlocks' 80 columns cut a column group; several
    schedule chunks per column)."""
    g = np.load(os.path.join(GOLD, "dvc_256x256.npz"))
    pairs = [(torch.from_numpy(g["input_image"]).to(dev), torch.from_numpy(g["referframe"]).to(dev))]
    gen = torch.Generator().manual_seed(17)
    pairs.append((torch.rand(2, 3, 192, 320, generator=gen).to(dev), torch.rand(2, 3, 192, 320, generator=gen).to(dev)))
    for cur, ref in pairs:
        monkeypatch.setenv("FVC_UP_FUSE", "1")
        a, ta = model(cur, ref, return_intermediates=True)
        monkeypatch.setenv("FVC_UP_FUSE", "0")
        b, tb = model(cur, ref, return_intermediates=True)
        monkeypatch.delenv("FVC_UP_FUSE")
        torch.cuda.synchronize()
        for x, y in zip(a, b):
            assert torch.equal(torch.as_tensor(x), torch.as_tensor(y))
        assert torch.equal(ta["prediction"], tb["prediction"])


def test_rejects_bad_sizes(model, dev):
    x = torch.rand(1, 3, 100, 64, device=dev)
    with pytest.raises(ValueError):
        model(x, x)


def test_gop_pipeline_bitexact(model, dev):
    """Three-stream encode/code/decode pipeline: decoder recon == encoder recon for every frame,
    and the pipelined bitstreams equal a serial (single-stream) run."""
    from fastvideocodec_amd.gop import encode_decode_gop
    from fastvideocodec_amd.synthetic import make_gop
    frames = torch.from_numpy(np.stack([make_gop(128, 192, 4, 7 + g) for g in range(2)])).to(dev)
    bss, dec, sses, enc = encode_decode_gop(model, frames, check=True, overlap=True)
    bss2, dec2, _, enc2 = encode_decode_gop(model, frames, check=True, overlap=False)
    torch.cuda.synchronize()
    for a, b, c, d in zip(dec, enc, dec2, enc2):
        assert torch.equal(a, b) and torch.equal(a, c) and torch.equal(b, d)
    for a, b in zip(bss, bss2):
        assert a.feature.to_bytes_list() == b.feature.to_bytes_list()
        assert a.mv.to_bytes_list() == b.mv.to_bytes_list()


def _parity_1080p_report(model, dev, cur, ref, inter, o_mse, o_bpp):
    """Symbol flip rates per latent, stage deviations, dPSNR and bpp deviation of one HIP forward
    against the oracle's intermediates."""
    out, t = model(cur.to(dev), ref.to(dev), return_intermediates=True)
    torch.cuda.synchronize()
    report = {}
    nflip = ntot = 0
    for name, gname in (("mvfeature", "quant_mv"), ("feature", "compressed_feature"), ("z", "compressed_z")):
        got = np.round(nhwc_to_nchw(t[name], STAGES[name]).numpy())
        d = got != inter[gname].numpy()
        report[gname] = float(d.mean())
        nflip += int(d.sum())
        ntot += d.size
    report["flip_rate_all"] = nflip / ntot
    report["flips"] = nflip
    for name in ("estmv", "warpframe", "prediction"):
        got = nhwc_to_nchw(t[name], STAGES[name]).numpy()
        exp = inter[name].numpy()
        d = np.abs(got - exp) / (np.abs(exp).max() + 1e-6)
        report[name] = float(d.max())
        report[name + "_mean"] = float(d.mean())
    psnr_got = 10 * np.log10(1.0 / float(out[1]))
    psnr_exp = 10 * np.log10(1.0 / float(o_mse))
    report["dpsnr_db"] = abs(psnr_got - psnr_exp)
    report["bpp_rel"] = abs(float(out[7]) - float(o_bpp)) / float(o_bpp)
    return report


@pytest.fixture(scope="module")
def oracle_1080p():
    from fastvideocodec_amd.synthetic import make_gop, gop_seed
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    frames = make_gop(1080, 1920, 2, gop_seed(7))
    cur, ref = torch.from_numpy(frames[1:2].copy()), torch.from_numpy(frames[0:1].copy())
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    (o_clip, o_mse, _, _, o_bf, o_bz, o_bmv, o_bpp), inter = dvc_ref.forward(
        seeded_torch_state_dict(), cur, ref, return_intermediates=True)
    return cur, ref, inter, o_mse, o_bpp


# T3 at BASELINE's full size: the reference itself flips 3 mv / 24 feature / 2 z of
# 1.86 M symbols between two CPU backends (aggregate 1.56e-5); the HIP path must stay inside that
# and inside the north star's 1e-4 dB. Per-latent bounds sit ~3x above the measured rates (r1, MI355X:
# mv 1.7e-5, feature 1.3e-6, z 0), so a regression to fp16-level accuracy (flip rates ~1e-3) fails.
TOL_1080P_FLIPS_ALL = 1.56e-5
TOL_1080P_FLIPS = {"quant_mv": 5e-5, "compressed_feature": 5e-6, "compressed_z": 3.1e-5}
TOL_1080P_MAX = {"estmv": 1e-4, "warpframe": 3e-3, "prediction": 1e-3}


def test_forward_vs_oracle_1080p(model, dev, oracle_1080p):
    """BASELINE.json's full size (1920x1080, replicate-padded to 1088): one synthetic P-frame
    through the HIP forward (default split-precision convs) and through the CPU oracle
    (golden-pinned restatement of net.py:70-220) with the same weights."""
    cur, ref, inter, o_mse, o_bpp = oracle_1080p
    report = _parity_1080p_report(model, dev, cur, ref, inter, o_mse, o_bpp)
    print("1080p parity (x3):", report)
    assert report["flip_rate_all"] <= TOL_1080P_FLIPS_ALL, report
    for gname, tol in TOL_1080P_FLIPS.items():
        assert report[gname] <= tol, (gname, report)
    for name in ("estmv", "warpframe", "prediction"):
        # mean deviation at the small-size tier; the max is a few isolated pixels where SpyNet's
        # warp-and-refine iterations amplify ulp-level differences (the reference itself moves
        # there between CPU backends) or a flipped MV symbol moves the warp: bounds
        # ~3x the measured maxima (r2, MI355X: estmv 2.9e-5, warpframe 1.0e-3, prediction 2.8e-4)
        assert report[name + "_mean"] <= 2e-6, report
        assert report[name] <= TOL_1080P_MAX[name], report
    assert report["dpsnr_db"] <= TOL_PSNR_DB, report
    assert report["bpp_rel"] <= 1e-5, report


def test_forward_x3_vs_f32_1080p(model, dev, oracle_1080p):
    """The split-precision convs add no symbol flips beyond fp32 noise: the same 1080p frame run
    on the fp32-MFMA kernels flips about as many symbols against the oracle as the x3 path."""
    from fastvideocodec_amd import kernels as K
    cur, ref, inter, o_mse, o_bpp = oracle_1080p
    r3 = _parity_1080p_report(model, dev, cur, ref, inter, o_mse, o_bpp)
    with K.precision("f32"):
        r32 = _parity_1080p_report(model, dev, cur, ref, inter, o_mse, o_bpp)
    print("1080p flips x3:", r3["flips"], "f32:", r32["flips"], r32)
    assert r32["dpsnr_db"] <= TOL_PSNR_DB
    assert r3["flips"] <= 2 * r32["flips"] + 10, (r3, r32)


def test_gop_streaming_back_to_back(model, dev):
    """join=False (bench.py's timed loop): three GOPs enqueued back to back, each next GOP's
    encoder overlapping the previous GOP's coder/decoder tail. Every GOP must still decode to its
    encoder's recon bit-for-bit and equal a joined run (no allocator reuse across streams)."""
    from fastvideocodec_amd.gop import encode_decode_gop
    from fastvideocodec_amd.synthetic import make_gop
    gops = [torch.from_numpy(np.stack([make_gop(128, 192, 5, 40 + g)])).to(dev) for g in range(3)]
    ref = [encode_decode_gop(model, f, overlap=True, join=True) for f in gops]
    torch.cuda.synchronize()
    ref = [([b.feature.to_bytes_list() for b in r[0]], [d.clone() for d in r[1]]) for r in ref]
    outs = [encode_decode_gop(model, f, overlap=True, join=False) for f in gops]
    torch.cuda.synchronize()
    for (bss, dec, _, enc), (rb, rd) in zip(outs, ref):
        for a, b in zip(dec, enc):
            assert torch.equal(a, b)
        for a, b in zip(dec, rd):
            assert torch.equal(a, b)
        assert [b.feature.to_bytes_list() for b in bss] == rb


def test_4k_pframe_compress_decompress(model, dev):
    """BASELINE configs[3] frame size (3840x2160, replicate-padded to 3840x2176): one P-frame
    encodes, decodes bit-exactly to the encoder's recon, stays inside the split-precision range,
    and its bits-estimate bpp is close to the real bitstream's."""
    from fastvideocodec_amd import kernels as K
    from fastvideocodec_amd.synthetic import make_gop, gop_seed
    frames = torch.from_numpy(make_gop(2160, 3840, 2, gop_seed(3))).to(dev)
    assert frames.shape[-2:] == (2176, 3840)
    K.x3_overflow(reset=True)
    bs, rec_enc = model.compress(frames[1:2], frames[0:1])
    rec_dec = model.decompress(bs, frames[0:1])
    out = model(frames[1:2], frames[0:1])
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    assert torch.equal(rec_enc, rec_dec)
    assert torch.equal(out[0], rec_enc)
    real_bpp = bs.nbytes() * 8 / (2176 * 3840)
    assert abs(real_bpp - float(out[7])) <= 0.02 * float(out[7]) + 1e-3, (real_bpp, float(out[7]))


def test_gop12_1080p_closed_loop_vs_reference(model, dev):
    """BASELINE configs[2]'s closed loop at its own size: one 1920x1080 GOP-12
    (GOP id 0, padded to 1088) through the reference's DVC-pretrained loop, models.py:368-383
    (frame 0 passed through as the I-frame; every P-frame coded against the previous
    reconstruction), on the HIP path, against the reference's own per-frame PSNR / bpp of the same
    chain (tests/golden/ref_fullsize_parity.json from gen_fullsize_parity.py: the reference itself,
    default oneDNN backend). The bounds come from the reference's own closed-loop cross-backend
    drift on this GOP -- five chains: ATen native convs, channels-last oneDNN, float64, oneDNN on 4
    and on 1 thread -- which with untrained weights is chaotic (1e3 symbols differ at frame 2, 5e5 of
    1.86e6 by frame 11):
    * frame 1 (same inputs: open loop): dPSNR <= max(the reference's frame-1 drift, 1e-4 dB), dbpp
      likewise (floor 1e-5);
    * frames 2..11, each: <= 2x the largest drift any reference chain reaches over the GOP;
    * frames 2..11, mean: <= 2x the largest mean drift of a reference chain.
    Why 2x: past frame 1 every chain (the HIP one included) is one more sample of the same chaotic
    divergence, and an implementation indistinguishable from the reference's own backends beats
    the maximum of 5 such samples only with probability 5/6, so a 1x bound is a coin with a 1-in-6
    false failure. r5 measured exactly that: the HIP chain's largest bpp drift was 1.03x the
    reference envelope (9.85e-4 vs 9.58e-4, channels-last) on the r5h box, with 3 chains in the
    fixture. The reference chains' own means span 4x (PSNR 7.3e-4 .. 2.9e-3 dB), so 2x the largest
    is inside the spread the reference shows, not a loosening beyond it. Measured r5 (MI355X):
    PSNR drift per frame 0, 2.8e-4 .. 4.6e-3 dB (mean 1.8e-3 against the reference means
    7.3e-4 .. 2.9e-3), bpp drift up to 9.9e-4 relative; scripts/gop12_drift.py.
    """
    import json
    from fastvideocodec_amd.synthetic import gop_seed, make_gop
    with open(os.path.join(GOLD, "ref_fullsize_parity.json")) as f:
        g = json.load(f)["p1080_gop12"]
    ref = g["chains"]["onednn8"]
    var = {k: c for k, c in g["chains"].items() if k != "onednn8"}
    frames = torch.from_numpy(make_gop(1080, 1920, 12, gop_seed(0))).to(dev)
    x_prev = frames[0:1]
    drift, dbpp = [], []
    for i in range(1, 12):
        out = model(frames[i:i + 1], x_prev)
        x_prev = out[0]
        r = ref[i - 1]
        assert r["frame"] == i
        drift.append(abs(float(10 * np.log10(1.0 / np.float64(float(out[1])))) - r["psnr_db"]))
        dbpp.append(abs(float(out[7]) - r["bpp"]) / r["bpp"])
    rp = {k: [c[j]["vs_onednn8"]["dpsnr_db"] for j in range(11)] for k, c in var.items()}
    rb = {k: [c[j]["vs_onednn8"]["dbpp_rel"] for j in range(11)] for k, c in var.items()}
    print("HIP dPSNR per frame:", " ".join(f"{x:.1e}" for x in drift))
    for k in rp:
        print(f"reference {k:6s}:", " ".join(f"{x:.1e}" for x in rp[k]))
    assert drift[0] <= max(max(v[0] for v in rp.values()), 1e-4), drift
    assert dbpp[0] <= max(max(v[0] for v in rb.values()), 1e-5), dbpp
    assert len(var) >= 5, sorted(var)
    assert max(drift[1:]) <= 2 * max(max(v[1:]) for v in rp.values()), drift
    assert max(dbpp[1:]) <= 2 * max(max(v[1:]) for v in rb.values()), dbpp
    assert np.mean(drift[1:]) <= 2 * max(np.mean(v[1:]) for v in rp.values()), drift
    assert np.mean(dbpp[1:]) <= 2 * max(np.mean(v[1:]) for v in rb.values()), dbpp
    # fixed ceilings, independent of the fixture: a regenerated fixture with a wider
    # reference spread cannot widen the gate past them (the committed fixture's 2x envelope is
    # 1.4e-2 dB and 1.9e-3 relative bpp, so they do not bind today)
    assert max(drift) <= 2e-2 and max(dbpp) <= 2e-3, (drift, dbpp)
