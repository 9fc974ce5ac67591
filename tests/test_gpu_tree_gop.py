"""LSVC tree GOP (models.py:683-728, 1347-1411 layer loop) driving the DVC codec on the GPU:
decoder == encoder bit-for-bit, and every frame of a layer batch equals coding it alone against
its parent's reconstruction (recon and bitstream bytes)."""
import numpy as np
import pytest
import torch

from fastvideocodec_amd.models import get_codec_model
from fastvideocodec_amd.synthetic import make_gop
from fastvideocodec_amd.tree_gop import coding_layers, encode_decode_tree_gop

pytestmark = pytest.mark.gpu
TREE_DRIFT_CAP_DB = 5e-3  # r2's fixed closed-loop cap


@pytest.fixture(scope="module")
def model(dev):
    return get_codec_model("DVC-pretrained", compression_level=2, device=dev)


@pytest.mark.parametrize("T", [7, 12])
def test_tree_gop_matches_per_frame_coding(model, dev, T):
    G = 2
    frames = torch.from_numpy(np.stack([make_gop(128, 192, T, 21 + g) for g in range(G)])).to(dev)
    bss, dec, sses, enc = encode_decode_tree_gop(model, frames, check=True)
    torch.cuda.synchronize()
    assert sorted(dec) == list(range(1, T))
    for t in dec:
        assert torch.equal(dec[t], enc[t]), t
    lay = coding_layers(T - 1)
    C = {"mv": 128, "z": 64, "feature": 96}
    for i, layer in enumerate(lay):
        parts = {k: getattr(bss[i], k).to_bytes_list() for k in C}
        for j, (t, p) in enumerate(layer):
            for g in range(G):
                ref = frames[g:g + 1, 0] if p == 0 else enc[p][g:g + 1]
                bs1, rec1 = model.compress(frames[g:g + 1, t], ref)
                assert torch.equal(rec1, enc[t][g:g + 1]), (t, g)
                b = j * G + g
                for k, c in C.items():
                    assert getattr(bs1, k).to_bytes_list() == parts[k][b * c:(b + 1) * c], (t, g, k)


def test_tree_gop_linear_equals_sequential_gop(model, dev):
    """isLinear (models.py 'default' graph) reduces the tree to the sequential DVC GOP."""
    from fastvideocodec_amd.gop import encode_decode_gop
    frames = torch.from_numpy(np.stack([make_gop(64, 128, 5, 33)])).to(dev)
    _, dec_t, _, enc_t = encode_decode_tree_gop(model, frames, isLinear=True)
    bss, dec, _, enc = encode_decode_gop(model, frames, overlap=False)
    torch.cuda.synchronize()
    for t in range(1, 5):
        assert torch.equal(enc_t[t], enc[t - 1]) and torch.equal(dec_t[t], dec[t - 1])


def test_tree_gop_vs_oracle(model, dev, seeded_sd):
    """The tree-coded frames against the CPU oracle (golden-pinned restatement of net.py:70-220),
    GOP-12 at 128x192 (layers [1, 8], [2, 5, 9], [3, 4, 6, 7, 10, 11]):
    * open loop, every frame: the oracle codes frame t against the device's reconstruction of its
      parent; symbols equal (flip rate <= 1e-3, 0 observed at these sizes) and, on identical
      symbols, the clipped recon within 4e-5 abs and PSNR within 1e-4 dB;
    * closed loop: the oracle runs the whole tree on its own reconstructions; the device's
      per-frame PSNR drift from it may not exceed twice the drift of the fp32-MFMA convs on the
      same tree (or 1e-4 dB): open-loop ulp differences compound down a tree path the way the
      reference's own cross-backend runs drift, so the bound is anchored to a plain
      fp32 implementation rather than to a constant (r3 measured 1.1e-3 dB at frame 10)."""
    from oracle import dvc_ref
    T = 12
    frames = torch.from_numpy(np.stack([make_gop(128, 192, T, 77)])).to(dev)
    _, dec, _, enc = encode_decode_tree_gop(model, frames, check=True)
    torch.cuda.synchronize()
    fr = frames[0].cpu()
    lay = coding_layers(T - 1)
    rec_o = {0: fr[0:1]}
    for layer in lay:
        for t, p in layer:
            cur = fr[t:t + 1]
            ref_dev = fr[0:1] if p == 0 else enc[p].cpu()
            (clip_o, mse_o, *_), inter = dvc_ref.forward(seeded_sd, cur, ref_dev, return_intermediates=True)
            _, t_dev = model(cur.to(dev), ref_dev.to(dev), return_intermediates=True)
            flips = 0
            for name, gname, c in (("mvfeature", "quant_mv", 128), ("feature", "compressed_feature", 96),
                                   ("z", "compressed_z", 64)):
                got = torch.round(t_dev[name][..., :c].permute(0, 3, 1, 2).cpu())
                flips += int((got != inter[gname]).sum())
            if flips == 0:
                # 2.0e-5 measured (r3, MI355X): a few isolated pixels of SpyNet's warp-and-refine path
                assert float((enc[t].cpu() - clip_o).abs().max()) <= 4e-5, t
                psnr_d = 10 * np.log10(1 / float(((enc[t].cpu() - cur) ** 2).mean()))
                psnr_o = 10 * np.log10(1 / float(((clip_o - cur) ** 2).mean()))
                assert abs(psnr_d - psnr_o) <= 1e-4, (t, psnr_d, psnr_o)
            assert flips <= 1e-3 * (128 * 8 * 12 + 96 * 8 * 12 + 64 * 2 * 3), (t, flips)
            # closed loop: the oracle's own tree
            rec_o[t] = dvc_ref.forward(seeded_sd, cur, rec_o[p])[0]
    # closed-loop drift bound anchored to the fp32-MFMA convs' own drift on the same tree
    from fastvideocodec_amd import kernels as K
    with K.precision("f32"):
        _, _, _, enc32 = encode_decode_tree_gop(model, frames, check=True)
        torch.cuda.synchronize()
    drift, drift32 = [], []
    for t in range(1, T):
        cur = fr[t:t + 1]
        po = 10 * np.log10(1 / float(((rec_o[t] - cur) ** 2).mean()))
        pd = 10 * np.log10(1 / float(((enc[t].cpu() - cur) ** 2).mean()))
        p32 = 10 * np.log10(1 / float(((enc32[t].cpu() - cur) ** 2).mean()))
        drift.append(abs(pd - po))
        drift32.append(abs(p32 - po))
    print("tree closed-loop PSNR drift (dB): x3", np.array(drift), "f32", np.array(drift32))
    # the anchored bound keeps the old fixed cap as a ceiling, and the fp32 drift itself
    # must stay under it (a kernel shared by both precisions cannot loosen the bound)
    assert max(drift32) <= TREE_DRIFT_CAP_DB, drift32
    assert max(drift) <= min(max(2 * max(drift32), 1e-4), TREE_DRIFT_CAP_DB), (drift, drift32)


def test_tree_gop_streaming_join_false(model, dev):
    """join=False (bench.py --tree's timed loop): two GOPs streamed back to back without a host
    wait equal the joined run; the overflow probes wait on the model for check_overflow."""
    from fastvideocodec_amd import gop
    gops = [torch.from_numpy(np.stack([make_gop(64, 128, 7, 50 + g)])).to(dev) for g in range(2)]
    ref = [encode_decode_tree_gop(model, f) for f in gops]
    torch.cuda.synchronize()
    ref = [({t: v.clone() for t, v in r[1].items()}, [b.feature.to_bytes_list() for b in r[0]]) for r in ref]
    model._overflow_probes = []
    outs = [encode_decode_tree_gop(model, f, join=False) for f in gops]
    assert len(model._overflow_probes) == 2 * len(coding_layers(6))
    torch.cuda.synchronize()
    assert gop.check_overflow(model) is False
    for (bss, dec, _, enc), (rd, rb) in zip(outs, ref):
        for t in dec:
            assert torch.equal(dec[t], enc[t]) and torch.equal(dec[t], rd[t])
        assert [b.feature.to_bytes_list() for b in bss] == rb
