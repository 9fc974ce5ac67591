"""RLVC path on the GPU against the CPU oracle (oracle/rlvc_ref.py, whose
ConvLSTM / RPM are pinned to the reference's own outputs): recurrent modules vs the golden
fixture, a 3-frame chain (first P-frame on the EntropyBottleneck, then RPM), real strings that
decode to the coded latents, and the reference's hidden-state layout."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rlvc_ref as R  # noqa: E402

from fastvideocodec_amd import kernels as K  # noqa: E402
from fastvideocodec_amd import rlvc  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
GOLD = os.path.join(ROOT, "tests", "golden", "rlvc_rpm.npz")
# tolerance of a split-precision conv stack vs fp32 CPU (tests/test_gpu_forward.py: ~1e-6 rel
# per conv); the latents' rounding is the discontinuity, checked separately as flips
TOL = 2e-4
# Y1_com of the device vs the oracle's synthesis on the same quantised latents (open loop)
TOL_Y1 = 1e-4


@pytest.fixture(scope="module")
def model():
    return rlvc.get_rlvc_model(device=DEV)


@pytest.fixture(scope="module")
def sd():
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in rlvc.seeded_state_dict().items()}


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous().to(DEV)


def _nchw(t):
    return t.permute(0, 3, 1, 2).contiguous().cpu()


def test_recurrent_modules_vs_reference(model):
    g = np.load(GOLD)
    C = 128
    lstm = model.mv_codec.enc_lstm
    st = torch.from_numpy(g["lstm_state"])
    with torch.no_grad():
        h, state = lstm.run(_nhwc(torch.from_numpy(g["lstm_x"])), {"c": _nhwc(st[:, :C]), "h": _nhwc(st[:, C:])})
    np.testing.assert_allclose(_nchw(h).numpy(), g["lstm_h"], rtol=TOL, atol=TOL)
    np.testing.assert_allclose(_nchw(state["c"]).numpy(), g["lstm_state_out"][:, :C], rtol=TOL, atol=TOL)
    rpm = model.mv_codec.entropy_bottleneck.RPM
    hid = torch.from_numpy(g["rpm_hidden"])
    with torch.no_grad():
        s, mu, hid2 = rpm.run(_nhwc(torch.from_numpy(g["rpm_prior"])), {"c": _nhwc(hid[:, :C]), "h": _nhwc(hid[:, C:])})
    np.testing.assert_allclose(_nchw(s).numpy(), g["rpm_sigma"], rtol=TOL, atol=TOL)
    np.testing.assert_allclose(_nchw(mu).numpy(), g["rpm_mu"], rtol=TOL, atol=TOL)
    np.testing.assert_allclose(_nchw(hid2["h"]).numpy(), g["rpm_hidden_out"][:, C:], rtol=TOL, atol=TOL)


def _strings_vs_c_coder(eb, lat, rpm_flag, strings):
    """T1 for one codec's frame: the device strings (compressai framing, one per item, (C,H,W)
    order) equal the C oracle coder (and the pure-Python coder) on the same symbols, indexes
    and tables."""
    sys.path.insert(0, ROOT)
    from oracle import coder_ref as CR
    x = K.nhwc_to_nchw(lat, 128).cpu()
    if rpm_flag:
        gc = eb.gaussian_conditional
        mu = K.nhwc_to_nchw(eb.mu, 128).cpu()
        sym = torch.round(x - mu).to(torch.int32).numpy()
        sig = K.nhwc_to_nchw(eb.sigma, 128).cpu().numpy()
        idx = CR.build_indexes(sig.reshape(sig.shape[0], -1), gc._table_dev.cpu().numpy()).reshape(sym.shape)
        tabs = gc
    else:
        tabs = eb.entropy_bottleneck
        med = tabs.quantiles[:, 0, 1].detach().cpu().view(1, -1, 1, 1)
        sym = torch.round(x - med).to(torch.int32).numpy()
        idx = np.broadcast_to(np.arange(128, dtype=np.int32)[None, :, None, None], sym.shape)
    cdf, ln, off = (t.cpu().numpy() for t in (tabs._quantized_cdf, tabs._cdf_length, tabs._offset))
    assert len(strings) == sym.shape[0]
    for i, st in enumerate(strings):
        assert st == CR.CRef.encode(sym[i].ravel(), np.ascontiguousarray(idx[i]).ravel(), cdf, ln, off)
        assert st == CR.rans_encode_py(sym[i].ravel(), np.ascontiguousarray(idx[i]).ravel(), cdf, ln, off)
    return sym


def test_chain_vs_oracle_and_strings(model, sd):
    """A 3-frame RLVC chain (frame 1 on the EntropyBottleneck, frame 2 on RPM), each frame checked
    open loop against the oracle fed the device's own previous recon, hidden states and priors:
    * encoder: latent symbols equal up to rounding-tie flips;
    * decoder, unconditionally: the oracle's synthesis (Coder2D decode half + MC) run on the
      DEVICE's quantised latents reconstructs the device's Y1_com;
    * img_loss / PSNR of the clipped Y1_com (models.py:1033-1034) and aux_loss (models.py:1030);
    * every string byte-equal to the C and pure-Python coders (T1), and decodable."""
    rng = np.random.default_rng(4)
    H = W = 128
    f = [torch.from_numpy(rng.random((1, 3, H, W), np.float32))]
    for t in range(2):
        f.append(torch.clamp(f[-1] + 0.05 * torch.from_numpy(rng.standard_normal((1, 3, H, W)).astype(np.float32)), 0, 1))
    hid_d = model.init_hidden(H, W, DEV)
    prev = f[0]
    pri_d = (None, None)
    measured = []
    for t in range(1, 3):
        rpm_flag = t > 1
        hid_ref = rlvc.hidden_to_reference(hid_d)
        pri_ref = tuple(None if p is None else torch.round(_nchw(p)) for p in pri_d)
        with torch.no_grad():
            o = R.forward(sd, prev, f[t], tuple(h.cpu() for h in hid_ref), rpm_flag, *pri_ref)
        out = model(prev.to(DEV), f[t].to(DEV), hid_d, rpm_flag, *pri_d)
        Y1, hid_new, bpp_est, img_loss, aux, bpp_act, psnr, mvp, resp = out
        assert model.last_precision == "x3"
        # encoder: the device and the oracle round the same values (flips only at .5 ties)
        lat_hat = {}
        for (name, lat), codec, strings in zip((("mv_codec", mvp), ("res_codec", resp)),
                                               (model.mv_codec, model.res_codec), model.last_strings):
            eb = codec.entropy_bottleneck
            flips = int((torch.round(_nchw(lat)) != o[name]["prior_latent"]).sum())
            assert flips <= max(1, o[name]["prior_latent"].numel() // 2000), (t, name, flips)
            sym = _strings_vs_c_coder(eb, lat, rpm_flag, strings)
            m = (K.nhwc_to_nchw(eb.mu, 128).cpu() if rpm_flag
                 else eb.entropy_bottleneck.quantiles[:, 0, 1].detach().cpu().view(1, -1, 1, 1))
            lat_hat[name] = torch.from_numpy(sym).float() + m   # round(x - m) + m, the decoder's latent
            dec = eb.decompress(strings, (H // 16, W // 16))
            assert torch.equal(K.nhwc_to_nchw(dec, 128).cpu(), lat_hat[name]), (t, name)
        # decoder, open loop on the device's latents, from the device's decoder states
        C = 128
        with torch.no_grad():
            mv_hat, _ = R.coder2d_decode(sd, "mv_codec", lat_hat["mv_codec"], hid_ref[0][:, 2 * C:].cpu(), 1)
            Y1_MC, _ = R.D.motion_compensation(sd, prev, mv_hat)
            res_hat, _ = R.coder2d_decode(sd, "res_codec", lat_hat["res_codec"], hid_ref[1][:, 2 * C:].cpu(), 2)
            Y1_o = torch.clip(res_hat + Y1_MC, 0, 1)
        dev_y1 = float((Y1.cpu() - Y1_o).abs().max())
        measured.append(dev_y1)
        assert dev_y1 <= TOL_Y1, (t, dev_y1)
        # losses of the clipped recon
        il = float(torch.mean((f[t].double() - Y1.cpu().double()) ** 2))
        assert abs(float(img_loss) - il) <= 1e-6 * il, (float(img_loss), il)
        assert abs(float(psnr) - 10 * np.log10(1 / il)) <= 1e-4
        assert abs(float(aux) - float(o["aux_loss"])) <= 1e-5 * abs(float(o["aux_loss"])) + 1e-6, (float(aux), float(o["aux_loss"]))
        assert abs(float(bpp_est) - float(o["bpp_est"])) <= 1e-3 * float(o["bpp_est"]) + 1e-4
        assert float(bpp_act) > 0
        hid_d, pri_d, prev = hid_new, (mvp, resp), Y1.cpu()
    print("RLVC open-loop decoder max |Y1 - oracle|:", measured)


def test_overflow_recompute(model):
    """An activation past the split-precision range (a 1e7 gain on Warp_net's last ResBlock's
    first conv, whose output the next x3 conv stages) is caught by the stream's overflow flag and
    the frame is recomputed on the fp32 kernels."""
    H = W = 64
    rng = np.random.default_rng(9)
    f0, f1 = (torch.from_numpy(rng.random((1, 3, H, W), np.float32)).to(DEV) for _ in range(2))
    conv = model.warpnet.conv5.conv1
    w0, b0 = conv.weight.data.clone(), conv.bias.data.clone()
    try:
        conv.weight.data.mul_(1e7)
        conv.bias.data.mul_(1e7)
        conv.invalidate()
        before = getattr(model, "overflow_events", 0)
        model(f0, f1, model.init_hidden(H, W, DEV), False, None, None)
        assert model.last_precision == "f32" and model.overflow_events == before + 1
    finally:
        conv.weight.data.copy_(w0)
        conv.bias.data.copy_(b0)
        conv.invalidate()
    model(f0, f1, model.init_hidden(H, W, DEV), False, None, None)
    assert model.last_precision == "x3"


def test_hidden_layout_roundtrip(model):
    hid = model.init_hidden(128, 192, DEV)
    g = torch.Generator().manual_seed(1)
    ref = tuple(torch.randn(t.shape, generator=g) for t in rlvc.hidden_to_reference(hid))
    back = rlvc.hidden_to_reference(rlvc.hidden_from_reference(ref, DEV))
    for a, b in zip(ref, back):
        assert torch.equal(a, b.cpu())
