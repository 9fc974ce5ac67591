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


def test_chain_vs_oracle_and_strings(model, sd):
    rng = np.random.default_rng(4)
    H = W = 128
    f = [torch.from_numpy(rng.random((1, 3, H, W), np.float32))]
    for t in range(2):
        f.append(torch.clamp(f[-1] + 0.05 * torch.from_numpy(rng.standard_normal((1, 3, H, W)).astype(np.float32)), 0, 1))
    hid_o = R.init_hidden(H, W)
    hid_d = model.init_hidden(H, W, DEV)
    prev_o = prev_d = f[0]
    pri_o = (None, None)
    pri_d = (None, None)
    for t in range(1, 3):
        rpm_flag = t > 1
        with torch.no_grad():
            o = R.forward(sd, prev_o, f[t], hid_o, rpm_flag, *pri_o)
        out = model(prev_d.to(DEV), f[t].to(DEV), hid_d, rpm_flag, *pri_d)
        Y1, hid_d, bpp_est, img_loss, aux, bpp_act, psnr, mvp, resp = out
        # latent symbols: the device and the oracle round the same values (flips only at .5 ties)
        for name, lat in (("mv_codec", mvp), ("res_codec", resp)):
            sym_d = torch.round(_nchw(lat))
            sym_o = o[name]["prior_latent"]
            flips = int((sym_d != sym_o).sum())
            assert flips <= max(1, sym_o.numel() // 2000), (t, name, flips)
        if all(int((torch.round(_nchw(l)) != o[n]["prior_latent"]).sum()) == 0
               for n, l in (("mv_codec", mvp), ("res_codec", resp))):
            np.testing.assert_allclose(Y1.cpu().numpy(), o["Y1_com"].numpy(), atol=TOL * 10)
            assert abs(float(bpp_est) - float(o["bpp_est"])) <= 1e-3 * float(o["bpp_est"]) + 1e-4
        assert float(bpp_act) > 0 and np.isfinite(float(psnr))
        # the frame's strings decode to the coded latents (decoder = same RPM state)
        for codec, strings in zip((model.mv_codec, model.res_codec), model.last_strings):
            eb = codec.entropy_bottleneck
            lat_hat_d = None
            B, h4, w4 = 1, H // 16, W // 16
            dec = eb.decompress(strings, (h4, w4))
            if rpm_flag:
                ref = torch.round(K.nhwc_to_nchw(mvp if codec is model.mv_codec else resp, 128) -
                                  K.nhwc_to_nchw(eb.mu, 128)) + K.nhwc_to_nchw(eb.mu, 128)
            else:
                _, med = eb.entropy_bottleneck.kernel_params()
                lat = K.nhwc_to_nchw(mvp if codec is model.mv_codec else resp, 128)
                ref = torch.round(lat - med.view(1, -1, 1, 1)) + med.view(1, -1, 1, 1)
            assert torch.allclose(K.nhwc_to_nchw(dec, 128), ref, atol=1e-5), (t, lat_hat_d)
        hid_o = o["hidden"]
        pri_o = (o["mv_prior_latent"], o["res_prior_latent"])
        pri_d = (mvp, resp)
        prev_o, prev_d = o["Y1_com"], Y1.cpu()


def test_hidden_layout_roundtrip(model):
    hid = model.init_hidden(128, 192, DEV)
    g = torch.Generator().manual_seed(1)
    ref = tuple(torch.randn(t.shape, generator=g) for t in rlvc.hidden_to_reference(hid))
    back = rlvc.hidden_to_reference(rlvc.hidden_from_reference(ref, DEV))
    for a, b in zip(ref, back):
        assert torch.equal(a, b.cpu())
