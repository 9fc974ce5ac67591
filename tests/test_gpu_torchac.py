"""Device side of the torchac-compatible coder: CDF normalisation, DVC's Laplace / BitEstimator
rows and symbol bounds on the GPU, end-to-end byte strings against the restated torchac algorithm
(oracle/torchac_ref.py; torchac itself is absent: parity unpinned against it), round trips, and
DVC's calrealbits forward (net.py:121-205)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import torchac_ref as T  # noqa: E402

from fastvideocodec_amd import torchac as TAC  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def test_float_cdf_api_bytes_equal_oracle():
    rng = np.random.default_rng(11)
    N, Lp = 3000, 300
    p = rng.random((N, Lp - 1)) ** 6 + 1e-9
    cdf = np.concatenate([np.zeros((N, 1)), np.cumsum(p, 1) / p.sum(1, keepdims=True)], 1)
    cdf = np.minimum(cdf, 1).astype(np.float32).reshape(2, 30, 50, Lp)
    sym = np.array([rng.choice(Lp - 1, p=q / q.sum()) for q in p], np.int16).reshape(2, 30, 50)
    cdf_d, sym_d = torch.from_numpy(cdf).to(DEV), torch.from_numpy(sym).to(DEV)
    # normalisation is exact float32 arithmetic: identical to the oracle's int16 rows
    rows = TAC._normalize(cdf_d, True).cpu().numpy().view(np.uint16)
    assert np.array_equal(rows, T.normalize(cdf))
    data = TAC.encode_float_cdf(cdf_d, sym_d, check_input_bounds=True)
    assert data == T.encode_float_cdf(cdf, sym, check_input_bounds=True)
    assert torch.equal(TAC.decode_float_cdf(cdf_d, data).cpu(), torch.from_numpy(sym))
    with pytest.raises(ValueError):
        TAC.encode_float_cdf(cdf_d, torch.full_like(sym_d, Lp - 1), check_input_bounds=True)


def _nhwc(a, cp):
    B, C, H, W = a.shape
    out = np.zeros((B, H, W, cp), np.float32)
    out[..., :C] = a.transpose(0, 2, 3, 1)
    return torch.from_numpy(out).to(DEV)


def test_laplace_feature_stream():
    rng = np.random.default_rng(5)
    B, C, H, W, cp = 2, 96, 9, 13, 96
    sigma = np.exp(rng.uniform(np.log(0.05), np.log(40), (B, C, H, W))).astype(np.float32)
    x = np.clip(rng.laplace(0, sigma), -140, 140).astype(np.float32)
    xd, sd = _nhwc(x, cp), _nhwc(sigma, cp)
    data = TAC.laplace_encode(xd, sd, C)
    # device rows vs the oracle's float32 Laplace rows: expm1f / the division may differ by an
    # ulp between the device and numpy, moving a rounded int16 entry by 1 (measured: 1.4e-4 of
    # the entries; torch's own CUDA vs CPU Laplace.cdf differ the same way)
    Lp = 300
    rows_dev = torch.empty((B * C * H * W, Lp), dtype=torch.int16, device=DEV)
    from fastvideocodec_amd import _lib, kernels as K
    _lib.call("fvc_torchac_laplace_rows", sd.data_ptr(), B, H, W, C, cp, 150, rows_dev.data_ptr(), K.stream_handle())
    rows_dev = rows_dev.cpu().numpy().view(np.uint16)
    rows_ref = T.normalize(T.laplace_cdf_rows(sigma.reshape(-1)))
    diff = rows_dev.astype(np.int64) - rows_ref
    assert np.abs(diff).max() <= 1 and np.count_nonzero(diff) <= 5e-4 * diff.size
    sym = (np.rint(x) + 150).astype(np.int64).reshape(-1)
    if np.count_nonzero(diff) == 0:
        assert data == T.encode_int16_normalized_cdf(rows_ref, sym)
    # the device bounds are the rows' entries: coding with the device rows in the oracle gives
    # the same bytes, and the decoder returns the symbols
    assert data == T.encode_int16_normalized_cdf(rows_dev, sym)
    back = TAC.laplace_decode(sd, C, data)
    assert torch.equal(back[..., :C].cpu(), torch.from_numpy(np.rint(x).transpose(0, 2, 3, 1)))
    # size: within 1 % (+ a few bytes) of the ideal code length under the same quantised rows
    r = rows_dev.astype(np.int64)
    lo = r[np.arange(len(sym)), sym]
    hi = np.where(sym == Lp - 2, 65536, r[np.arange(len(sym)), np.minimum(sym + 1, Lp - 1)])
    ideal = float(np.sum(-np.log2((hi - lo) / 65536.0))) / 8
    assert ideal <= len(data) <= 1.01 * ideal + 8
    with pytest.raises(ValueError):
        TAC.laplace_encode(_nhwc(np.full_like(x, 149.0), cp), sd, C)


def test_bitest_streams(model):
    bz, bmv = model._be_params()
    rng = np.random.default_rng(8)
    for params, C, shape in ((bz, 64, (2, 3, 5)), (bmv, 128, (2, 7, 6))):
        B, H, W = shape
        x = np.rint(rng.laplace(0, 3, (B, C, H, W))).astype(np.float32)
        xd = _nhwc(x, C)
        data = TAC.bitest_encode(xd, params, C)
        back = TAC.bitest_decode(params, (B, H, W, C), C, data)
        assert torch.equal(back.cpu(), xd.cpu())


@pytest.fixture(scope="module")
def model():
    from fastvideocodec_amd.models import get_codec_model
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        m = get_codec_model("DVC-pretrained", compression_level=2)
    return m.to(DEV).eval()


def test_calrealbits_forward(model):
    """calrealbits=True (net.py:147-149,174-176,201-203): bits = 8 x torchac bytes of each
    latent; the strings decode back to the rounded latents."""
    rng = np.random.default_rng(2)
    cur = torch.from_numpy(rng.random((1, 3, 64, 64), np.float32)).to(DEV)
    ref = torch.clamp(cur + 0.02 * torch.randn_like(cur), 0, 1)
    est = model(cur, ref)
    model.calrealbits = True
    try:
        real, t = model(cur, ref, return_intermediates=True)
    finally:
        model.calrealbits = False
    assert torch.equal(real[0], est[0])
    bz, bmv = model._be_params()
    fs = TAC.laplace_encode(t["feature"], t["sigma"], 96)
    zs = TAC.bitest_encode(t["z"], bz, 64)
    ms = TAC.bitest_encode(t["mvfeature"], bmv, 128)
    npx = 64 * 64
    assert abs(float(real[4]) - 8 * len(fs) / npx) < 1e-6
    assert abs(float(real[5]) - 8 * len(zs) / npx) < 1e-6
    assert abs(float(real[6]) - 8 * len(ms) / npx) < 1e-6
    back = TAC.laplace_decode(t["sigma"], 96, fs)
    assert torch.equal(back[..., :96], torch.round(t["feature"][..., :96]))
    # real bits track the estimate (the estimate clamps each symbol's bits to [0, 50])
    assert 0.5 * float(est[7]) < float(real[7]) < 2.0 * float(est[7]) + 1.0
