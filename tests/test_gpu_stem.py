"""conv_stem_kernel (fvc_conv_stem.hip): the split-precision streaming conv of the small-input stems
(Warp_net feature_ext 3x3 6->64, endecoder.py:253-261; mvEncoder conv1 3x3 s2 2->128,
analysis_mv.py:19-21; resEncoder conv1 5x5 s2 3->64, analysis.py:15-17) against a float64 conv of
the same op and against the direct x3 kernel it replaces (FVC_STEM=0)."""
import os

import pytest
import torch
import torch.nn.functional as F

from fastvideocodec_amd import kernels as K

pytestmark = pytest.mark.gpu


def _packs(dev, w, b, stride):
    k = w.shape[-1]
    old = os.environ.get("FVC_STEM")
    os.environ["FVC_STEM"] = "1"
    try:
        ps = K.PackedConv(w, b, k, stride, False, dev, precision="x3")
    finally:
        if old is None:
            del os.environ["FVC_STEM"]
        else:
            os.environ["FVC_STEM"] = old
    assert ps.stem is not None
    old = os.environ.get("FVC_STEM")
    os.environ["FVC_STEM"] = "0"
    try:
        pd = K.PackedConv(w, b, k, stride, False, dev, precision="x3")
    finally:
        if old is None:
            del os.environ["FVC_STEM"]
        else:
            os.environ["FVC_STEM"] = old
    assert pd.stem is None
    return ps, pd


def _ref(x, w, b, stride, act):
    cin = w.shape[1]
    y = F.conv2d(x[..., :cin].permute(0, 3, 1, 2).double().cpu(), w.double(), b.double(), stride=stride,
                 padding=w.shape[-1] // 2).permute(0, 2, 3, 1)
    if act == K.ACT_RELU:
        y = torch.relu(y)
    elif act == K.ACT_LRELU:
        y = F.leaky_relu(y, 0.1)
    return y


CASES = [
    # (cin, cout, k, stride, B, H, W, act)
    (6, 64, 3, 1, 2, 37, 70, K.ACT_RELU),      # Warp_net feature_ext, ragged strips
    (2, 128, 3, 2, 1, 40, 136, K.ACT_LRELU),   # mvEncoder conv1
    (3, 64, 5, 2, 3, 30, 66, K.ACT_NONE),      # resEncoder conv1
    (8, 128, 5, 2, 1, 18, 64, K.ACT_NONE),
    (4, 64, 3, 2, 2, 16, 34, K.ACT_RELU),
    (1, 128, 3, 1, 1, 9, 33, K.ACT_NONE),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[1]}k{c[2]}s{c[3]}" for c in CASES])
def test_stem_vs_float64_and_direct(dev, case):
    cin, cout, k, s, B, H, W, act = case
    g = torch.Generator().manual_seed(cin * 1000 + cout + k)
    x = torch.randn(B, H, W, K.cp4(cin), generator=g)
    x[..., cin:] = 0.0
    w = torch.randn(cout, cin, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    ps, pd = _packs(dev, w, b, s)
    xd = x.to(dev)
    K.x3_overflow(reset=True)
    ys, yd = ps(xd, act=act), pd(xd, act=act)
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    ref = _ref(x, w, b, s, act)
    scale = float(ref.abs().max())
    es = float((ys.double().cpu() - ref).abs().max()) / scale
    ed = float((yd.double().cpu() - ref).abs().max()) / scale
    print(f"{case}: stem {es:.2e}, direct x3 {ed:.2e} (of output scale)")
    # the same split arithmetic: fp32-level, no worse than the direct kernel beyond rounding order
    assert es <= 2e-6 and es <= 2 * ed + 2e-7, (es, ed)
    # deterministic
    assert torch.equal(ys, ps(xd, act=act))


def test_stem_overflow_flag(dev):
    """An input past the fp16 range of the split (>= 65520) raises the overflow flag."""
    g = torch.Generator().manual_seed(5)
    w = torch.randn(64, 6, 3, 3, generator=g) * 0.1
    ps, _ = _packs(dev, w, torch.zeros(64), 1)
    x = torch.randn(1, 8, 32, 8, generator=g)
    x[0, 3, 5, 2] = 1e5
    K.x3_overflow(reset=True)
    ps(x.to(dev))
    torch.cuda.synchronize()
    assert K.x3_overflow(reset=True)
    x[0, 3, 5, 2] = 6e4  # inside the range: no flag
    ps(x.to(dev))
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)


def test_stem_rejects_unsupported(dev):
    from fastvideocodec_amd import _lib
    lib = _lib.load()
    assert lib.fvc_conv_stem_supported(6, 64, 3, 1, 0) == 1
    assert lib.fvc_conv_stem_supported(9, 64, 3, 1, 0) == 0   # cin > 8
    assert lib.fvc_conv_stem_supported(6, 32, 3, 1, 0) == 0   # cout
    assert lib.fvc_conv_stem_supported(6, 64, 5, 1, 0) == 0   # 5x5 stride 1
    assert lib.fvc_conv_stem_supported(6, 64, 3, 2, 1) == 0   # transposed


@pytest.mark.parametrize("case", [(6, 64, 3, 1, K.ACT_RELU), (2, 128, 3, 2, K.ACT_LRELU), (3, 64, 5, 2, K.ACT_NONE)],
                         ids=["feature_ext", "mvEncoder_conv1", "resEncoder_conv1"])
def test_stem_full_size_matches_direct(dev, case):
    """The production geometries at 1088x1920, two frames (thousands of tiles per launch, every
    persistent block looping over many): equal to the direct x3 kernel within the two kernels'
    rounding (both ~2e-7 of scale from float64), deterministic, no overflow."""
    cin, cout, k, s, act = case
    g = torch.Generator().manual_seed(11 + cin)
    w = torch.randn(cout, cin, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    ps, pd = _packs(dev, w, b, s)
    x = torch.rand(2, 1088, 1920, K.cp4(cin), generator=g)
    x[..., cin:] = 0.0
    xd = x.to(dev)
    K.x3_overflow(reset=True)
    ys, yd = ps(xd, act=act), pd(xd, act=act)
    ys2 = ps(xd, act=act)
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    assert torch.equal(ys, ys2)
    scale = float(yd.abs().max())
    diff = float((ys - yd).abs().max()) / scale
    assert diff <= 1e-6, diff


@pytest.mark.parametrize("cin", [2, 3, 6])
def test_stem_pad_channels_masked(dev, cin):
    """the pad channels (cin .. pitch-1) are masked at staging, so garbage a producer left
    there (NaN, Inf, huge values) changes nothing: the output equals the zero-padded input's, bit for
    bit, and the overflow flag stays clear."""
    g = torch.Generator().manual_seed(40 + cin)
    cout, k, s = (128, 3, 2) if cin == 2 else ((64, 5, 2) if cin == 3 else (64, 3, 1))
    w = torch.randn(cout, cin, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    ps, _ = _packs(dev, w, torch.zeros(cout), s)
    x = torch.rand(2, 24, 70, K.cp4(cin), generator=g)
    x[..., cin:] = 0.0
    xg = x.clone()
    pads = K.cp4(cin) - cin
    fill = torch.tensor([float("nan"), float("inf"), -1e30, 7.0])
    xg[..., cin:] = fill[torch.arange(pads) % 4]
    K.x3_overflow(reset=True)
    y0, y1 = ps(x.to(dev)), ps(xg.to(dev))
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    assert torch.equal(y0, y1)
