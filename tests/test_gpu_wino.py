"""The Winograd F(2x2,3x3) split-precision conv (fvc_conv_wino.hip) against float64 torch convs of
the same op (the ATen conv2d the reference's Warp_net ResBlocks call, endecoder.py:228-296) and
against the direct split-precision kernel: ragged sizes (tile rows, 32-column groups and images
cut at the edges), every epilogue form (ReLU input, ReLU / none activation, residual, the fused
2x2 pool), the dynamic and static schedules, the 32-bit-offset batch split, determinism and the
overflow flag."""
import os

import pytest
import torch
import torch.nn.functional as F

from fastvideocodec_amd import kernels as K

pytestmark = pytest.mark.gpu


def to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def from_nhwc(y):
    return y.permute(0, 3, 1, 2).contiguous()


def _packs(dev, w, b):
    """(winograd, direct x3) packs of the same 64->64 3x3 layer."""
    pw = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")
    assert pw.wino
    old = os.environ.get("FVC_WINO")
    os.environ["FVC_WINO"] = "0"
    try:
        pd = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")
    finally:
        if old is None:
            del os.environ["FVC_WINO"]
        else:
            os.environ["FVC_WINO"] = old
    assert not pd.wino and pd.x3
    return pw, pd


def _ref(x, w, b, in_relu, act_relu, res):
    xr = torch.relu(x) if in_relu else x
    y = F.conv2d(xr.double(), w.double(), b.double(), 1, 1)
    if act_relu:
        y = torch.relu(y)
    if res is not None:
        y = y + res.double()
    return y


# (B, H, W, in_relu, act_relu, with_res): Warp_net's forms, sizes cut at every edge
CASES = [
    (1, 40, 72, True, True, False),    # ResBlock conv1
    (2, 37, 70, False, False, True),   # ResBlock conv2 (residual), odd height, partial column group
    (1, 2, 30, True, False, False),    # a single tile row narrower than one column group
    (3, 68, 120, True, True, True),
    (1, 136, 96, False, True, False),  # more than one 16-row schedule chunk per column
]


@pytest.mark.parametrize("case", CASES)
def test_wino_vs_float64_and_direct(dev, case):
    B, H, W, in_relu, act_relu, with_res = case
    g = torch.Generator().manual_seed(100 + H)
    x = torch.randn(B, 64, H, W, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(64, generator=g) * 0.1
    res = torch.randn(B, 64, H, W, generator=g) if with_res else None
    ref = _ref(x, w, b, in_relu, act_relu, res)
    pw, pd = _packs(dev, w, b)
    kw = dict(in_op=K.IN_RELU if in_relu else K.IN_NONE, act=K.ACT_RELU if act_relu else K.ACT_NONE,
              res=to_nhwc(res).to(dev) if with_res else None)
    xd = to_nhwc(x).to(dev)
    yw, yd = pw(xd, **kw), pd(xd, **kw)
    torch.cuda.synchronize()
    ew = float((from_nhwc(yw.cpu()).double() - ref).abs().max())
    ed = float((from_nhwc(yd.cpu()).double() - ref).abs().max())
    scale = float(ref.abs().max())
    print(f"{case}: wino err {ew / scale:.2e}, direct x3 err {ed / scale:.2e} (of output scale)")
    # split-precision accuracy (test_gpu_kernels: direct x3 3-4e-7, fp32-MFMA ~1e-6 of scale)
    assert ew <= 2e-6 * scale, (ew, ed, scale)


@pytest.mark.parametrize("xscale", [1e-4, 1.0, 3000.0])
def test_wino_accuracy_across_activation_scales(dev, xscale):
    """Winograd's transforms add and subtract up to 4 inputs (and 4 products per output): the
    error stays at the split-precision level from tiny to large activations, and within 2x the
    fp32-MFMA kernel's own error."""
    g = torch.Generator().manual_seed(12)
    x = (torch.rand(1, 64, 40, 72, generator=g) - 0.3) * xscale
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.04
    b = torch.randn(64, generator=g) * 0.1 * xscale
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    xd = to_nhwc(x).to(dev)
    pw = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")
    assert pw.wino
    yw = pw(xd)
    y32 = K.PackedConv(w, b, 3, 1, False, dev, precision="f32")(xd)
    torch.cuda.synchronize()
    ew = float((from_nhwc(yw.cpu()).double() - ref).abs().max())
    e32 = float((from_nhwc(y32.cpu()).double() - ref).abs().max())
    scale = float(ref.abs().max())
    print(f"xscale {xscale}: wino err {ew / scale:.2e}, f32 err {e32 / scale:.2e}")
    assert ew <= 4e-6 * scale and ew <= 2 * e32 + 1e-7 * scale, (ew, e32, scale)


def test_wino_pool_epilogue_bitexact(dev):
    """call_pool on the Winograd kernel: y equals the plain launch bit for bit and pool equals
    fvc_avgpool2_nhwc of y bit for bit (ATen's summation order)."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 36, 98, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(64, generator=g) * 0.1
    res = to_nhwc(torch.randn(2, 64, 36, 98, generator=g)).to(dev)
    pw, _ = _packs(dev, w, b)
    xd = to_nhwc(x).to(dev)
    y, p = pw.call_pool(xd, res=res)
    y2 = pw(xd, res=res)
    p2 = K.avgpool2(y)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    assert torch.equal(p, p2)


def test_wino_schedules_and_determinism(dev, monkeypatch):
    """Dynamic (counter) and static chunk schedules and repeated launches give identical bits; the
    schedule scratch is left zeroed."""
    g = torch.Generator().manual_seed(6)
    x = to_nhwc(torch.randn(2, 64, 100, 130, generator=g)).to(dev)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    pw, _ = _packs(dev, w, torch.zeros(64))
    a = pw(x, in_op=K.IN_RELU, act=K.ACT_RELU)
    b = pw(x, in_op=K.IN_RELU, act=K.ACT_RELU)
    monkeypatch.setenv("FVC_X3_DYN", "0")
    c = pw(x, in_op=K.IN_RELU, act=K.ACT_RELU)
    monkeypatch.setenv("FVC_X3_RESERVE", "100")
    d = pw(x, in_op=K.IN_RELU, act=K.ACT_RELU)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c) and torch.equal(a, d)
    assert int(K.sched_scratch(dev)[:2].abs().sum()) == 0


def test_wino_overflow_flag(dev):
    """A transformed input >= 65000 cannot be split into fp16 halves: the kernel raises the
    stream's overflow flag (here one input of 7e4)."""
    g = torch.Generator().manual_seed(7)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    pw, _ = _packs(dev, w, torch.zeros(64))
    x = torch.randn(1, 64, 16, 32, generator=g)
    K.x3_overflow(reset=True)
    pw(to_nhwc(x).to(dev))
    assert not K.x3_overflow(reset=True)
    x[0, 5, 7, 9] = 7e4
    pw(to_nhwc(x).to(dev))
    assert K.x3_overflow(reset=True)


@pytest.mark.parametrize("shape", [(2, 19, 45), (1, 36, 98), (3, 5, 33)])
def test_wino_tap_epilogue(dev, shape, monkeypatch):
    """Winograd conv (residual, no activation: Warp_net conv5.conv2) with conv6's 27 tap partials in
    its epilogue (fvc_conv2d_nhwc_wino_tap) + the gather, against float64 torch and against the
    direct kernel's tap epilogue (FVC_WINO_TAP=0); ragged tile rows and column groups."""
    from fastvideocodec_amd import net
    B, H, W = shape
    g = torch.Generator().manual_seed(40 + H)
    x = torch.randn(B, 64, H, W, generator=g)
    res = torch.randn(B, 64, H, W, generator=g)
    w1 = torch.randn(64, 64, 3, 3, generator=g) * 0.04
    b1 = torch.randn(64, generator=g) * 0.1
    w2 = torch.randn(3, 64, 3, 3, generator=g) * (1.0 / (64 * 9) ** 0.5)
    b2 = torch.randn(3, generator=g) * 0.1
    y = F.conv2d(x.double(), w1.double(), b1.double(), 1, 1) + res.double()
    ref = F.conv2d(y, w2.double(), b2.double(), 1, 1)
    prod = net._ConvP(64, 64, 3, 1, False)
    prod.weight.data.copy_(w1)
    prod.bias.data.copy_(b1)
    cons = net._ConvP(64, 3, 3, 1, False)
    cons.weight.data.copy_(w2)
    cons.bias.data.copy_(b2)
    prod.to(dev)
    cons.to(dev)
    xd, rd = to_nhwc(x).to(dev), to_nhwc(res).to(dev)
    t = cons.tap_consumer()
    assert prod.packed().wino and t.wino_wpack is not None and prod.packed()._wino_tap(t)
    K.x3_overflow(reset=True)
    out_w = net.conv_then_tap(prod, xd, cons, res=rd)
    monkeypatch.setenv("FVC_WINO_TAP", "0")
    out_d = net.conv_then_tap(prod, xd, cons, res=rd)
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    scale = float(ref.abs().max())
    ew = float((from_nhwc(out_w.cpu())[:, :3].double() - ref).abs().max())
    ed = float((from_nhwc(out_d.cpu())[:, :3].double() - ref).abs().max())
    print(f"{shape}: wino tap err {ew / scale:.2e}, direct tap err {ed / scale:.2e} (of output scale)")
    assert ew <= 2e-6 * scale, (ew, ed, scale)
    assert float(out_w[..., 3:].abs().max()) == 0.0


# (B, H, W, in_op, act): the MV stacks' 128 -> 128 3x3 stride-1 forms (analysis_mv.py:58-66,
# synthesis_mv.py:59-79: ReLU act, conv8 none), sizes cut at every edge
CASES128 = [
    (2, 17, 30, K.IN_NONE, K.ACT_RELU),
    (1, 34, 60, K.IN_NONE, K.ACT_NONE),
    (3, 9, 70, K.IN_RELU, K.ACT_LRELU),
    (1, 40, 33, K.IN_NONE, K.ACT_RELU),
]


@pytest.mark.parametrize("case", CASES128, ids=lambda c: f"b{c[0]}_{c[1]}x{c[2]}_io{c[3]}_a{c[4]}")
def test_wino128_quarters_vs_float64_and_direct(dev, case, monkeypatch):
    """fvc_conv2d_nhwc_wino128 (four 64 -> 64 Winograd quarters on 128-channel pixels, the second
    input half adding the first's partial sum before the activation) against float64 torch and the
    direct x3 kernel (FVC_WINO128=0); determinism; the overflow flag stays clear."""
    B, H, W, in_op, act = case
    g = torch.Generator().manual_seed(B * 1000 + H * W + act)
    w = torch.randn(128, 128, 3, 3, generator=g) * (1.0 / (128 * 9) ** 0.5)
    b = torch.randn(128, generator=g) * 0.1
    x = torch.randn(B, 128, H, W, generator=g) * 2
    xr = torch.relu(x) if in_op == K.IN_RELU else x
    ref = F.conv2d(xr.double(), w.double(), b.double(), 1, 1)
    ref = {K.ACT_NONE: ref, K.ACT_RELU: torch.relu(ref), K.ACT_LRELU: F.leaky_relu(ref, 0.1)}[act]
    monkeypatch.setenv("FVC_WINO128_MINPIX", "0")  # test sizes are below the production gate
    monkeypatch.setenv("FVC_WINO128", "1")
    pw = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")
    monkeypatch.setenv("FVC_WINO128", "0")
    pd = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")
    assert pw.wino128 and not pd.wino128 and pd.x3
    xd = to_nhwc(x).to(dev)
    K.x3_overflow(reset=True)
    yw = pw(xd, in_op=in_op, act=act)
    yw2 = pw(xd, in_op=in_op, act=act)
    yd = pd(xd, in_op=in_op, act=act)
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    assert torch.equal(yw, yw2)
    assert not torch.equal(yw, yd)  # two algorithms ran
    scale = float(ref.abs().max())
    ew = float((from_nhwc(yw.cpu()).double() - ref).abs().max())
    ed = float((from_nhwc(yd.cpu()).double() - ref).abs().max())
    print(f"{case}: wino128 {ew / scale:.2e}, direct {ed / scale:.2e} of output scale")
    assert ew <= 1e-6 * scale and ew <= 2 * ed + 1e-7 * scale, (ew, ed, scale)


def test_wino128_rejects_residual_and_wrong_pitch_forms():
    """The quarter form takes no residual (PackedConv keeps such calls on the direct kernel) and
    the C-ABI refuses null buffers."""
    from fastvideocodec_amd import _lib
    lib = _lib.load()
    assert lib.fvc_conv_wino128_supported(128, 128, 3, 1, 0) == 1
    assert lib.fvc_conv_wino128_supported(128, 128, 3, 2, 0) == 0
    assert lib.fvc_conv_wino128_supported(64, 64, 3, 1, 0) == 0
    assert lib.fvc_conv2d_nhwc_wino128(None, None, None, None, None, 1, 4, 4, 0, 0, 0, None, None, 0, None) < 0


# (B, H, W): the fused upsample-add input (Warp_net c3_u / c4_u feeding ResBlock conv1), sizes cut
# at every edge: partial column groups, one tile row, several 16-row schedule chunks per column,
# chunks of 1, 2 and 4 items (the staging two items ahead falls back at chunk ends)
UP_CASES = [(1, 40, 72), (2, 36, 70), (1, 2, 30), (3, 68, 120), (1, 136, 96), (2, 4, 64), (2, 34, 66), (1, 66, 40)]


@pytest.mark.parametrize("case", UP_CASES)
def test_wino_up_fused_matches_upsample_then_conv(dev, case, monkeypatch):
    """call_up (X = skip + up2(low) formed in the Winograd kernel's staging) against the
    standalone upsample-add kernel followed by the plain Winograd launch: X and y bit for bit,
    under the dynamic and the static chunk schedule, for the ResBlock conv1 form and a plain one;
    the schedule scratch is left zeroed."""
    B, H, W = case
    g = torch.Generator().manual_seed(300 + H + W)
    skip = to_nhwc(torch.randn(B, 64, H, W, generator=g)).to(dev)
    low = to_nhwc(torch.randn(B, 64, H // 2, W // 2, generator=g)).to(dev)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(64, generator=g) * 0.1
    pw, _ = _packs(dev, w, b)
    assert pw.up_fusable()
    xs_ref = K.upsample2x_add(low, skip=skip, align_corners=True)
    for in_op, act in ((K.IN_RELU, K.ACT_RELU), (K.IN_NONE, K.ACT_NONE)):
        y_ref = pw(xs_ref, in_op=in_op, act=act)
        y, xs = pw.call_up(skip, low, in_op=in_op, act=act)
        monkeypatch.setenv("FVC_X3_DYN", "0")
        y2, xs2 = pw.call_up(skip, low, in_op=in_op, act=act)
        monkeypatch.delenv("FVC_X3_DYN")
        torch.cuda.synchronize()
        assert torch.equal(xs, xs_ref), float((xs - xs_ref).abs().max())
        assert torch.equal(y, y_ref), float((y - y_ref).abs().max())
        assert torch.equal(xs2, xs_ref) and torch.equal(y2, y_ref)
    assert int(K.sched_scratch(dev)[:2].abs().sum()) == 0


def test_wino_up_vs_float64(dev):
    """The fused input against float64 torch: F.interpolate(low, 2x, bilinear, align_corners=True)
    + skip, then the ResBlock conv1 (endecoder.py:228-293)."""
    g = torch.Generator().manual_seed(31)
    skip = torch.randn(2, 64, 68, 98, generator=g)
    low = torch.randn(2, 64, 34, 49, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(64, generator=g) * 0.1
    xr = skip.double() + F.interpolate(low.double(), scale_factor=2, mode="bilinear", align_corners=True)
    ref = torch.relu(F.conv2d(torch.relu(xr), w.double(), b.double(), 1, 1))
    pw, _ = _packs(dev, w, b)
    y, xs = pw.call_up(to_nhwc(skip).to(dev), to_nhwc(low).to(dev), in_op=K.IN_RELU, act=K.ACT_RELU)
    torch.cuda.synchronize()
    ex = float((from_nhwc(xs.cpu()).double() - xr).abs().max())
    ey = float((from_nhwc(y.cpu()).double() - ref).abs().max())
    print(f"fused up: X err {ex:.2e} (scale {float(xr.abs().max()):.2f}), y err {ey / float(ref.abs().max()):.2e} of scale")
    assert ex <= 4e-6 * float(xr.abs().max())
    assert ey <= 2e-6 * float(ref.abs().max())
