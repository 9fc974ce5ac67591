"""Per-kernel parity of libfvc (HIP, cuda:0) against plain PyTorch fp32 CPU references of the
same op (the ATen ops the reference forward calls) and the coder oracle (byte-exact)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fastvideocodec_amd import kernels as K
from fastvideocodec_amd import entropy_models as EM
from oracle import coder_ref as R
from oracle import dvc_ref

pytestmark = pytest.mark.gpu


def to_nhwc(x, cp=None):
    B, C, H, W = x.shape
    cp = cp or K.cp4(C)
    y = torch.zeros(B, H, W, cp)
    y[..., :C] = x.permute(0, 2, 3, 1)
    return y.contiguous()


def from_nhwc(y, c):
    return y[..., :c].permute(0, 3, 1, 2).contiguous()


def close(a, b, tol):
    scale = float(b.abs().max()) + 1e-6
    err = float((a - b).abs().max())
    assert err <= tol * scale + 1e-6, f"max err {err:.3e} vs scale {scale:.3e}"


# (cin, cout, k, stride, transposed, H, W, in_op, act, post, with_res)
CONV_CASES = [
    (8, 32, 7, 1, False, 36, 70, K.IN_NONE, K.ACT_RELU, K.POST_NONE, False),
    (32, 64, 7, 1, False, 20, 40, K.IN_NONE, K.ACT_RELU, K.POST_NONE, False),
    (64, 32, 7, 1, False, 17, 33, K.IN_NONE, K.ACT_RELU, K.POST_NONE, False),
    (32, 16, 7, 1, False, 16, 32, K.IN_NONE, K.ACT_RELU, K.POST_NONE, False),
    (16, 2, 7, 1, False, 24, 40, K.IN_NONE, K.ACT_NONE, K.POST_NONE, True),
    (2, 128, 3, 2, False, 32, 64, K.IN_NONE, K.ACT_LRELU, K.POST_NONE, False),
    (128, 128, 3, 1, False, 12, 40, K.IN_NONE, K.ACT_LRELU, K.POST_NONE, False),
    (128, 128, 3, 2, False, 16, 34, K.IN_NONE, K.ACT_LRELU, K.POST_NONE, False),
    (128, 128, 3, 2, True, 5, 9, K.IN_ROUND, K.ACT_LRELU, K.POST_NONE, False),
    (128, 2, 3, 1, False, 16, 24, K.IN_NONE, K.ACT_NONE, K.POST_NONE, False),
    (6, 64, 3, 1, False, 24, 48, K.IN_NONE, K.ACT_RELU, K.POST_NONE, False),
    (64, 64, 3, 1, False, 19, 45, K.IN_RELU, K.ACT_RELU, K.POST_NONE, True),
    (64, 3, 3, 1, False, 16, 32, K.IN_NONE, K.ACT_NONE, K.POST_NONE, True),
    (3, 64, 5, 2, False, 32, 64, K.IN_NONE, K.ACT_NONE, K.POST_NONE, False),
    (64, 64, 5, 2, False, 16, 70, K.IN_NONE, K.ACT_NONE, K.POST_NONE, False),
    (64, 96, 5, 2, False, 8, 16, K.IN_NONE, K.ACT_NONE, K.POST_NONE, False),
    (96, 64, 3, 1, False, 4, 8, K.IN_ABS, K.ACT_RELU, K.POST_NONE, False),
    (96, 64, 5, 2, True, 4, 6, K.IN_ROUND, K.ACT_NONE, K.POST_NONE, False),
    (64, 64, 5, 2, True, 8, 12, K.IN_NONE, K.ACT_RELU, K.POST_NONE, False),
    (64, 3, 5, 2, True, 16, 17, K.IN_NONE, K.ACT_NONE, K.POST_NONE, True),
    (64, 96, 3, 1, True, 4, 8, K.IN_NONE, K.ACT_NONE, K.POST_EXP, False),
]


def _in_op(x, op):
    return {K.IN_NONE: x, K.IN_RELU: F.relu(x), K.IN_ABS: x.abs(), K.IN_ROUND: torch.round(x)}[op]


@pytest.mark.parametrize("precision", ["x3", "f32"])
@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: f"ci{c[0]}co{c[1]}k{c[2]}s{c[3]}{'T' if c[4] else ''}")
def test_conv(dev, case, precision):
    cin, cout, k, s, tr, H, W, in_op, act, post, with_res = case
    g = torch.Generator().manual_seed(cin * 1000 + cout + k)
    x = torch.randn(2, cin, H, W, generator=g) * 2.0
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    w = torch.randn(wshape, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    xin = _in_op(x, in_op)
    if tr:
        ref = F.conv_transpose2d(xin, w, b, s, k // 2, s - 1)
    else:
        ref = F.conv2d(xin, w, b, s, k // 2)
    if act == K.ACT_RELU:
        ref = F.relu(ref)
    elif act == K.ACT_LRELU:
        ref = F.leaky_relu(ref, 0.1)
    res = torch.randn(ref.shape, generator=g) if with_res else None
    if res is not None:
        ref = ref + res
    if post == K.POST_EXP:
        ref = torch.exp(ref)
    pc = K.PackedConv(w, b, k, s, tr, dev, precision=precision)
    K.x3_overflow(reset=True)
    y = pc(to_nhwc(x).to(dev), in_op=in_op, act=act, post=post,
           res=None if res is None else to_nhwc(res).to(dev))
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    yc = y.cpu()
    assert yc.shape[1:3] == ref.shape[2:]
    close(from_nhwc(yc, cout), ref, 2e-5)
    if K.cp4(cout) > cout:
        assert float(yc[..., cout:].abs().max()) == 0.0, "pad channels must be zero"


@pytest.mark.parametrize("case", [CONV_CASES[i] for i in (0, 8, 11, 12, 19)],
                         ids=lambda c: f"ci{c[0]}co{c[1]}k{c[2]}s{c[3]}{'T' if c[4] else ''}")
def test_conv_x3_weight_paths_identical(dev, case, monkeypatch):
    """Weights staged per chunk in LDS (FVC_X3_BLDS=1, where they fit) and weights read from L2 by
    every wave (default) feed the same MFMAs in the same order: bit-identical outputs."""
    cin, cout, k, s, tr, H, W, in_op, act, post, with_res = case
    g = torch.Generator().manual_seed(7 + cin + cout)
    x = to_nhwc(torch.randn(2, cin, H, W, generator=g)).to(dev)
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    pc = K.PackedConv(w, b, k, s, tr, dev, precision="x3")
    assert pc.x3
    ho, wo = pc.out_hw(H, W)
    res = to_nhwc(torch.randn(2, cout, ho, wo, generator=g)).to(dev) if with_res else None
    outs = []
    for bl in ("1", "0"):
        monkeypatch.setenv("FVC_X3_BLDS", bl)
        outs.append(pc(x, in_op=in_op, act=act, post=post, res=res))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("case", [CONV_CASES[i] for i in (9, 12, 19)],
                         ids=lambda c: f"ci{c[0]}co{c[1]}k{c[2]}s{c[3]}{'T' if c[4] else ''}")
def test_conv_tap_partial_path(dev, case, monkeypatch):
    """cout <= 4 layers as a 1x1 x3 GEMM to k*k*cout tap partials + fvc_tap_gather_nhwc (forced
    for every eligible geometry with FVC_TAPSUM=2) against the fp32 torch conv."""
    monkeypatch.setenv("FVC_TAPSUM", "2")
    cin, cout, k, s, tr, H, W, in_op, act, post, with_res = case
    g = torch.Generator().manual_seed(cin + 31 * cout)
    x = torch.randn(2, cin, H, W, generator=g) * 2.0
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    xin = _in_op(x, in_op)
    ref = F.conv_transpose2d(xin, w, b, s, k // 2, s - 1) if tr else F.conv2d(xin, w, b, s, k // 2)
    res = torch.randn(ref.shape, generator=g) if with_res else None
    if res is not None:
        ref = ref + res
    pc = K.PackedConv(w, b, k, s, tr, dev, precision="x3")
    assert pc.tap is not None
    y = pc(to_nhwc(x).to(dev), in_op=in_op, act=act, post=post, res=None if res is None else to_nhwc(res).to(dev))
    torch.cuda.synchronize()
    yc = y.cpu()
    close(from_nhwc(yc, cout), ref, 2e-5)
    assert float(yc[..., cout:].abs().max()) == 0.0


# (producer cin, cout, k, stride, transposed, act, with_res, consumer cout, k, H, W, batch)
TAP_FUSE_CASES = [
    (128, 128, 3, 2, True, K.ACT_LRELU, False, 2, 3, 9, 21, 2),    # mvDecoder deconv7 -> deconv8
    (64, 64, 3, 1, False, K.ACT_NONE, True, 3, 3, 19, 45, 2),      # Warp_net conv5.conv2 -> conv6
    (64, 64, 3, 1, False, K.ACT_RELU, False, 2, 5, 17, 33, 1),     # 5x5 consumer, 50 partials > 32: refused
    (32, 32, 3, 1, False, K.ACT_NONE, True, 3, 3, 16, 40, 3),      # one N-tile producer
]


@pytest.mark.parametrize("case", TAP_FUSE_CASES, ids=lambda c: f"p{c[0]}-{c[1]}k{c[2]}{'T' if c[4] else ''}-c{c[7]}k{c[8]}")
def test_conv_then_tap_fused(dev, case, monkeypatch):
    """Producer conv with the consumer's 1x1 tap-partial GEMM in its epilogue
    (fvc_*_x3_tap + fvc_tap_gather_nhwc) against the fp32 torch pair, and against the unfused
    two-layer path (FVC_TAP_FUSE=0)."""
    from fastvideocodec_amd import net
    ci, co, k, s, tr, act, with_res, c2, k2, H, W, B = case
    g = torch.Generator().manual_seed(ci + 7 * co + k2)
    x = torch.randn(B, ci, H, W, generator=g)
    w1 = torch.randn((ci, co, k, k) if tr else (co, ci, k, k), generator=g) * (1.0 / (ci * k * k) ** 0.5)
    b1 = torch.randn(co, generator=g) * 0.1
    w2 = torch.randn(c2, co, k2, k2, generator=g) * (1.0 / (co * k2 * k2) ** 0.5)
    b2 = torch.randn(c2, generator=g) * 0.1
    y = F.conv_transpose2d(x, w1, b1, s, k // 2, s - 1) if tr else F.conv2d(x, w1, b1, s, k // 2)
    y = {K.ACT_NONE: y, K.ACT_RELU: F.relu(y), K.ACT_LRELU: F.leaky_relu(y, 0.1)}[act]
    res = torch.randn(y.shape, generator=g) if with_res else None
    if res is not None:
        y = y + res
    ref = F.conv2d(y, w2, b2, 1, k2 // 2)
    res2 = torch.randn(ref.shape, generator=g)
    ref = ref + res2

    prod = net._ConvP(ci, co, k, s, tr)
    prod.weight.data.copy_(w1)
    prod.bias.data.copy_(b1)
    cons = net._ConvP(co, c2, k2, 1, False)
    cons.weight.data.copy_(w2)
    cons.bias.data.copy_(b2)
    prod.to(dev)
    cons.to(dev)
    xd = to_nhwc(x).to(dev)
    rd = None if res is None else to_nhwc(res).to(dev)
    r2d = to_nhwc(res2).to(dev)
    t = cons.tap_consumer()
    fusable = t is not None and prod.packed().tap_fusable(t)
    assert fusable == (c2 * k2 * k2 <= 32), "fusion must cover exactly the <= 32-partial consumers"
    K.x3_overflow(reset=True)
    out = net.conv_then_tap(prod, xd, cons, act=act, res=rd, cons_res=r2d)
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    oc = out.cpu()
    close(from_nhwc(oc, c2), ref, 2e-5)
    assert float(oc[..., c2:].abs().max()) == 0.0
    monkeypatch.setenv("FVC_TAP_FUSE", "0")
    out2 = net.conv_then_tap(prod, xd, cons, act=act, res=rd, cons_res=r2d)
    torch.cuda.synchronize()
    close(from_nhwc(out2.cpu(), c2), from_nhwc(oc, c2), 2e-6)


@pytest.mark.parametrize("inverse", [True, False])
def test_gdn_then_tap_fused(dev, inverse, monkeypatch):
    """IGDN / GDN (64 ch) with the next 64->3 5x5 s2 transposed conv's 75 tap partials computed
    in the GDN kernel (fvc_gdn_tap_nhwc, 3 P tiles) + the transposed gather, against torch fp32
    (GDN.py:63-93 then conv_transpose2d + residual), and the model path with and without the
    fusion (FVC_GDN_TAP) on a decoder-sized call."""
    g = torch.Generator().manual_seed(21 + int(inverse))
    B, H, W = 2, 13, 22
    x = torch.randn(B, 64, H, W, generator=g)
    beta = torch.rand(64, generator=g) + 0.5
    gamma = torch.rand(64, 64, generator=g) * 0.05 + torch.eye(64) * 0.2
    w = torch.randn(64, 3, 5, 5, generator=g) * (1.0 / (64 * 25) ** 0.5)
    b = torch.randn(3, generator=g) * 0.1
    norm = torch.sqrt(F.conv2d(x * x, gamma[:, :, None, None], beta))
    y = x * norm if inverse else x / norm
    ref = F.conv_transpose2d(y, w, b, 2, 2, 1)
    res = torch.randn(ref.shape, generator=g)
    ref = ref + res
    t = K.GdnTap(w, b, 5, 2, True, dev)
    assert (t.np, t.pcp, t.ntiles) == (75, 76, 3)
    K.x3_overflow(reset=True)
    out = t(to_nhwc(x).to(dev), beta.to(dev), gamma.to(dev).contiguous(), inverse, res=to_nhwc(res).to(dev))
    torch.cuda.synchronize()
    assert not K.x3_overflow(reset=True)
    oc = out.cpu()
    close(from_nhwc(oc, 3), ref, 2e-5)
    assert float(oc[..., 3:].abs().max()) == 0.0


@pytest.mark.parametrize("shape", [(2, 64, 64, 38, 70), (1, 64, 64, 33, 45), (3, 32, 64, 16, 32), (2, 64, 32, 20, 96)])
@pytest.mark.parametrize("with_res", [False, True])
def test_conv_x3_pool_epilogue(dev, shape, with_res, monkeypatch):
    """Conv with avg_pool2d(y, 2) in its epilogue (fvc_conv2d_nhwc_x3_pool): y identical to the
    plain launch, the pool identical (bits) to fvc_avgpool2_nhwc of y, odd sizes floored; also
    through the batch split (FVC_X3_SPLIT_BYTES)."""
    B, ci, co, H, W = shape
    g = torch.Generator().manual_seed(B + ci + H)
    x = to_nhwc(torch.randn(B, ci, H, W, generator=g)).to(dev)
    w = torch.randn(co, ci, 3, 3, generator=g) * (1.0 / (ci * 9) ** 0.5)
    b = torch.randn(co, generator=g) * 0.1
    res = to_nhwc(torch.randn(B, co, H, W, generator=g)).to(dev) if with_res else None
    pc = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")
    assert pc.pool_fusable()
    y0 = pc(x, act=K.ACT_RELU, res=res)
    p0 = K.avgpool2(y0[:, :H // 2 * 2, :W // 2 * 2].contiguous())  # avg_pool2d floors odd sizes
    y1, p1 = pc.call_pool(x, act=K.ACT_RELU, res=res)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert p1.shape == (B, H // 2, W // 2, K.cp4(co))
    assert torch.equal(p0, p1)
    if B > 1:
        monkeypatch.setenv("FVC_X3_SPLIT_BYTES", str(H * W * K.cp4(co) * 4 + 4))  # one image per launch
        y2, p2 = pc.call_pool(x, act=K.ACT_RELU, res=res)
        torch.cuda.synchronize()
        assert torch.equal(y0, y2) and torch.equal(p0, p2)


@pytest.mark.parametrize("wn", ["1", "2", "4"])
def test_conv_x3_ntile_groupings(dev, wn, monkeypatch):
    """The stride-2 128->128 conv with 1, 2 or all 4 N-tiles per block (FVC_X3_WN; 4 is the
    default at full size) against the fp32 torch conv; all three must give identical bits."""
    monkeypatch.setenv("FVC_X3_WN", wn)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 128, 48, 96, generator=g)
    w = torch.randn(128, 128, 3, 3, generator=g) * (1.0 / (128 * 9) ** 0.5)
    b = torch.randn(128, generator=g) * 0.1
    ref = F.leaky_relu(F.conv2d(x, w, b, 2, 1), 0.1)
    pc = K.PackedConv(w, b, 3, 2, False, dev, precision="x3")
    y = pc(to_nhwc(x).to(dev), act=K.ACT_LRELU)
    torch.cuda.synchronize()
    close(from_nhwc(y.cpu(), 128), ref, 2e-5)
    monkeypatch.setenv("FVC_X3_WN", "1")
    y1 = pc(to_nhwc(x).to(dev), act=K.ACT_LRELU)
    torch.cuda.synchronize()
    assert torch.equal(y, y1)


@pytest.mark.parametrize("with_res", [False, True])
def test_conv_x3_batch_split(dev, with_res, monkeypatch):
    """Outputs >= 4 GB are computed as launches over sub-batches (32-bit buffer offsets); the
    split (forced here at a small size with FVC_X3_SPLIT_BYTES) must give the same bits as one
    launch, with and without a residual (a missing residual must stay missing in every part)."""
    g = torch.Generator().manual_seed(9)
    x = to_nhwc(torch.randn(5, 64, 20, 40, generator=g)).to(dev)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.04
    b = torch.randn(64, generator=g) * 0.1
    res = to_nhwc(torch.randn(5, 64, 20, 40, generator=g)).to(dev) if with_res else None
    pc = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")
    y1 = pc(x, in_op=K.IN_RELU, res=res)
    monkeypatch.setenv("FVC_X3_SPLIT_BYTES", str(2 * 20 * 40 * 64 * 4))  # parts of <= 1 image
    y2 = pc(x, in_op=K.IN_RELU, res=res)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)


def test_conv_x3_overflow_flag(dev):
    """|activation| >= 65000 cannot be split into fp16 halves: the x3 kernel must flag it."""
    w = torch.randn(64, 64, 3, 3) * 0.05
    pc = K.PackedConv(w, torch.zeros(64), 3, 1, False, dev, precision="x3")
    assert pc.x3
    x = torch.zeros(1, 64, 16, 32)
    K.x3_overflow(reset=True)
    pc(to_nhwc(x).to(dev))
    assert not K.x3_overflow(reset=True)
    x[0, 5, 3, 7] = 7.0e4
    pc(to_nhwc(x).to(dev))
    assert K.x3_overflow(reset=True)


def test_conv_x3_matches_f32_closely(dev):
    """The split-precision kernel tracks the fp32 MFMA kernel to ~1e-6 relative on a 3x3 64-ch
    layer at a realistic activation scale (ulp-level differences only)."""
    g = torch.Generator().manual_seed(11)
    x = torch.rand(1, 64, 48, 96, generator=g) * 3.0
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.04
    b = torch.randn(64, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1).float()
    xd = to_nhwc(x).to(dev)
    y3 = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")(xd)
    y32 = K.PackedConv(w, b, 3, 1, False, dev, precision="f32")(xd)
    torch.cuda.synchronize()
    e3 = float((from_nhwc(y3.cpu(), 64) - ref).abs().max())
    e32 = float((from_nhwc(y32.cpu(), 64) - ref).abs().max())
    scale = float(ref.abs().max())
    assert e3 <= 4e-6 * scale, (e3, e32, scale)


@pytest.mark.parametrize("xscale", [1e-4, 1e-2, 1.0, 3e3])
def test_conv_x3_accuracy_across_activation_scales(dev, xscale):
    """The split keeps fp32-level accuracy from tiny activations (residual halves in fp16's
    subnormal range) to large ones: max error vs a float64 conv within 4e-6 of the output
    scale, and within 4x the fp32-MFMA kernel's own error."""
    g = torch.Generator().manual_seed(12)
    x = (torch.rand(1, 64, 40, 72, generator=g) - 0.3) * xscale
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.04
    b = torch.randn(64, generator=g) * 0.1 * xscale
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    xd = to_nhwc(x).to(dev)
    y3 = K.PackedConv(w, b, 3, 1, False, dev, precision="x3")(xd)
    y32 = K.PackedConv(w, b, 3, 1, False, dev, precision="f32")(xd)
    torch.cuda.synchronize()
    e3 = float((from_nhwc(y3.cpu(), 64).double() - ref).abs().max())
    e32 = float((from_nhwc(y32.cpu(), 64).double() - ref).abs().max())
    scale = float(ref.abs().max())
    print(f"xscale {xscale}: x3 err {e3 / scale:.2e}, f32 err {e32 / scale:.2e} (relative to output scale)")
    assert e3 <= 4e-6 * scale, (e3, e32, scale)
    assert e3 <= 4 * e32 + 1e-7 * scale, (e3, e32, scale)


def test_conv_deterministic(dev):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(1, 64, 33, 65, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    pc = K.PackedConv(w, torch.zeros(64), 3, 1, False, dev)
    xd = to_nhwc(x).to(dev)
    a, b = pc(xd), pc(xd)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_warp(dev):
    g = torch.Generator().manual_seed(1)
    im = torch.rand(2, 3, 40, 72, generator=g)
    flow = torch.randn(2, 2, 40, 72, generator=g) * 6.0
    ref = dvc_ref.warp(im, flow)
    y = K.warp(to_nhwc(im).to(dev), to_nhwc(flow).to(dev))
    close(from_nhwc(y.cpu(), 3), ref, 1e-5)


@pytest.mark.parametrize("ac", [False, True])
@pytest.mark.parametrize("scale", [1.0, 2.0])
def test_upsample_add(dev, ac, scale):
    """Against the oracle's upsample (both align_corners modes, scale 1 and SpyNet's 2), and the
    channel-padded run (68 = 64 + 4 zero pad channels) bit-identical on the real channels."""
    g = torch.Generator().manual_seed(2)
    src = torch.randn(2, 64, 9, 15, generator=g)
    skip = torch.randn(2, 64, 18, 30, generator=g)
    ref = skip + dvc_ref.up2(src, ac) * scale
    y = K.upsample2x_add(to_nhwc(src).to(dev), to_nhwc(skip).to(dev), align_corners=ac, scale=scale)
    close(from_nhwc(y.cpu(), 64), ref, 1e-6)
    y68 = K.upsample2x_add(to_nhwc(src, 68).to(dev), to_nhwc(skip, 68).to(dev), align_corners=ac, scale=scale)
    torch.cuda.synchronize()
    assert torch.equal(y68[..., :64], y)


@pytest.mark.parametrize("shape", [(2, 9, 15), (1, 1, 1), (1, 1, 7), (3, 6, 1), (1, 34, 60)])
@pytest.mark.parametrize("with_skip", [False, True])
def test_upsample_64ch_forms_bit_identical(dev, shape, with_skip, monkeypatch):
    """The 64-channel upsample-add forms (FVC_UP2_Q16: 1 = 32-bit-index float4 per thread, 0 =
    generic) give the same bits, including images of one source row / column, and match the oracle."""
    B, h, w = shape
    g = torch.Generator().manual_seed(h * 100 + w)
    src = to_nhwc(torch.randn(B, 64, h, w, generator=g)).to(dev)
    skip = to_nhwc(torch.randn(B, 64, 2 * h, 2 * w, generator=g)).to(dev) if with_skip else None
    outs = []
    for form in ("1", "0"):
        monkeypatch.setenv("FVC_UP2_Q16", form)
        outs.append(K.upsample2x_add(src, skip, align_corners=False, scale=1.0))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = dvc_ref.up2(from_nhwc(src.cpu(), 64), False)
    if skip is not None:
        ref = from_nhwc(skip.cpu(), 64) + ref
    close(from_nhwc(outs[0].cpu(), 64), ref, 1e-6)


@pytest.mark.parametrize("shape", [(2, 3, 17, 29), (1, 2, 64, 96), (3, 1, 5, 3), (1, 4, 2, 1), (1, 6, 8, 8)])
def test_nchw_to_nhwc(dev, shape):
    """The boundary layout conversion: NCHW -> NHWC padded to a multiple of 4 channels (pad = 0);
    C <= 4 into 4 channels takes the 16-B-store kernel (k_nchw_to_nhwc4), the rest the generic one."""
    x = torch.randn(*shape)
    y = K.nchw_to_nhwc(x.to(dev)).cpu()
    B, C, H, W = shape
    cp = (C + 3) // 4 * 4
    ref = torch.zeros(B, H, W, cp)
    ref[..., :C] = x.permute(0, 2, 3, 1)
    assert torch.equal(y, ref)


def test_avgpool(dev):
    x = torch.randn(2, 64, 18, 34)
    y = K.avgpool2(to_nhwc(x).to(dev))
    close(from_nhwc(y.cpu(), 64), F.avg_pool2d(x, 2, 2), 1e-6)


def test_upsample_avgpool_tall(dev):
    # more output rows than one grid dimension holds (65535): the row loop strides past it
    g = torch.Generator().manual_seed(4)
    src = torch.randn(1, 3, 33000, 3, generator=g)
    skip = torch.randn(1, 3, 66000, 6, generator=g)
    y = K.upsample2x_add(to_nhwc(src).to(dev), to_nhwc(skip).to(dev), align_corners=False, scale=2.0)
    close(from_nhwc(y.cpu(), 3), skip + dvc_ref.up2(src, False) * 2.0, 1e-6)
    p = K.avgpool2(to_nhwc(skip).to(dev))
    close(from_nhwc(p.cpu(), 3), F.avg_pool2d(skip, 2, 2), 1e-6)


def test_spynet_assemble(dev):
    g = torch.Generator().manual_seed(3)
    im1, im2 = torch.rand(1, 3, 32, 48, generator=g), torch.rand(1, 3, 32, 48, generator=g)
    fprev = torch.randn(1, 2, 16, 24, generator=g) * 2
    fup = dvc_ref.up2(fprev, False) * 2.0
    ref = torch.cat([im1, dvc_ref.warp(im2, fup), fup], 1)
    fu, x8 = K.spynet_assemble(to_nhwc(im1).to(dev), to_nhwc(im2).to(dev), to_nhwc(fprev).to(dev))
    close(from_nhwc(x8.cpu(), 8), ref, 1e-5)
    close(from_nhwc(fu.cpu(), 2), fup, 1e-6)


@pytest.mark.parametrize("shape", [(1, 32, 48), (3, 18, 26), (2, 2, 2)])
def test_assemble_q_forms_bitexact(dev, shape, monkeypatch):
    """The 32-bit, two-pixels-per-iteration SpyNet / MC assembly kernels (FVC_ASSEMBLE_Q=1, the
    default: magic-number pixel division, branch-free clamped taps) equal the 64-bit kernels bit
    for bit, with flows large enough that most taps clamp at the border (odd pixel counts leave
    one thread a single pixel)."""
    B, H, W = shape
    g = torch.Generator().manual_seed(11)
    im1 = to_nhwc(torch.rand(B, 3, H, W, generator=g)).to(dev)
    im2 = to_nhwc(torch.rand(B, 3, H, W, generator=g)).to(dev)
    fprev = to_nhwc(torch.randn(B, 2, H // 2, W // 2, generator=g) * 3 * W).to(dev)
    mv = to_nhwc(torch.randn(B, 2, H, W, generator=g) * 2 * W).to(dev)
    outs = []
    for form in ("0", "1"):
        monkeypatch.setenv("FVC_ASSEMBLE_Q", form)
        outs.append(K.spynet_assemble(im1, im2, fprev) + K.mc_assemble(im1, mv) + K.spynet_assemble(im1, im2, None))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("inverse", [False, True])
def test_gdn(dev, seeded_sd, inverse):
    from fastvideocodec_amd.net import _GDNP
    g = torch.Generator().manual_seed(4)
    x = torch.randn(1, 64, 12, 20, generator=g) * 3
    p = _GDNP(64, inverse).to(dev)
    with torch.no_grad():
        p.beta.copy_(torch.rand(64, generator=g) + 0.5)
        p.gamma.copy_(torch.rand(64, 64, generator=g) * 0.1)
    sd = {"t.beta": p.beta.cpu(), "t.gamma": p.gamma.cpu()}
    ref = dvc_ref.gdn(sd, "t", x, inverse)
    b, gm = p.effective()
    y = K.gdn(to_nhwc(x).to(dev), b, gm, inverse)
    close(from_nhwc(y.cpu(), 64), ref, 2e-6)


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("shape", [(1, 12, 20), (2, 13, 22), (3, 1, 31), (1, 37, 65)])
def test_gdn_x3_vs_fp32_and_float64(dev, shape, inverse, monkeypatch):
    """The split-precision GDN kernel (k_gdn_x3: norm on fp16 hi/lo MFMAs) against float64 torch
    (GDN.py:63-93) and against the fp32-MFMA kernel (FVC_GDN_X3=0) at ragged pixel counts (groups
    of 32 cut anywhere), with off-diagonal gamma entries 6 orders of magnitude below the diagonal;
    a 5000-valued input (x^2 = 2.5e7, past the fp16 range unscaled) is taken by the per-pixel
    power-of-two scale with no flag."""
    B, H, W = shape
    g = torch.Generator().manual_seed(H * W + int(inverse))
    x = torch.randn(B, 64, H, W, generator=g) * 3
    beta = torch.rand(64, generator=g) + 0.5
    gamma = torch.rand(64, 64, generator=g) * 1e-7 + torch.eye(64) * 0.1
    gamma[5, :] = torch.rand(64, generator=g) * 0.02
    big = x.clone()
    big.view(-1)[(B * 64 * H * W) // 2] = 5000.0
    for xin in (x, big):
        norm = torch.sqrt(F.conv2d(xin.double() ** 2, gamma.double()[:, :, None, None], beta.double()))
        ref = xin.double() * norm if inverse else xin.double() / norm
        outs = {}
        for flag in ("1", "0"):
            monkeypatch.setenv("FVC_GDN_X3", flag)
            outs[flag] = from_nhwc(K.gdn(to_nhwc(xin).to(dev), beta.to(dev), gamma.to(dev).contiguous(),
                                         inverse).cpu(), 64).double()
        scale = float(ref.abs().max())
        e3 = float((outs["1"] - ref).abs().max())
        e32 = float((outs["0"] - ref).abs().max())
        print(f"{shape} inv={inverse} big={xin is big}: x3 {e3 / scale:.2e}, fp32 {e32 / scale:.2e} of scale")
        assert e3 <= 1e-6 * scale and e3 <= 4 * e32 + 1e-7 * scale, (e3, e32, scale)


@pytest.mark.parametrize("inverse", [False, True])
def test_gdn_x3_small_activations_small_beta(dev, inverse, monkeypatch):
    """small activations (|x| ~ 1e-2 .. 1e-4, so x^2 is far below the fp16 normal range
    without a scale) with a small beta (1e-3 .. 1e-6, compressai's beta_min is 1e-6): the norm is
    dominated by the gamma . x^2 term, and its relative error must stay at the split-precision
    level (per-pixel power-of-two scale) -- compared elementwise against float64, relative to each
    output value, not to the tensor's max."""
    g = torch.Generator().manual_seed(1234 + int(inverse))
    B, H, W = 2, 13, 37
    x = torch.randn(B, 64, H, W, generator=g) * 1e-2
    x[:, :, :, :9] *= 1e-2  # some pixels two orders of magnitude smaller still
    beta = torch.rand(64, generator=g) * 1e-3 + 1e-6
    gamma = torch.rand(64, 64, generator=g) * 0.05 + torch.eye(64) * 0.5
    norm = torch.sqrt(F.conv2d(x.double() ** 2, gamma.double()[:, :, None, None], beta.double()))
    ref = x.double() * norm if inverse else x.double() / norm
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("FVC_GDN_X3", flag)
        outs[flag] = from_nhwc(K.gdn(to_nhwc(x).to(dev), beta.to(dev), gamma.to(dev).contiguous(),
                                     inverse).cpu(), 64).double()
    den = ref.abs() + 1e-30
    r3 = float(((outs["1"] - ref).abs() / den).max())
    r32 = float(((outs["0"] - ref).abs() / den).max())
    print(f"small x, small beta, inv={inverse}: max relative error x3 {r3:.2e}, fp32 {r32:.2e}")
    assert r3 <= 2e-6 and r3 <= 4 * r32 + 1e-7, (r3, r32)


def test_gdn_x3_tap_form_vs_fp32_form(dev, monkeypatch):
    """GDN + the next layer's tap partials: the x3 kernel against the fp32-MFMA kernel and float64."""
    g = torch.Generator().manual_seed(77)
    B, H, W = 2, 17, 29
    x = torch.randn(B, 64, H, W, generator=g)
    beta = torch.rand(64, generator=g) + 0.5
    gamma = torch.rand(64, 64, generator=g) * 0.05 + torch.eye(64) * 0.2
    w = torch.randn(64, 3, 5, 5, generator=g) * (1.0 / (64 * 25) ** 0.5)
    b = torch.randn(3, generator=g) * 0.1
    norm = torch.sqrt(F.conv2d(x.double() ** 2, gamma.double()[:, :, None, None], beta.double()))
    ref = F.conv_transpose2d(x.double() * norm, w.double(), b.double(), 2, 2, 1)
    t = K.GdnTap(w, b, 5, 2, True, dev)
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("FVC_GDN_X3", flag)
        K.x3_overflow(reset=True)
        outs[flag] = from_nhwc(t(to_nhwc(x).to(dev), beta.to(dev), gamma.to(dev).contiguous(), True).cpu(), 3)
        torch.cuda.synchronize()
        assert not K.x3_overflow(reset=True)
    scale = float(ref.abs().max())
    e3 = float((outs["1"].double() - ref).abs().max())
    e32 = float((outs["0"].double() - ref).abs().max())
    assert e3 <= 2e-6 * scale and e3 <= 3 * e32 + 1e-7 * scale, (e3, e32, scale)


def test_bits(dev, seeded_sd):
    g = torch.Generator().manual_seed(5)
    feat = torch.randn(1, 96, 8, 12, generator=g) * 4
    sigma = torch.exp(torch.randn(1, 96, 8, 12, generator=g))
    ref = float(dvc_ref.bits_laplace(torch.round(feat), sigma))
    got = float(K.bits_laplace(to_nhwc(feat).to(dev), to_nhwc(sigma).to(dev), 96).cpu())
    assert abs(got - ref) <= 1e-4 * abs(ref)
    from fastvideocodec_amd.net import BitEstimator
    be = BitEstimator(128)
    be.load_state_dict({k[len("bitEstimator_mv."):]: v for k, v in seeded_sd.items() if k.startswith("bitEstimator_mv.")})
    v = torch.randn(1, 128, 8, 12, generator=g) * 5
    ref = float(dvc_ref.bits_factorized(seeded_sd, "bitEstimator_mv", torch.round(v)))
    got = float(K.bits_factorized(to_nhwc(v).to(dev), be.params().to(dev), 128).cpu())
    assert abs(got - ref) <= 1e-4 * abs(ref)


def test_recon_finalize(dev):
    g = torch.Generator().manual_seed(6)
    r, x, w, p = (torch.rand(2, 3, 16, 24, generator=g) * 1.4 - 0.2 for _ in range(4))
    clipped, sse = K.recon_finalize(*(to_nhwc(t).to(dev) for t in (r, x, w, p)))
    assert torch.equal(clipped.cpu(), r.clamp(0, 1))
    assert sse.shape == (4,)
    for i, t in enumerate((r, w, p, r.clamp(0, 1))):
        assert abs(float(sse[i]) - float(((t.double() - x.double()) ** 2).sum())) < 1e-9 * float(((t - x) ** 2).sum()) + 1e-6


def test_symbols_and_indexes(dev):
    g = torch.Generator().manual_seed(8)
    lat = torch.randn(2, 96, 6, 10, generator=g) * 7
    sym = K.latent_to_symbols(to_nhwc(lat).to(dev), 96).cpu()
    assert torch.equal(sym, torch.round(lat).to(torch.int32).view(2, 96, 60))
    back = K.symbols_to_latent(sym.to(dev), 6, 10, 96).cpu()
    assert torch.equal(from_nhwc(back, 96), torch.round(lat))
    sigma = torch.exp(torch.randn(2, 96, 6, 10, generator=g) * 2)
    table = EM.get_scale_table()
    idx = K.build_indexes(to_nhwc(sigma).to(dev), table.to(dev), 96).cpu().numpy()
    ref = R.build_indexes(sigma.numpy(), table.numpy()).reshape(2, 96, 60)
    assert (idx == ref).all()


def _rand_streams(S, n, ntab, rng, escapes=True):
    sym = np.round(rng.laplace(0, 3, (S, n))).astype(np.int32)
    if escapes:
        k = max(1, S * n // 50)
        sym.flat[rng.integers(0, S * n, k)] = rng.integers(-70000, 70000, k)
    idx = rng.integers(0, ntab, (S, n)).astype(np.int32)
    return sym, idx


def test_rans_device_vs_oracle(dev):
    rng = np.random.default_rng(11)
    lt = EM.LaplaceTables()
    coder = EM.RangeCoder(lt.cdf, lt.cdf_length, lt.offset, dev)
    for S, n in [(1, 1), (3, 257), (37, 500)]:
        sym, idx = _rand_streams(S, n, 64, rng)
        enc = coder.encode(torch.from_numpy(sym).to(dev), torch.from_numpy(idx).to(dev))
        strings = enc.to_bytes_list()
        for s in range(S):
            assert strings[s] == R.CRef.encode(sym[s], idx[s], lt.cdf, lt.cdf_length, lt.offset)
        dec = coder.decode(enc, torch.from_numpy(idx).to(dev)).cpu().numpy()
        assert (dec == sym).all()


@pytest.mark.parametrize("spb", [1, 7, 16, 64])
def test_rans_decode_streams_per_block(dev, spb, monkeypatch):
    """fvc_rans_decode with 1..64 streams per block (ragged last block) decodes the same symbols;
    the pipeline's throughput setting (64) and the latency default (16) included."""
    rng = np.random.default_rng(40 + spb)
    lt = EM.LaplaceTables()
    coder = EM.RangeCoder(lt.cdf, lt.cdf_length, lt.offset, dev)
    sym, idx = _rand_streams(45, 700, 64, rng)
    enc = coder.encode(torch.from_numpy(sym).to(dev), torch.from_numpy(idx).to(dev))
    monkeypatch.setitem(K._STATE, "rans_spb", spb)
    dec = coder.decode(enc, torch.from_numpy(idx).to(dev)).cpu().numpy()
    assert (dec == sym).all()
    with K.rans_throughput():
        assert K.rans_streams_per_block() == 64
    assert K.rans_streams_per_block() == spb


def test_rans_compressai_api(dev):
    rng = np.random.default_rng(12)
    ft_prm = rng.normal(0, 0.01, (11, 8)).astype(np.float32)
    ft = EM.FactorizedTables(ft_prm)
    cdfs = [list(ft.cdf[i, : ft.cdf_length[i]]) for i in range(8)]
    sym = list(np.round(rng.normal(0, 20, 300)).astype(int))
    idx = list(rng.integers(0, 8, 300))
    s = EM.RansEncoder(dev).encode_with_indexes(sym, idx, cdfs, list(ft.cdf_length), list(ft.offset))
    assert s == R.rans_encode_py(sym, idx, ft.cdf, ft.cdf_length, ft.offset)
    assert EM.RansDecoder(dev).decode_with_indexes(s, idx, cdfs, list(ft.cdf_length), list(ft.offset)) == sym


def test_rans_decode_tails_and_escapes(dev):
    """Factorized per-channel streams with heavy tails + escapes, and wide Laplace symbols."""
    rng = np.random.default_rng(13)
    ft = EM.FactorizedTables(rng.normal(0, 0.01, (11, 8)).astype(np.float32))
    coder = EM.RangeCoder(ft.cdf, ft.cdf_length, ft.offset, dev)
    S, n = 40, 700
    sym = np.round(rng.normal(0, 25, (S, n))).astype(np.int32)
    sym.flat[rng.integers(0, S * n, 60)] = rng.integers(-5000, 5000, 60)
    idx = np.repeat((np.arange(S) % 8)[:, None], n, 1).astype(np.int32)
    enc = coder.encode(torch.from_numpy(sym).to(dev), torch.from_numpy(idx).to(dev))
    assert (coder.decode(enc, torch.from_numpy(idx).to(dev)).cpu().numpy() == sym).all()
    lt = EM.LaplaceTables()
    lc = EM.RangeCoder(lt.cdf, lt.cdf_length, lt.offset, dev)
    sym = np.round(rng.laplace(0, 60, (S, n))).astype(np.int32)
    idx = rng.integers(0, 64, (S, n)).astype(np.int32)
    enc = lc.encode(torch.from_numpy(sym).to(dev), torch.from_numpy(idx).to(dev))
    assert (lc.decode(enc, torch.from_numpy(idx).to(dev)).cpu().numpy() == sym).all()


@pytest.mark.parametrize("shape", [(2, 32, 16, 7, 20, 67), (1, 16, 16, 3, 13, 31), (3, 32, 16, 5, 9, 95)])
def test_conv_pair_tap_form(dev, shape, monkeypatch):
    """16-output-channel convs in pair-tap form (SpyNet conv4, endecoder.py:155: rows 16-31 of the
    MFMA tile carry the odd tap of each (ky, even kx) pair, added from the next lane; 31 output columns
    per 32-pixel strip) against float64 torch and against the plain padded-N form (FVC_X3_PT=0);
    widths cut at every strip edge."""
    B, cin, cout, k, H, W = shape
    g = torch.Generator().manual_seed(cin + k + W)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), 1, k // 2))
    xd = to_nhwc(x).to(dev)
    outs = {}
    for pt in ("1", "0"):
        monkeypatch.setenv("FVC_X3_PT", pt)
        pc = K.PackedConv(w, b, k, 1, False, dev, precision="x3")
        assert pc.x3
        outs[pt] = pc(xd, act=K.ACT_RELU)
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    e1 = float((from_nhwc(outs["1"].cpu(), cout).double() - ref).abs().max())
    e0 = float((from_nhwc(outs["0"].cpu(), cout).double() - ref).abs().max())
    print(f"{shape}: pair-tap err {e1 / scale:.2e}, padded-N err {e0 / scale:.2e} (of output scale)")
    assert e1 <= 2e-6 * scale, (e1, e0, scale)
