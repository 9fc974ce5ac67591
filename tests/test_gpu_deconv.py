"""The all-classes stride-2 transposed conv (fvc_deconv_x3.hip) against float64 torch
conv_transpose2d (the ATen calls of synthesis_mv.py:15-41, synthesis.py:14-27 and the hyperprior
decoder) and against the per-class conv_x3_kernel path (FVC_DX=0): the production geometries plus
ragged sizes (tile rows, 32-column groups and images cut at every edge), every in_op, activation,
residual and exp, the static and dynamic schedules, determinism and the overflow flag."""
import pytest
import torch
import torch.nn.functional as F

from fastvideocodec_amd import _lib
from fastvideocodec_amd import kernels as K

pytestmark = pytest.mark.gpu


def to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def from_nhwc(y, c):
    return y[..., :c].permute(0, 3, 1, 2).contiguous()


# (cin, cout, k, B, H, W, in_op, act, with_res, post)
CASES = [
    (128, 128, 3, 2, 5, 9, K.IN_ROUND, K.ACT_LRELU, False, K.POST_NONE),   # mvDecoder deconv1 (rounded latents)
    (128, 128, 3, 1, 34, 70, K.IN_NONE, K.ACT_RELU, False, K.POST_NONE),   # 2 column groups + 6 cut columns
    (128, 128, 3, 3, 7, 33, K.IN_RELU, K.ACT_NONE, True, K.POST_NONE),     # odd rows, 3 cut columns
    (128, 128, 3, 1, 19, 47, K.IN_NONE, K.ACT_LRELU, False, K.POST_NONE),  # 8-row items cut at 3 rows
    (96, 64, 5, 2, 4, 6, K.IN_ROUND, K.ACT_NONE, False, K.POST_NONE),      # resDecoder deconv1
    (64, 64, 5, 2, 17, 30, K.IN_NONE, K.ACT_RELU, False, K.POST_NONE),     # hyperprior deconv, 17 rows
    (64, 64, 5, 1, 35, 66, K.IN_ABS, K.ACT_NONE, True, K.POST_NONE),
    (64, 128, 3, 2, 6, 40, K.IN_NONE, K.ACT_NONE, False, K.POST_EXP),
]


def _ref(x, w, b, k, in_op, act, res, post):
    xin = {K.IN_NONE: x, K.IN_RELU: F.relu(x), K.IN_ABS: x.abs(), K.IN_ROUND: torch.round(x)}[in_op]
    y = F.conv_transpose2d(xin.double(), w.double(), b.double(), 2, k // 2, 1)
    y = {K.ACT_NONE: y, K.ACT_RELU: F.relu(y), K.ACT_LRELU: F.leaky_relu(y, 0.1)}[act]
    if res is not None:
        y = y + res.double()
    if post == K.POST_EXP:
        y = torch.exp(y)
    return y


def _pack(w, b, k, dev, monkeypatch, dx):
    monkeypatch.setenv("FVC_DX", "1" if dx else "0")
    pc = K.PackedConv(w, b, k, 2, True, dev, precision="x3")
    assert pc.x3
    return pc


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"ci{c[0]}co{c[1]}k{c[2]}b{c[3]}_{c[4]}x{c[5]}")
def test_deconv_all_classes_vs_float64_and_per_class(dev, case, monkeypatch):
    cin, cout, k, B, H, W, in_op, act, with_res, post = case
    lib = _lib.load()
    assert lib.fvc_deconv_x3_all_classes(cin, cout, k, 2) == 1
    g = torch.Generator().manual_seed(cin * 7 + cout + k + H)
    x = torch.randn(B, cin, H, W, generator=g) * (2.0 if post != K.POST_EXP else 0.5)
    w = torch.randn(cin, cout, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5) * (1.0 if post != K.POST_EXP else 0.3)
    b = torch.randn(cout, generator=g) * 0.1
    res = torch.randn(B, cout, 2 * H, 2 * W, generator=g) if with_res else None
    ref = _ref(x, w, b, k, in_op, act, res, post)
    xd = to_nhwc(x).to(dev)
    rd = None if res is None else to_nhwc(res).to(dev)
    outs = {}
    for dx in (True, False):
        pc = _pack(w, b, k, dev, monkeypatch, dx)
        K.x3_overflow(reset=True)
        outs[dx] = pc(xd, in_op=in_op, act=act, post=post, res=rd)
        torch.cuda.synchronize()
        assert not K.x3_overflow(reset=True)
    scale = float(ref.abs().max())
    e_dx = float((from_nhwc(outs[True].cpu(), cout).double() - ref).abs().max())
    e_pc = float((from_nhwc(outs[False].cpu(), cout).double() - ref).abs().max())
    print(f"{case}: all-classes err {e_dx / scale:.2e}, per-class err {e_pc / scale:.2e} (of output scale)")
    # split-precision accuracy (test_gpu_kernels: x3 3-4e-7 of scale); same products as the
    # per-class path, summed in another order
    assert e_dx <= 2e-6 * scale, (e_dx, e_pc, scale)
    assert e_dx <= 3 * e_pc + 1e-7 * scale
    if K.cp4(cout) > cout:
        assert float(outs[True][..., cout:].abs().max()) == 0.0


def test_deconv_all_classes_schedules_and_determinism(dev, monkeypatch):
    """Dynamic (counter) and static item schedules, a CU reserve and repeated launches give
    identical bits; the schedule scratch is left zeroed."""
    g = torch.Generator().manual_seed(3)
    w = torch.randn(128, 128, 3, 3, generator=g) * 0.03
    b = torch.randn(128, generator=g) * 0.1
    pc = _pack(w, b, 3, dev, monkeypatch, True)
    x = to_nhwc(torch.randn(3, 128, 41, 100, generator=g)).to(dev)
    a = pc(x, act=K.ACT_RELU)
    a2 = pc(x, act=K.ACT_RELU)
    monkeypatch.setenv("FVC_X3_DYN", "0")
    c = pc(x, act=K.ACT_RELU)
    monkeypatch.setenv("FVC_X3_RESERVE", "100")
    d = pc(x, act=K.ACT_RELU)
    # wave-tiles paired on SIMD partners or dealt one by one: the same sums per output
    monkeypatch.setenv("FVC_DX_PAIR", "0")
    e = pc(x, act=K.ACT_RELU)
    monkeypatch.setenv("FVC_DX_PAIR", "1")
    f = pc(x, act=K.ACT_RELU)
    torch.cuda.synchronize()
    assert torch.equal(a, a2) and torch.equal(a, c) and torch.equal(a, d)
    assert torch.equal(a, e) and torch.equal(a, f)
    assert int(K.sched_scratch(dev)[:2].abs().sum()) == 0


def test_deconv_all_classes_batch_split(dev, monkeypatch):
    """The >= 4 GB output split (forced low with FVC_X3_SPLIT_BYTES) cuts the batch into launches
    with the same per-image results."""
    g = torch.Generator().manual_seed(4)
    w = torch.randn(64, 64, 5, 5, generator=g) * 0.03
    pc = _pack(w, torch.zeros(64), 5, dev, monkeypatch, True)
    x = to_nhwc(torch.randn(5, 64, 12, 40, generator=g)).to(dev)
    a = pc(x)
    monkeypatch.setenv("FVC_X3_SPLIT_BYTES", str(2 * 24 * 80 * 64 * 4))
    c = pc(x)
    torch.cuda.synchronize()
    assert torch.equal(a, c)


def test_deconv_all_classes_overflow_flag(dev, monkeypatch):
    """An input >= 65000 cannot be split into fp16 halves: the kernel raises the stream's flag."""
    g = torch.Generator().manual_seed(8)
    w = torch.randn(128, 128, 3, 3, generator=g) * 0.03
    pc = _pack(w, torch.zeros(128), 3, dev, monkeypatch, True)
    x = torch.randn(1, 128, 9, 20, generator=g)
    K.x3_overflow(reset=True)
    pc(to_nhwc(x).to(dev))
    assert not K.x3_overflow(reset=True)
    x[0, 77, 4, 13] = 7e4
    pc(to_nhwc(x).to(dev))
    assert K.x3_overflow(reset=True)


def test_pack_layout_switch_refused(dev, monkeypatch):
    """an x3 pack launched after a layout switch flipped (FVC_DX here: the all-classes
    pack has one full-channel chunk, the per-class pack 32-channel chunks) is refused instead of
    running on a pack of another layout; flipping back makes it usable again."""
    from fastvideocodec_amd import _lib
    g = torch.Generator().manual_seed(11)
    w = torch.randn(128, 128, 3, 3, generator=g) * 0.03
    pc = _pack(w, torch.zeros(128), 3, dev, monkeypatch, True)
    x = to_nhwc(torch.randn(1, 128, 8, 16, generator=g)).to(dev)
    a = pc(x)
    monkeypatch.setenv("FVC_DX", "0")
    with pytest.raises(_lib.FvcError):
        pc(x)
    with pytest.raises(_lib.FvcError):  # and again: the refusal is not cached away
        pc(x)
    monkeypatch.setenv("FVC_DX", "1")
    b = pc(x)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
