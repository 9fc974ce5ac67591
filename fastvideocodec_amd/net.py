"""DVC P-frame codec (``DVC/net.py:VideoCompressor``) on the libfvc HIP kernels.

Module tree, parameter names and shapes mirror the reference exactly
(``DVC/net.py:38-57`` and ``DVC/subnet/*``) so ``state_dict``s are interchangeable; the
forward is a straight-line schedule of HIP kernels over NHWC activations:

  SpyNet (4 levels x [assemble, 5 conv7x7])  -> estmv
  mvEncoder (8 conv3x3)                      -> mvfeature        (round fused downstream)
  mvDecoder (4 deconv + 4 conv, in_op=round) -> quant_mv_upsample
  mc_assemble + Warp_net (13 conv3x3, pool/upsample skips) + warpframe -> prediction
  resEncoder (conv5x5 s2 + GDN) x4           -> feature
  respriorEncoder (abs fused) / respriorDecoder (round fused, exp fused) -> recon_sigma
  resDecoder (deconv5x5 s2 + IGDN, round fused, + prediction fused) -> recon
  recon_finalize (clamp + 3 SSE reductions), Laplace/BitEstimator bit reductions.

``forward`` returns the reference 8-tuple. ``compress``/``decompress`` add the real range
coder (the reference's DVC path only estimates bits unless ``calrealbits``, net.py:57).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn
from torch.nn import Parameter

from . import kernels as K
from . import torchac as TAC
from ._lib import FvcError
from .entropy_models import FactorizedTables, LaplaceTables, RangeCoder, get_scale_table
from .weights import OUT_CHANNEL_M, OUT_CHANNEL_MV, OUT_CHANNEL_N


# ------------------------------------------------------------------ parameter holders
class _ConvP(nn.Module):
    """Parameters of an nn.Conv2d / nn.ConvTranspose2d (same names/shapes as torch)."""

    def __init__(self, cin, cout, k, stride=1, transposed=False, bias=True):
        super().__init__()
        shape = (cin, cout, k, k) if transposed else (cout, cin, k, k)
        self.weight = Parameter(torch.zeros(shape), requires_grad=False)
        # bias=False: no `bias` entry in the state_dict (nn.Conv2d(..., bias=False)); the kernels
        # get a zero bias vector
        self.bias = Parameter(torch.zeros(cout), requires_grad=False) if bias else None
        self.cout = cout
        self.k, self.stride, self.transposed = k, stride, transposed
        self._packed = {}

    def _bias(self):
        return self.bias if self.bias is not None else torch.zeros(self.cout, device=self.weight.device)

    def packed(self) -> K.PackedConv:
        """The weight pack for the active conv precision (x3 by default; f32 when a frame is
        recomputed after a split-precision overflow), built once per precision."""
        p = K.conv_precision()
        if p not in self._packed:
            self._packed[p] = K.PackedConv(self.weight, self._bias(), self.k, self.stride, self.transposed,
                                           self.weight.device, precision=p)
        return self._packed[p]

    def tap_consumer(self):
        """This (cout <= 4) layer in tap-partial form for fusion into its producer (cached), or
        None when it has more than 32 partials (k*k*cout)."""
        if "tap" not in self._packed:
            try:
                self._packed["tap"] = K.TapConsumer(self.weight, self._bias(), self.k, self.stride, self.transposed,
                                                    self.weight.device)
            except ValueError:
                self._packed["tap"] = None
        return self._packed["tap"]

    def gdn_tap(self):
        """This (cout <= 4, 64-input) layer fused behind a GDN kernel (cached)."""
        if "gdntap" not in self._packed:
            self._packed["gdntap"] = K.GdnTap(self.weight, self._bias(), self.k, self.stride, self.transposed,
                                              self.weight.device)
        return self._packed["gdntap"]

    def invalidate(self):
        self._packed = {}


def conv_then_tap(prod: _ConvP, x, cons: _ConvP, act=K.ACT_NONE, res=None, cons_act=K.ACT_NONE,
                  cons_res=None):
    """cons(prod(x, act, res), cons_act, cons_res) for a cout <= 4 consumer: on the split-precision
    path the consumer's 1x1 tap-partial GEMM runs in the producer's epilogue (the producer's
    output never reaches HBM; fvc_conv2d_nhwc_x3_tap + fvc_tap_gather_nhwc), else two layers.
    FVC_TAP_FUSE=0 disables the fusion (A/B and tests)."""
    p = prod.packed()
    if K.conv_precision() == "x3" and os.environ.get("FVC_TAP_FUSE", "1") != "0":
        t = cons.tap_consumer()
        if t is not None and p.tap_fusable(t):
            return t.gather(p.call_tap(x, t, act=act, res=res), act=cons_act, res=cons_res)
    return cons.packed()(p(x, act=act, res=res), act=cons_act, res=cons_res)


class _GDNP(nn.Module):
    """GDN parameters (GDN.py:45-61) and their effective values (GDN.py:75-84)."""

    def __init__(self, ch, inverse=False):
        super().__init__()
        self.inverse = inverse
        self.beta = Parameter(torch.ones(ch), requires_grad=False)
        self.gamma = Parameter(torch.eye(ch), requires_grad=False)
        self._eff = None

    def effective(self):
        if self._eff is None:
            pedestal = np.float32((2.0 ** -18) ** 2)
            beta_bound = np.float32((1e-6 + float(pedestal)) ** 0.5)
            gamma_bound = np.float32(2.0 ** -18)
            b = self.beta.detach().cpu().numpy().astype(np.float32)
            g = self.gamma.detach().cpu().numpy().astype(np.float32)
            b = np.maximum(b, beta_bound) ** 2 - pedestal
            g = np.maximum(g, gamma_bound) ** 2 - pedestal
            dev = self.beta.device
            self._eff = (torch.from_numpy(b.astype(np.float32)).to(dev),
                         torch.from_numpy(np.ascontiguousarray(g, np.float32)).to(dev))
        return self._eff

    def invalidate(self):
        self._eff = None


class Bitparm(nn.Module):
    def __init__(self, channel, final=False):
        super().__init__()
        self.final = final
        self.h = Parameter(torch.zeros(1, channel, 1, 1), requires_grad=False)
        self.b = Parameter(torch.zeros(1, channel, 1, 1), requires_grad=False)
        self.a = None if final else Parameter(torch.zeros(1, channel, 1, 1), requires_grad=False)


class BitEstimator(nn.Module):
    """bitEstimator.py:27-42 parameters; evaluated by fvc_bits_factorized / the CDF tables."""

    def __init__(self, channel):
        super().__init__()
        self.channel = channel
        self.f1, self.f2, self.f3 = Bitparm(channel), Bitparm(channel), Bitparm(channel)
        self.f4 = Bitparm(channel, True)

    def params(self) -> torch.Tensor:
        rows = []
        for f in (self.f1, self.f2, self.f3):
            rows += [f.h.view(-1), f.b.view(-1), f.a.view(-1)]
        rows += [self.f4.h.view(-1), self.f4.b.view(-1)]
        return torch.stack(rows, 0).detach().contiguous()


# ------------------------------------------------------------------ sub-networks
class MEBasic(nn.Module):
    """endecoder.py:142-169: 5x conv7x7 8->32->64->32->16->2."""

    def __init__(self):
        super().__init__()
        ch = [8, 32, 64, 32, 16, 2]
        for i in range(5):
            setattr(self, f"conv{i+1}", _ConvP(ch[i], ch[i + 1], 7))

    def run(self, x8, flow_up):
        x = self.conv1.packed()(x8, act=K.ACT_RELU)
        x = self.conv2.packed()(x, act=K.ACT_RELU)
        x = self.conv3.packed()(x, act=K.ACT_RELU)
        x = self.conv4.packed()(x, act=K.ACT_RELU)
        return self.conv5.packed()(x, res=flow_up)  # flow = flow_up + MEBasic(...) (endecoder.py:354)


class ME_Spynet(nn.Module):
    """endecoder.py:312-356."""

    def __init__(self):
        super().__init__()
        self.L = 4
        self.moduleBasic = nn.ModuleList([MEBasic() for _ in range(4)])

    def run(self, im1, im2):
        im1l, im2l = [im1], [im2]
        for lvl in range(self.L - 1):
            im1l.append(K.avgpool2(im1l[lvl]))
            im2l.append(K.avgpool2(im2l[lvl]))
        flow = None  # zeros at 1/16 (endecoder.py:348-351)
        for lvl in range(self.L):
            i = self.L - 1 - lvl
            flow_up, x8 = K.spynet_assemble(im1l[i], im2l[i], flow)
            flow = self.moduleBasic[lvl].run(x8, flow_up)
        return flow


class Analysis_mv_net(nn.Module):
    """analysis_mv.py:8-66."""

    def __init__(self):
        super().__init__()
        mv = OUT_CHANNEL_MV
        for i in range(1, 9):
            setattr(self, f"conv{i}", _ConvP(2 if i == 1 else mv, mv, 3, 2 if i % 2 == 1 else 1))

    def run(self, x):
        for i in range(1, 9):
            x = getattr(self, f"conv{i}").packed()(x, act=K.ACT_LRELU if i < 8 else K.ACT_NONE)
        return x


class Synthesis_mv_net(nn.Module):
    """synthesis_mv.py:9-79; consumes round(mvfeature) (net.py:76) via in_op=round."""

    def __init__(self):
        super().__init__()
        mv = OUT_CHANNEL_MV
        for i in range(1, 9):
            cout = 2 if i == 8 else mv
            setattr(self, f"deconv{i}", _ConvP(mv, cout, 3, 2 if i % 2 == 1 else 1, transposed=(i % 2 == 1)))

    def run(self, q):
        x = q
        for i in range(1, 7):
            x = getattr(self, f"deconv{i}").packed()(x, in_op=K.IN_ROUND if i == 1 else K.IN_NONE,
                                                     act=K.ACT_LRELU)
        # deconv7 (128 ch at full resolution) feeds only the 128->2 deconv8: fused
        return conv_then_tap(self.deconv7, x, self.deconv8, act=K.ACT_LRELU)


class ResBlock(nn.Module):
    """endecoder.py:228-260 (pre-activation, identity skip: cin == cout)."""

    def __init__(self, ch=64):
        super().__init__()
        self.conv1 = _ConvP(ch, ch, 3)
        self.conv2 = _ConvP(ch, ch, 3)

    def run(self, x):
        y = self.conv1.packed()(x, in_op=K.IN_RELU, act=K.ACT_RELU)
        return self.conv2.packed()(y, res=x)

    def run_pool(self, x):
        """(out, avg_pool2d(out, 2)): the pool (endecoder.py:272,274) comes out of conv2's epilogue
        on the split-precision path (FVC_POOL_FUSE=0: separate kernel)."""
        y = self.conv1.packed()(x, in_op=K.IN_RELU, act=K.ACT_RELU)
        p = self.conv2.packed()
        if os.environ.get("FVC_POOL_FUSE", "1") != "0" and p.pool_fusable():
            return p.call_pool(y, res=x)
        out = p(y, res=x)
        return out, K.avgpool2(out)


class Warp_net(nn.Module):
    """endecoder.py:262-296."""

    def __init__(self):
        super().__init__()
        self.feature_ext = _ConvP(6, 64, 3)
        for i in range(6):
            setattr(self, f"conv{i}", ResBlock(64))
        self.conv6 = _ConvP(64, 3, 3)

    def run(self, x8, warpframe):
        fe = self.feature_ext.packed()(x8, act=K.ACT_RELU)
        c0, p0 = self.conv0.run_pool(fe)
        c1, p1 = self.conv1.run_pool(p0)
        c2 = self.conv2.run(p1)
        c3 = self.conv3.run(c2)
        # c3_u = c1 + up(c3), c4_u = c0 + up(c4) (endecoder.py:288-293): formed inside the ResBlock
        # conv1 that reads them (its staging), which also writes them for conv2's residual
        y, c3u = self._conv1_up(self.conv4, c1, c3)
        c4 = self.conv4.conv2.packed()(y, res=c3u)
        y, c4u = self._conv1_up(self.conv5, c0, c4)
        # c5 = conv5(c4u) feeds only conv6 (64->3): its second conv runs fused with conv6's taps;
        # prediction = warpnet(...) + warpframe (net.py:67)
        return conv_then_tap(self.conv5.conv2, y, self.conv6, res=c4u, cons_res=warpframe)

    @staticmethod
    def _conv1_up(block, skip, low):
        """(relu(conv1(relu(skip + up(low)))), skip + up(low)): one Winograd launch when the conv
        takes the fused input, else the standalone upsample-add then conv1."""
        p = block.conv1.packed()
        if p.up_fusable():
            return p.call_up(skip, low, in_op=K.IN_RELU, act=K.ACT_RELU)
        xs = K.upsample2x_add(low, skip=skip, align_corners=True)
        return p(xs, in_op=K.IN_RELU, act=K.ACT_RELU), xs


class Analysis_net(nn.Module):
    """analysis.py:10-48."""

    def __init__(self):
        super().__init__()
        N, M = OUT_CHANNEL_N, OUT_CHANNEL_M
        cins, couts = [3, N, N, N], [N, N, N, M]
        for i in range(4):
            setattr(self, f"conv{i+1}", _ConvP(cins[i], couts[i], 5, 2))
            if i < 3:
                setattr(self, f"gdn{i+1}", _GDNP(N))

    def run(self, x):
        for i in range(1, 5):
            x = getattr(self, f"conv{i}").packed()(x)
            if i < 4:
                b, g = getattr(self, f"gdn{i}").effective()
                x = K.gdn(x, b, g, False)
        return x


class Synthesis_net(nn.Module):
    """synthesis.py:8-58; input round(feature) via in_op=round; + prediction fused."""

    def __init__(self):
        super().__init__()
        N, M = OUT_CHANNEL_N, OUT_CHANNEL_M
        cins, couts = [M, N, N, N], [N, N, N, 3]
        for i in range(4):
            setattr(self, f"deconv{i+1}", _ConvP(cins[i], couts[i], 5, 2, transposed=True))
            if i < 3:
                setattr(self, f"igdn{i+1}", _GDNP(N, inverse=True))

    def run(self, feature, prediction):
        x = feature
        for i in range(1, 4):
            x = getattr(self, f"deconv{i}").packed()(x, in_op=K.IN_ROUND if i == 1 else K.IN_NONE)
            b, g = getattr(self, f"igdn{i}").effective()
            if i == 3 and K.conv_precision() == "x3" and os.environ.get("FVC_GDN_TAP", "1") != "0":
                # igdn3 feeds only deconv4 (64 -> 3): its 75 tap partials come out of the IGDN
                # kernel and igdn3's output never reaches HBM (FVC_GDN_TAP=0: two launches)
                return self.deconv4.gdn_tap()(x, b, g, True, res=prediction)
            x = K.gdn(x, b, g, True)
        return self.deconv4.packed()(x, res=prediction)


class Analysis_prior_net(nn.Module):
    """analysis_prior.py:10-56 (abs fused into conv1 staging)."""

    def __init__(self):
        super().__init__()
        N, M = OUT_CHANNEL_N, OUT_CHANNEL_M
        self.conv1 = _ConvP(M, N, 3)
        self.conv2 = _ConvP(N, N, 5, 2)
        self.conv3 = _ConvP(N, N, 5, 2)

    def run(self, x):
        x = self.conv1.packed()(x, in_op=K.IN_ABS, act=K.ACT_RELU)
        x = self.conv2.packed()(x, act=K.ACT_RELU)
        return self.conv3.packed()(x)


class Synthesis_prior_net(nn.Module):
    """synthesis_prior.py:11-58 (round(z) fused into deconv1 staging, exp fused into deconv3)."""

    def __init__(self):
        super().__init__()
        N, M = OUT_CHANNEL_N, OUT_CHANNEL_M
        self.deconv1 = _ConvP(N, N, 5, 2, transposed=True)
        self.deconv2 = _ConvP(N, N, 5, 2, transposed=True)
        self.deconv3 = _ConvP(N, M, 3, 1, transposed=True)

    def run(self, z):
        x = self.deconv1.packed()(z, in_op=K.IN_ROUND, act=K.ACT_RELU)
        x = self.deconv2.packed()(x, act=K.ACT_RELU)
        return self.deconv3.packed()(x, post=K.POST_EXP)


# ------------------------------------------------------------------ the codec
FRAMINGS = ("channel", "item", "segment")
# 'segment' framing: each (frame, latent, channel) row of HW symbols is cut into equal contiguous
# segments of >= 512 symbols (a power-of-two count dividing HW), one rANS stream each. A stream's
# decode is one sequential chain of symbols, so the chain length sets a frame's decode latency:
# at 1080p (HW = 68 x 120 = 8160) the mv / feature rows become 8 streams of 1020 symbols. Each
# stream is still exactly compressai's encode_with_indexes of its symbols (T1 parity per stream);
# the cost is one rANS flush (4 bytes) per extra stream.
SEGMENT_MIN = 512


def segments(hw: int) -> int:
    """Streams per (frame, latent, channel) row of hw symbols in the 'segment' framing."""
    s = 1
    while s < 64 and hw % (2 * s) == 0 and hw // (2 * s) >= SEGMENT_MIN:
        s *= 2
    return s


def stream_rows(framing: str, B: int, C: int, hw: int):
    """(streams, symbols per stream) of a [B, C, hw] latent in a framing (symbols are contiguous
    per (frame, channel) row, so every framing is a view of the same memory)."""
    if framing == "item":
        return B, C * hw
    if framing == "segment":
        s = segments(hw)
        return B * C * s, hw // s
    return B * C, hw


def bitstream_rows(framing: str, B: int, C: int, hw: int, nstreams: int):
    """(streams, symbols per stream) of a coded [B, C, hw] latent, read from the stream count the
    bitstream carries rather than re-derived from SEGMENT_MIN / segments(): a file written under
    another segmenting rule still decodes, and a count that cannot cut the rows is rejected."""
    if framing == "segment":
        s = nstreams // max(B * C, 1)
        if s < 1 or s * B * C != nstreams or hw % s:
            raise FvcError(f"segment framing: {nstreams} streams cannot cut {B * C} rows of {hw} symbols")
        return nstreams, hw // s
    rows = stream_rows(framing, B, C, hw)
    if rows[0] != nstreams:
        raise FvcError(f"{framing} framing: expected {rows[0]} streams, bitstream has {nstreams}")
    return rows


class PFrameBitstream:
    """In-memory P-frame bitstream: three latents (mv, z, feature) of ``batch`` frames.

    framing 'segment' (the codec's default): one rANS stream per contiguous segment of a (frame,
    latent, channel) row (stream_rows / segments above); 'channel': one stream per (frame, latent,
    channel), so the decoder runs C-way parallel per frame; 'item': compressai's framing (EntropyModel.compress,
    entropy_models.py:80-86), one stream per (frame, latent) over the whole (C,H,W) latent in C
    order. Either way each stream equals compressai's encode_with_indexes on its symbols.
    precision: the conv precision the encoder's reconstruction used ('x3', or 'f32' when the
    frame was recomputed after a split-precision overflow); the decoder must use the same."""

    def __init__(self, mv, z, feature, batch, hw16, hw64, framing="segment", precision="x3"):
        self.mv, self.z, self.feature = mv, z, feature
        self.batch, self.hw16, self.hw64 = batch, hw16, hw64
        self.framing, self.precision = framing, precision

    def nbytes(self) -> int:
        return int((self.mv.pack_off[-1] + self.z.pack_off[-1] + self.feature.pack_off[-1]).item()) * 4

    def check(self):
        for part in (self.mv, self.z, self.feature):
            part.check()


class VideoCompressor(nn.Module):
    """DVC/net.py:38-220 — same submodule names, same forward contract."""

    def __init__(self):
        super().__init__()
        self.opticFlow = ME_Spynet()
        self.mvEncoder = Analysis_mv_net()
        self.Q = None
        self.mvDecoder = Synthesis_mv_net()
        self.warpnet = Warp_net()
        self.resEncoder = Analysis_net()
        self.resDecoder = Synthesis_net()
        self.respriorEncoder = Analysis_prior_net()
        self.respriorDecoder = Synthesis_prior_net()
        self.bitEstimator_z = BitEstimator(OUT_CHANNEL_N)
        self.bitEstimator_mv = BitEstimator(OUT_CHANNEL_MV)
        self.warp_weight = 0
        self.mxrange = 150
        self.calrealbits = False
        self._coders = None
        self.eval()

    # -- cache invalidation when weights/device change
    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self.invalidate()
        return r

    def load_state_dict(self, *args, **kwargs):
        r = super().load_state_dict(*args, **kwargs)
        self.invalidate()
        return r

    def invalidate(self):
        for m in self.modules():
            if isinstance(m, (_ConvP, _GDNP)):
                m.invalidate()
        self._coders = None
        self._be = None

    def _be_params(self):
        if getattr(self, "_be", None) is None:
            self._be = (self.bitEstimator_z.params(), self.bitEstimator_mv.params())
        return self._be

    # -- entropy coders (EntropyBottleneck/GaussianConditional.update(force=True) analogue)
    def update(self, force=False):
        if self._coders is not None and not force:
            return False
        dev = self.bitEstimator_z.f1.h.device
        bz, bmv = (p.cpu().numpy() for p in self._be_params())
        tz, tmv, tf = FactorizedTables(bz), FactorizedTables(bmv), LaplaceTables()
        self._coders = {
            "z": RangeCoder(tz.cdf, tz.cdf_length, tz.offset, dev),
            "mv": RangeCoder(tmv.cdf, tmv.cdf_length, tmv.offset, dev),
            "feature": RangeCoder(tf.cdf, tf.cdf_length, tf.offset, dev),
            "scale_table": torch.from_numpy(tf.scale_table).to(dev),
            "tables": (tz, tmv, tf),
        }
        return True

    def motioncompensation(self, ref4, mv4):
        """net.py:64-68 on NHWC tensors: returns (prediction, warpframe)."""
        warpframe, x8 = K.mc_assemble(ref4, mv4)
        prediction = self.warpnet.run(x8, warpframe)
        return prediction, warpframe

    @staticmethod
    def _check_frames(input_image, referframe):
        if input_image.dim() != 4 or input_image.shape[1] != 3 or input_image.shape != referframe.shape:
            raise ValueError("expected [B,3,H,W] frames of equal shape")
        B, _, H, W = input_image.shape
        if H % 64 or W % 64:
            raise ValueError(f"H and W must be multiples of 64 (got {H}x{W}); replicate-pad first")
        if not input_image.is_cuda:
            raise ValueError("VideoCompressor runs on the GPU (libfvc); move the model and frames to cuda")

    def _encode_graph(self, input_image, referframe):
        """The full encoder-side forward on NHWC tensors; returns a dict of device tensors."""
        cur4 = K.nchw_to_nhwc(input_image.float().contiguous(), 4)
        ref4 = K.nchw_to_nhwc(referframe.float().contiguous(), 4)
        estmv = self.opticFlow.run(cur4, ref4)
        mvfeature = self.mvEncoder.run(estmv)
        mv_up = self.mvDecoder.run(mvfeature)
        prediction, warpframe = self.motioncompensation(ref4, mv_up)
        residual = K.sub(cur4, prediction)
        feature = self.resEncoder.run(residual)
        z = self.respriorEncoder.run(feature)
        sigma = self.respriorDecoder.run(z)
        recon = self.resDecoder.run(feature, prediction)
        return dict(cur4=cur4, ref4=ref4, estmv=estmv, mvfeature=mvfeature, mv_up=mv_up,
                    prediction=prediction, warpframe=warpframe, feature=feature, z=z, sigma=sigma,
                    recon=recon)

    # -- split-precision overflow: every x3 conv ORs into its stream's flag;
    # a frame that set it is recomputed on the fp32 kernels (on_overflow="recompute", default)
    # or rejected (on_overflow="raise")
    on_overflow = "recompute"

    def _run_checked(self, fn):
        """Run fn() (a frame's encoder-side work on the current stream) and check the stream's
        overflow flag once its work is done: a copy to pinned memory behind the queued kernels,
        then a wait for that copy only. Returns (result, precision used)."""
        if K.conv_precision() == "f32":
            return fn(), "f32"
        K.overflow_flag().zero_()
        out = fn()
        if not K.OverflowProbe().result():
            return out, "x3"
        self.overflow_events = getattr(self, "overflow_events", 0) + 1
        if self.on_overflow == "raise":
            raise FvcError("split-precision conv operand overflow (|activation| >= 65000); "
                           "set on_overflow='recompute' or FVC_CONV_PRECISION=f32")
        with K.precision("f32"):
            return fn(), "f32"

    def forward(self, input_image, referframe, quant_noise_feature=None, quant_noise_z=None,
                quant_noise_mv=None, return_intermediates=False):
        if self.training:
            raise NotImplementedError("training-mode forward (additive quantisation noise) is out of scope")
        self._check_frames(input_image, referframe)
        with torch.no_grad():
            (out, t), self.last_precision = self._run_checked(
                lambda: self._forward_impl(input_image, referframe))
        if return_intermediates:
            return out, t
        return out

    def _forward_impl(self, input_image, referframe):
        t = self._encode_graph(input_image, referframe)
        B, _, H, W = input_image.shape
        clipped, sse = K.recon_finalize(t["recon"], t["cur4"], t["warpframe"], t["prediction"])
        npx = B * H * W
        if self.calrealbits:
            # DVC's real-bits mode (net.py:123-205): lengths of the torchac byte strings of the three
            # latents (one string per tensor, 2*mxrange-bin CDF rows), from the torchac-compatible
            # coder (torchac.py)
            bz, bmv = self._be_params()
            lens = (TAC.laplace_encode(t["feature"], t["sigma"], OUT_CHANNEL_M, self.mxrange),
                    TAC.bitest_encode(t["z"], bz, OUT_CHANNEL_N, self.mxrange),
                    TAC.bitest_encode(t["mvfeature"], bmv, OUT_CHANNEL_MV, self.mxrange))
            bits_f, bits_z, bits_mv = (torch.tensor([8.0 * len(s)], dtype=torch.float64, device=input_image.device)
                                       for s in lens)
        else:
            bz, bmv = self._be_params()
            bits_f = K.bits_laplace(t["feature"], t["sigma"], OUT_CHANNEL_M)
            bits_z = K.bits_factorized(t["z"], bz, OUT_CHANNEL_N)
            bits_mv = K.bits_factorized(t["mvfeature"], bmv, OUT_CHANNEL_MV)
        mse_loss = (sse[0] / (3 * npx)).float()
        warploss = (sse[1] / (3 * npx)).float()
        interloss = (sse[2] / (3 * npx)).float()
        bpp_feature = (bits_f[0] / npx).float()
        bpp_z = (bits_z[0] / npx).float()
        bpp_mv = (bits_mv[0] / npx).float()
        bpp = bpp_feature + bpp_z + bpp_mv
        return (clipped, mse_loss, warploss, interloss, bpp_feature, bpp_z, bpp_mv, bpp), t

    # ---------------------------------------------------------------- real bitstream
    def compress_tensors(self, t, framing="segment") -> PFrameBitstream:
        """Range-code the latents of an encoder pass (NHWC device tensors mvfeature, z, feature,
        sigma). framing: 'segment' (the codec's default: one stream per contiguous >= 512-symbol
        segment of a frame x channel row), 'channel' (one stream per frame x channel) or 'item'
        (compressai's one string per frame per latent)."""
        if framing not in FRAMINGS:
            raise ValueError(f"framing must be one of {FRAMINGS}")
        self.update()
        c = self._coders
        B, H16, W16, _ = t["mvfeature"].shape
        H64, W64 = t["z"].shape[1:3]
        sym_mv = K.latent_to_symbols(t["mvfeature"], OUT_CHANNEL_MV)
        sym_z = K.latent_to_symbols(t["z"], OUT_CHANNEL_N)
        sym_f = K.latent_to_symbols(t["feature"], OUT_CHANNEL_M)
        idx_mv = K.channel_indexes(B, H16 * W16, OUT_CHANNEL_MV, sym_mv.device)
        idx_z = K.channel_indexes(B, H64 * W64, OUT_CHANNEL_N, sym_z.device)
        idx_f = K.build_indexes(t["sigma"], c["scale_table"], OUT_CHANNEL_M)
        # symbols are [B, C, HW] in memory either way: the framing only chooses the stream cut
        rows = lambda C, hw: stream_rows(framing, B, C, hw)  # noqa: E731
        enc_mv = c["mv"].encode(sym_mv.view(rows(OUT_CHANNEL_MV, H16 * W16)), idx_mv.view(rows(OUT_CHANNEL_MV, H16 * W16)))
        enc_z = c["z"].encode(sym_z.view(rows(OUT_CHANNEL_N, H64 * W64)), idx_z.view(rows(OUT_CHANNEL_N, H64 * W64)))
        enc_f = c["feature"].encode(sym_f.view(rows(OUT_CHANNEL_M, H16 * W16)), idx_f.view(rows(OUT_CHANNEL_M, H16 * W16)))
        return PFrameBitstream(enc_mv, enc_z, enc_f, B, (H16, W16), (H64, W64), framing, K.conv_precision())

    def compress(self, input_image, referframe, return_sse=False, framing="segment"):
        """Encode one P-frame: returns (bitstream, clipped_recon[, sse]). The recon is what
        ``decompress`` reproduces bit-for-bit; sse = device doubles {recon, warp, pred} SSE."""
        self._check_frames(input_image, referframe)

        def run():
            t = self._encode_graph(input_image, referframe)
            bs = self.compress_tensors(t, framing)
            clipped, sse = K.recon_finalize(t["recon"], t["cur4"], t["warpframe"], t["prediction"])
            return bs, clipped, sse

        with torch.no_grad():
            (bs, clipped, sse), self.last_precision = self._run_checked(run)
        if return_sse:
            return bs, clipped, sse
        return bs, clipped

    def decode_latents(self, bs: PFrameBitstream, check=True):
        """Entropy-decode a P-frame bitstream into its three quantised latents (NHWC device
        tensors): z -> respriorDecoder -> sigma -> scale indexes -> feature; mv. Needs no
        reference frame, so it can run ahead of the reconstruction chain."""
        self.update()
        c = self._coders
        B = bs.batch
        (H16, W16), (H64, W64) = bs.hw16, bs.hw64
        dev = bs.mv.packed.device
        rows = lambda C, hw, part: bitstream_rows(bs.framing, B, C, hw, part.nstreams)  # noqa: E731
        # stream checks are collected on the device and read once at the end (one host wait per
        # frame instead of two per latent)
        st = [] if check else None
        with torch.no_grad(), K.precision(bs.precision):
            idx_z = K.channel_indexes(B, H64 * W64, OUT_CHANNEL_N, dev)
            sym_z = c["z"].decode(bs.z, idx_z.view(rows(OUT_CHANNEL_N, H64 * W64, bs.z)), check, st).view(B, OUT_CHANNEL_N, H64 * W64)
            z = K.symbols_to_latent(sym_z, H64, W64, OUT_CHANNEL_N)
            sigma = self.respriorDecoder.run(z)
            idx_f = K.build_indexes(sigma, c["scale_table"], OUT_CHANNEL_M)
            sym_f = c["feature"].decode(bs.feature, idx_f.view(rows(OUT_CHANNEL_M, H16 * W16, bs.feature)), check, st).view(B, OUT_CHANNEL_M, H16 * W16)
            feature = K.symbols_to_latent(sym_f, H16, W16, OUT_CHANNEL_M)
            idx_mv = K.channel_indexes(B, H16 * W16, OUT_CHANNEL_MV, dev)
            sym_mv = c["mv"].decode(bs.mv, idx_mv.view(rows(OUT_CHANNEL_MV, H16 * W16, bs.mv)), check, st).view(B, OUT_CHANNEL_MV, H16 * W16)
            mvq = K.symbols_to_latent(sym_mv, H16, W16, OUT_CHANNEL_MV)
        if st and int(torch.cat(st).abs().max()) != 0:
            raise FvcError("corrupt rANS stream (or a failed encode)")
        return {"mv": mvq, "feature": feature, "z": z, "precision": bs.precision}

    def reconstruct(self, lat, referframe):
        """Decoder synthesis from decoded latents: mvDecoder -> motion compensation ->
        resDecoder (+ prediction) -> clamp. Returns the NCHW reconstruction."""
        with torch.no_grad(), K.precision(lat.get("precision")):
            ref4 = K.nchw_to_nhwc(referframe.float().contiguous(), 4)
            mv_up = self.mvDecoder.run(lat["mv"])
            prediction, _ = self.motioncompensation(ref4, mv_up)
            recon = self.resDecoder.run(lat["feature"], prediction)
            return K.nhwc_to_nchw(recon, 3, clamp01=True)

    def decompress(self, bs: PFrameBitstream, referframe, check=True):
        """Decode a P-frame from its bitstream and the reference frame (z -> sigma -> feature;
        mv -> motion compensation; residual synthesis)."""
        return self.reconstruct(self.decode_latents(bs, check), referframe)
