"""RLVC path: the reference's recurrent learned video codec
``IterPredVideoCodecs('RLVC')`` (models.py:954-1051) with ``Coder2D`` (GDN + ConvLSTM
auto-encoder, models.py:520-681) and ``RecProbModel`` (entropy_models.py:26-148: a compressai
``EntropyBottleneck`` for the first P-frame, then the recurrent probability model ``RPM``
(entropy_models.py:328-357) driving a ``GaussianConditional`` with means), on the GPU:

* convolutions: the split-precision conv kernels (``K.PackedConv``); ConvLSTM's 256 -> 512 conv
  runs as 4 gates x (x-part, h-part) convs whose h-part feeds the x-part's residual epilogue (no
  concatenation), then one fused gate kernel (``fvc_lstm_gates``);
* compressai GDN / IGDN (x * rsqrt(norm)) at 128 channels (``fvc_gdn_nhwc_cai``);
* entropy models: eval forward (x_hat + estimated bits) in ``fvc_eb_forward`` /
  ``fvc_gc_forward``; real strings (one per batch item, compressai framing) from the device rANS
  coder through the ``entropy_models`` mirror classes; RPM's sigma transform in ``fvc_rpm_scale``.

Tensors are NHWC on the device. Hidden states are NHWC dicts; ``hidden_to_reference`` /
``hidden_from_reference`` convert to and from the reference's NCHW ``cat(c, h)`` layout. The
reference's decoder applies ``enc_lstm`` to the decoder state (models.py:661) -- reproduced.
Parity: oracle/rlvc_ref.py (CPU restatement; ConvLSTM / RPM pinned by reference-generated
fixtures, tests/golden/rlvc_rpm.npz).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.nn as nn
from torch.nn import Parameter

from . import _lib
from . import kernels as K
from ._lib import FvcError
from .entropy_models import ConditionalEntropyModel, _CompressaiEntropyModel, _pack_tables, get_scale_table
from .net import ME_Spynet, Warp_net, _ConvP, _GDNP

CHANNELS = 128
FILTERS = (3, 3, 3, 3)


def _gdn_cai(x, gdn: _GDNP):
    B, H, W, C = x.shape
    beta, gamma = gdn.effective()
    y = torch.empty_like(x)
    _lib.call("fvc_gdn_nhwc_cai", x.data_ptr(), y.data_ptr(), beta.data_ptr(), gamma.data_ptr(), B, H, W, C,
              int(gdn.inverse), K.stream_handle())
    return y


class ConvLSTM(nn.Module):
    """entropy_models.py:359-378 (conv 2C -> 4C, gates j, i, f, o; forget bias 1; relu)."""

    def __init__(self, channels=CHANNELS, forget_bias=1.0):
        super().__init__()
        self.conv = _ConvP(2 * channels, 4 * channels, 3)
        self._forget_bias = float(forget_bias)
        self._channels = channels
        self._packs = {}

    def invalidate(self):
        self._packs = {}

    def _gate_convs(self):
        """Per gate (x-part, h-part) packs for the active conv precision (cached per precision, so
        a frame recomputed under ``K.precision('f32')`` runs its gates on the fp32 kernels too)."""
        p = K.conv_precision()
        if p not in self._packs:
            C = self._channels
            w, b = self.conv.weight, self.conv.bias
            packs = []
            for g in range(4):
                wg = w[g * C:(g + 1) * C]
                packs.append((K.PackedConv(wg[:, :C].contiguous(), b[g * C:(g + 1) * C], 3, 1, False, w.device,
                                           precision=p),
                              K.PackedConv(wg[:, C:].contiguous(), torch.zeros(C, device=w.device), 3, 1, False,
                                           w.device, precision=p)))
            self._packs[p] = packs
        return self._packs[p]

    def run(self, x, state):
        """x [B,H,W,C]; state {'c', 'h'} -> (h, new state)."""
        gates = [px(x, res=ph(state["h"])) for px, ph in self._gate_convs()]
        c = torch.empty_like(x)
        h = torch.empty_like(x)
        _lib.call("fvc_lstm_gates", gates[0].data_ptr(), gates[1].data_ptr(), gates[2].data_ptr(),
                  gates[3].data_ptr(), state["c"].data_ptr(), c.data_ptr(), h.data_ptr(), x.numel(),
                  self._forget_bias, K.stream_handle())
        return h, {"c": c, "h": h}


class RPM(nn.Module):
    """entropy_models.py:328-357: 4 conv3x3+ReLU, ConvLSTM, 3 conv3x3+ReLU, conv3x3 -> 2C + ReLU."""

    def __init__(self, channels=CHANNELS):
        super().__init__()
        for i in range(1, 8):
            setattr(self, f"conv{i}", _ConvP(channels, channels, 3))
        self.conv8 = _ConvP(channels, 2 * channels, 3)
        self.channels = channels
        self.lstm = ConvLSTM(channels)
        self._split = {}

    def invalidate(self):
        self._split = {}

    def _conv8(self):
        p = K.conv_precision()
        if p not in self._split:
            C, w, b = self.channels, self.conv8.weight, self.conv8.bias
            self._split[p] = tuple(K.PackedConv(w[i * C:(i + 1) * C].contiguous(), b[i * C:(i + 1) * C], 3, 1,
                                                False, w.device, precision=p) for i in range(2))
        return self._split[p]

    def run(self, prior, hidden, round_input=True):
        """prior: the previous frame's latent (rounded here, as entropy_models.py:67 / :122 do
        before it reaches RPM); returns (sigma_raw, mu, hidden)."""
        x = self.conv1.packed()(prior, in_op=K.IN_ROUND if round_input else K.IN_NONE, act=K.ACT_RELU)
        for i in range(2, 5):
            x = getattr(self, f"conv{i}").packed()(x, act=K.ACT_RELU)
        x, hidden = self.lstm.run(x, hidden)
        for i in range(5, 8):
            x = getattr(self, f"conv{i}").packed()(x, act=K.ACT_RELU)
        ps, pm = self._conv8()
        return ps(x, act=K.ACT_RELU), pm(x, act=K.ACT_RELU), hidden


class LearnedEntropyBottleneck(_CompressaiEntropyModel, nn.Module):
    """compressai ``EntropyBottleneck(channels)`` (filters (3,3,3,3), init_scale 10, tail_mass
    1e-9): parameters ``_matrix{i}``, ``_bias{i}``, ``_factor{i}``, ``quantiles``; eval forward on
    the GPU (``fvc_eb_forward``); tables from ``update()`` (Appendix A.1, float32 torch on the
    host, as compressai computes them); compress/decompress with means = medians, table = channel."""

    def __init__(self, channels=CHANNELS, device=None):
        nn.Module.__init__(self)
        _CompressaiEntropyModel.__init__(self, device)
        self.channels = channels
        filters = (1,) + FILTERS + (1,)
        for i in range(len(FILTERS) + 1):
            self.register_parameter(f"_matrix{i}", Parameter(torch.zeros(channels, filters[i + 1], filters[i]),
                                                             requires_grad=False))
            self.register_parameter(f"_bias{i}", Parameter(torch.zeros(channels, filters[i + 1], 1),
                                                           requires_grad=False))
            if i < len(FILTERS):
                self.register_parameter(f"_factor{i}", Parameter(torch.zeros(channels, filters[i + 1], 1),
                                                                 requires_grad=False))
        self.quantiles = Parameter(torch.tensor([-10.0, 0.0, 10.0]).repeat(channels, 1, 1), requires_grad=False)
        self._prm = None

    def invalidate(self):
        self._prm = None
        self._coder = None
        self._aux = None

    def kernel_params(self):
        """[C, 58] softplus(matrices), biases, tanh(factors) + medians [C] (device)."""
        if self._prm is None:
            C = self.channels
            sp = [torch.nn.functional.softplus(getattr(self, f"_matrix{i}").detach().cpu()).reshape(C, -1)
                  for i in range(5)]
            bs = [getattr(self, f"_bias{i}").detach().cpu().reshape(C, -1) for i in range(5)]
            fs = [torch.tanh(getattr(self, f"_factor{i}").detach().cpu()).reshape(C, -1) for i in range(4)]
            prm = torch.cat(sp + bs + fs, 1).float().contiguous()
            assert prm.shape[1] == 58
            dev = self.quantiles.device
            self._prm = (prm.to(dev), self.quantiles[:, 0, 1].detach().float().contiguous().to(dev))
        return self._prm

    def loss(self):
        """compressai ``EntropyBottleneck.loss()``: sum |logits_cumulative(quantiles) - target|,
        target = (-t, 0, t), t = log(2 / tail_mass - 1) (tail_mass 1e-9). A function of the
        parameters only (host, float32, like ``update()``); cached until the weights change."""
        if getattr(self, "_aux", None) is None:
            t = float(np.log(2 / 1e-9 - 1))
            target = torch.tensor([-t, 0.0, t], dtype=torch.float32)
            logits = self._logits_cumulative(self.quantiles.detach().cpu().float())
            self._aux = torch.abs(logits - target).sum().to(self.quantiles.device)
        return self._aux

    def _logits_cumulative(self, inputs):
        logits = inputs
        for i in range(len(FILTERS) + 1):
            logits = torch.matmul(torch.nn.functional.softplus(getattr(self, f"_matrix{i}").detach().cpu()), logits)
            logits = logits + getattr(self, f"_bias{i}").detach().cpu()
            if i < len(FILTERS):
                logits = logits + torch.tanh(getattr(self, f"_factor{i}").detach().cpu()) * torch.tanh(logits)
        return logits

    def update(self, force=False):
        if self._coder is not None and not force:
            return False
        q = self.quantiles.detach().cpu().float()
        medians = q[:, 0, 1]
        minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
        maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
        pmf_start = medians - minima
        pmf_length = maxima + minima + 1
        max_length = int(pmf_length.max())
        samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
        lower = self._logits_cumulative(samples - 0.5)
        upper = self._logits_cumulative(samples + 0.5)
        sign = -torch.sign(lower + upper)
        pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
        tail = (torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:]))[:, 0]
        lengths = pmf_length.numpy().astype(np.int64)
        self._set_tables(_pack_tables(pmf.numpy(), tail.numpy(), lengths), (lengths + 2).astype(np.int32),
                         (-minima).numpy().astype(np.int32))
        return True

    def _build_indexes(self, size):
        return (torch.arange(self.channels, dtype=torch.int32, device=self.device)
                .view(1, -1, *([1] * (len(size) - 2))).expand(size).contiguous())

    def _medians(self, size):
        _, med = self.kernel_params()
        return med.view(1, -1, *([1] * (len(size) - 2))).expand(size)

    def compress(self, x):
        return _CompressaiEntropyModel.compress(self, x, self._build_indexes(x.size()), self._medians(x.size()))

    def decompress(self, strings, size):
        out = (len(strings), self.channels, *size)
        return _CompressaiEntropyModel.decompress(self, strings, self._build_indexes(out), means=self._medians(out))


class RecProbModel(nn.Module):
    """entropy_models.py:26-148 (eval): factorized ``entropy_bottleneck`` when RPM_flag is False,
    else RPM(prior_latent) -> sigma = exp(max(sigma, -7))/10, mu -> GaussianConditional."""

    def __init__(self, channels=CHANNELS):
        super().__init__()
        self.channels = channels
        self.entropy_bottleneck = LearnedEntropyBottleneck(channels)
        self.RPM = RPM(channels)
        self.gaussian_conditional = ConditionalEntropyModel(None, "gaussian")
        self.RPM_flag = False
        self.sigma = self.mu = None

    def set_RPM(self, flag):
        self.RPM_flag = bool(flag)

    def update(self, scale_table=None, force=False):
        dev = self.entropy_bottleneck.quantiles.device
        self.entropy_bottleneck.device = self.gaussian_conditional.device = dev
        updated = self.gaussian_conditional.update_scale_table(
            get_scale_table() if scale_table is None else scale_table, force=force)
        updated |= self.entropy_bottleneck.update(force=force)
        return updated

    def forward_latent(self, x, rpm_hidden, prior_latent):
        """-> (x_hat, estimated bits (device float64 [1]), rpm_hidden, prior_latent)."""
        B, H, W, C = x.shape
        xhat = torch.empty_like(x)
        bits = torch.empty(1, dtype=torch.float64, device=x.device)
        ws = K._ws(x.device)
        if self.RPM_flag:
            if prior_latent is None:
                raise ValueError("prior latent is none!")
            s_raw, mu, rpm_hidden = self.RPM.run(prior_latent, rpm_hidden)
            sigma = torch.empty_like(s_raw)
            _lib.call("fvc_rpm_scale", s_raw.data_ptr(), sigma.data_ptr(), s_raw.numel(), K.stream_handle())
            self.sigma, self.mu = sigma, mu
            _lib.call("fvc_gc_forward", x.data_ptr(), sigma.data_ptr(), mu.data_ptr(), xhat.data_ptr(),
                      bits.data_ptr(), ws.data_ptr(), B, H, W, C, C, K.stream_handle())
        else:
            prm, med = self.entropy_bottleneck.kernel_params()
            _lib.call("fvc_eb_forward", x.data_ptr(), prm.data_ptr(), med.data_ptr(), xhat.data_ptr(),
                      bits.data_ptr(), ws.data_ptr(), B, H, W, C, C, K.stream_handle())
        return xhat, bits, rpm_hidden, x  # prior_latent = round(x), rounded where RPM consumes it

    def compress(self, x):
        """x NHWC -> one string per batch item (compressai framing, C order (C, H, W))."""
        xn = K.nhwc_to_nchw(x, self.channels)
        if self.RPM_flag:
            sig = K.nhwc_to_nchw(self.sigma, self.channels)
            idx = self.gaussian_conditional.build_indexes(sig)
            return self.gaussian_conditional.compress(xn, idx, means=K.nhwc_to_nchw(self.mu, self.channels))
        return self.entropy_bottleneck.compress(xn)

    def decompress(self, strings, shape):
        """-> NHWC x_hat; RPM mode uses the sigma/mu of the last forward_latent (the decoder runs
        RPM on the same prior first)."""
        if self.RPM_flag:
            sig = K.nhwc_to_nchw(self.sigma, self.channels)
            idx = self.gaussian_conditional.build_indexes(sig)
            out = self.gaussian_conditional.decompress(strings, idx, means=K.nhwc_to_nchw(self.mu, self.channels))
        else:
            out = self.entropy_bottleneck.decompress(strings, shape)
        return K.nchw_to_nhwc(out.contiguous(), self.channels)

    @staticmethod
    def get_actual_bits(strings):
        return float(len(b"".join(strings)) * 8)

    def loss(self):
        """entropy_models.py:50-53: 0 in RPM mode, else the bottleneck's auxiliary loss."""
        if self.RPM_flag:
            return torch.zeros((), device=self.entropy_bottleneck.quantiles.device)
        return self.entropy_bottleneck.loss()


class Coder2D(nn.Module):
    """models.py:520-681 with keyword 'RLVC' (downsample, conv_type 'rec', entropy 'rpm')."""

    def __init__(self, keyword="RLVC", in_channels=2, channels=CHANNELS, kernel=3, padding=1):
        super().__init__()
        if keyword not in ("RLVC", "rpm"):
            raise ValueError(f"Coder2D keyword {keyword!r}: only the RLVC recurrent model is built")
        for i in range(1, 5):
            # enc_conv4 has no bias in the reference (models.py:528)
            setattr(self, f"enc_conv{i}", _ConvP(in_channels if i == 1 else channels, channels, kernel, 2,
                                                 bias=i != 4))
            setattr(self, f"dec_conv{i}", _ConvP(channels, in_channels if i == 4 else channels, kernel, 2,
                                                 transposed=True))
        for i in range(1, 4):
            setattr(self, f"gdn{i}", _GDNP(channels))
            setattr(self, f"igdn{i}", _GDNP(channels, inverse=True))
        self.entropy_bottleneck = RecProbModel(channels)
        self.enc_lstm = ConvLSTM(channels)
        self.dec_lstm = ConvLSTM(channels)  # present in the reference; its forward never calls it
        self.channels = channels
        self.in_channels = in_channels
        self.kernel, self.padding = kernel, padding

    def encode(self, x, state_enc):
        x = _gdn_cai(self.enc_conv1.packed()(x), self.gdn1)
        x = _gdn_cai(self.enc_conv2.packed()(x), self.gdn2)
        x, state_enc = self.enc_lstm.run(x, state_enc)
        x = _gdn_cai(self.enc_conv3.packed()(x), self.gdn3)
        return self.enc_conv4.packed()(x), state_enc

    def decode(self, latent_hat, state_dec, res=None):
        x = _gdn_cai(self.dec_conv1.packed()(latent_hat), self.igdn1)
        x = _gdn_cai(self.dec_conv2.packed()(x), self.igdn2)
        x, state_dec = self.enc_lstm.run(x, state_dec)  # models.py:661 uses enc_lstm here
        x = _gdn_cai(self.dec_conv3.packed()(x), self.igdn3)
        return self.dec_conv4.packed()(x, res=res), state_dec

    def run(self, x, rae_hidden, rpm_hidden, RPM_flag, prior_latent, res=None, real=True):
        """Coder2D.forward (eval): -> (hat [+ res], rae_hidden, rpm_hidden, bits_act, bits_est,
        prior_latent, strings)."""
        latent, enc = self.encode(x, rae_hidden["enc"])
        eb = self.entropy_bottleneck
        eb.set_RPM(RPM_flag)
        latent_hat, bits_est, rpm_hidden, prior_latent = eb.forward_latent(latent, rpm_hidden, prior_latent)
        strings = eb.compress(latent) if real else None
        bits_act = eb.get_actual_bits(strings) if real else float(bits_est.item())
        hat, dec = self.decode(latent_hat, rae_hidden["dec"], res=res)
        self.aux_loss = eb.loss()  # models.py:679
        return hat, {"enc": enc, "dec": dec}, rpm_hidden, bits_act, bits_est, prior_latent, strings


class RLVC(nn.Module):
    """IterPredVideoCodecs('RLVC') (models.py:954-1051), eval forward with real bitstreams."""

    def __init__(self, name="RLVC", channels=CHANNELS, compression_level=2):
        super().__init__()
        self.name = name
        self.opticFlow = ME_Spynet()
        self.warpnet = Warp_net()
        self.mv_codec = Coder2D(name, 2, channels, 3, 1)
        self.res_codec = Coder2D(name, 3, channels, 5, 2)
        self.channels = channels
        self.compression_level = compression_level
        self.r = {0: 256, 1: 512, 2: 1024, 3: 2048}.get(compression_level, 1024)
        self.eval()

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
            if isinstance(m, (_ConvP, _GDNP, ConvLSTM, RPM, LearnedEntropyBottleneck)):
                m.invalidate()

    def update(self, force=True):
        self.mv_codec.entropy_bottleneck.update(force=force)
        self.res_codec.entropy_bottleneck.update(force=force)

    def init_hidden(self, h, w, device, batch=1):
        """models.py:1042-1051 as NHWC state dicts (zeros)."""
        C = self.channels
        z = lambda s: torch.zeros((batch, h // s, w // s, C), device=device)
        rae = lambda: {"enc": {"c": z(4), "h": z(4)}, "dec": {"c": z(4), "h": z(4)}}
        return rae(), rae(), {"c": z(16), "h": z(16)}, {"c": z(16), "h": z(16)}

    # split-precision overflow: as VideoCompressor._run_checked -- every x3 conv ORs into the
    # stream's flag; a frame that set it is recomputed on the fp32 kernels (or rejected)
    on_overflow = "recompute"

    def forward(self, Y0_com, Y1_raw, hidden_states, RPM_flag, mv_prior_latent, res_prior_latent, real=True):
        """models.py:982-1040 (eval): -> (Y1_com, hidden_states, bpp_est, img_loss, aux_loss,
        bpp_act, psnr, mv_prior_latent, res_prior_latent); frames NCHW [B,3,H,W], H, W multiples of
        64. ``self.last_strings`` holds the frame's (mv, res) strings; ``self.last_precision`` the
        conv precision the frame was coded with ('x3', or 'f32' after an overflow recompute).
        ConvLSTM's cell state carries across frames unbounded, so the overflow check matters here."""
        if self.mv_codec.entropy_bottleneck.entropy_bottleneck._coder is None:
            self.update(force=True)
        B, _, H, W = Y1_raw.shape
        if H % 64 or W % 64:
            raise ValueError("H and W must be multiples of 64")
        args = (Y0_com, Y1_raw, hidden_states, RPM_flag, mv_prior_latent, res_prior_latent, real)
        if K.conv_precision() == "f32":
            self.last_precision = "f32"
            return self._forward_impl(*args)
        K.overflow_flag().zero_()
        out = self._forward_impl(*args)
        if not K.OverflowProbe().result():
            self.last_precision = "x3"
            return out
        self.overflow_events = getattr(self, "overflow_events", 0) + 1
        if self.on_overflow == "raise":
            raise FvcError("split-precision conv operand overflow (|activation| >= 65000) in RLVC")
        with K.precision("f32"):
            self.last_precision = "f32"
            return self._forward_impl(*args)

    def _forward_impl(self, Y0_com, Y1_raw, hidden_states, RPM_flag, mv_prior_latent, res_prior_latent, real):
        B, _, H, W = Y1_raw.shape
        rae_mv, rae_res, rpm_mv, rpm_res = hidden_states
        with torch.no_grad():
            cur4 = K.nchw_to_nhwc(Y1_raw.float().contiguous(), 4)
            ref4 = K.nchw_to_nhwc(Y0_com.float().contiguous(), 4)
            mv = self.opticFlow.run(cur4, ref4)  # models.py:991 opticFlow(Y1_raw, Y0_com)
            mv_hat, rae_mv, rpm_mv, mv_act, mv_est, mv_prior_latent, mv_str = self.mv_codec.run(
                mv, rae_mv, rpm_mv, RPM_flag, mv_prior_latent, real=real)
            warpframe, x8 = K.mc_assemble(ref4, mv_hat)
            Y1_MC = self.warpnet.run(x8, warpframe)
            res = K.sub(cur4, Y1_MC)
            recon, rae_res, rpm_res, res_act, res_est, res_prior_latent, res_str = self.res_codec.run(
                res, rae_res, rpm_res, RPM_flag, res_prior_latent, res=Y1_MC, real=real)
            clipped, sse = K.recon_finalize(recon, cur4, warpframe, Y1_MC)
        npx = B * H * W
        # img_loss / PSNR of the clipped Y1_com (models.py:1019,1033-1034): recon_finalize's 4th SSE
        img_loss = (sse[3] / (3 * npx)).float()
        psnr = 10.0 * torch.log10(1.0 / img_loss)
        bpp_est = ((mv_est + res_est) / npx).float()[0]
        bpp_act = torch.tensor((mv_act + res_act) / npx)
        self.last_strings = (mv_str, res_str)
        # models.py:1030-1031 at stage 'REC' (init_training_params, models.py:70): mv_aux + res_aux / 2
        aux_loss = self.mv_codec.aux_loss + self.res_codec.aux_loss / 2
        return (clipped, (rae_mv, rae_res, rpm_mv, rpm_res), bpp_est, img_loss, aux_loss, bpp_act, psnr,
                mv_prior_latent, res_prior_latent)


# ---------------------------------------------------------------- reference layout helpers
def hidden_to_reference(hidden):
    """NHWC state dicts -> the reference's (rae_mv, rae_res, rpm_mv, rpm_res) NCHW tensors
    (rae: cat(enc c, enc h, dec c, dec h); rpm: cat(c, h))."""
    def t(x):
        return x.permute(0, 3, 1, 2).contiguous()
    rae = lambda r: torch.cat([t(r["enc"]["c"]), t(r["enc"]["h"]), t(r["dec"]["c"]), t(r["dec"]["h"])], 1)
    rpm = lambda r: torch.cat([t(r["c"]), t(r["h"])], 1)
    return rae(hidden[0]), rae(hidden[1]), rpm(hidden[2]), rpm(hidden[3])


def hidden_from_reference(hidden, device):
    def t(x):
        return x.permute(0, 2, 3, 1).contiguous().float().to(device)
    def rae(r):
        c, h, dc, dh = torch.chunk(r, 4, 1)
        return {"enc": {"c": t(c), "h": t(h)}, "dec": {"c": t(dc), "h": t(dh)}}
    def rpm(r):
        c, h = torch.chunk(r, 2, 1)
        return {"c": t(c), "h": t(h)}
    return rae(hidden[0]), rae(hidden[1]), rpm(hidden[2]), rpm(hidden[3])


def seeded_state_dict(seed: int = 20261016, dvc_seed: int = 20261015):
    """Seeded RLVC weights with compressai/torch initialisation shapes: SpyNet / Warp_net from the
    DVC seeded state (weights.seeded_state_dict), Coder2D convs xavier-normal scaled for a stable
    forward, GDN at compressai's init (beta 1, gamma 0.1 I, reparametrised), ConvLSTM / RPM convs
    small, EntropyBottleneck at compressai's init plus small noise; quantiles [-10, 0, 10]."""
    from .weights import seeded_state_dict as dvc_sd, _gdn, _xavier_normal
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {k: v for k, v in dvc_sd(dvc_seed).items() if k.startswith(("opticFlow.", "warpnet."))}
    C = CHANNELS
    for name, cin, k in (("mv_codec", 2, 3), ("res_codec", 3, 5)):
        for i in range(1, 5):
            ci = cin if i == 1 else C
            # the last encoder conv is scaled so that latents span a few quantisation steps
            sd[f"{name}.enc_conv{i}.weight"] = _xavier_normal(rng, (C, ci, k, k), math.sqrt(2.0) * (12.0 if i == 4 else 1.0))
            if i != 4:  # enc_conv4 is bias-free (models.py:528)
                sd[f"{name}.enc_conv{i}.bias"] = rng.uniform(-0.05, 0.05, C).astype(np.float32)
            co = cin if i == 4 else C
            sd[f"{name}.dec_conv{i}.weight"] = _xavier_normal(rng, (C, co, k, k), 1.0)
            sd[f"{name}.dec_conv{i}.bias"] = rng.uniform(-0.05, 0.05, co).astype(np.float32)
        for g in ("gdn", "igdn"):
            for i in range(1, 4):
                b, gm = _gdn(C)
                sd[f"{name}.{g}{i}.beta"] = b
                sd[f"{name}.{g}{i}.gamma"] = gm
        for lstm in ("enc_lstm", "dec_lstm", "entropy_bottleneck.RPM.lstm"):
            sd[f"{name}.{lstm}.conv.weight"] = _xavier_normal(rng, (4 * C, 2 * C, 3, 3), 0.5)
            sd[f"{name}.{lstm}.conv.bias"] = rng.uniform(-0.05, 0.05, 4 * C).astype(np.float32)
        for i in range(1, 9):
            co = 2 * C if i == 8 else C
            sd[f"{name}.entropy_bottleneck.RPM.conv{i}.weight"] = _xavier_normal(rng, (co, C, 3, 3), 0.7)
            sd[f"{name}.entropy_bottleneck.RPM.conv{i}.bias"] = rng.uniform(-0.05, 0.05, co).astype(np.float32)
        filters = (1,) + FILTERS + (1,)
        scale = 10.0 ** (1 / (len(FILTERS) + 1))
        for i in range(len(FILTERS) + 1):
            init = np.log(np.expm1(1 / scale / filters[i + 1]))
            sd[f"{name}.entropy_bottleneck.entropy_bottleneck._matrix{i}"] = (
                init + 0.1 * rng.standard_normal((C, filters[i + 1], filters[i]))).astype(np.float32)
            sd[f"{name}.entropy_bottleneck.entropy_bottleneck._bias{i}"] = rng.uniform(
                -0.5, 0.5, (C, filters[i + 1], 1)).astype(np.float32)
            if i < len(FILTERS):
                sd[f"{name}.entropy_bottleneck.entropy_bottleneck._factor{i}"] = (
                    0.1 * rng.standard_normal((C, filters[i + 1], 1))).astype(np.float32)
        q = np.tile(np.array([[-10.0, 0.0, 10.0]], np.float32), (C, 1, 1))
        q[:, 0, 1] += rng.uniform(-0.3, 0.3, C).astype(np.float32)
        sd[f"{name}.entropy_bottleneck.entropy_bottleneck.quantiles"] = q
    return sd


# Entries of a reference RLVC state_dict that load_state_dict_all itself skips (models.py:446-448):
# the coder tables, rebuilt by update().
_SKIPPED_SUFFIXES = ("._offset", "._quantized_cdf", "._cdf_length", ".scale_table")


def _derived_buffers():
    """compressai 1.2.x constant buffers a reference RLVC state_dict carries and this build derives
    from the same constructor constants instead of storing (restated from compressai's published
    source, which is not importable here -- SURVEY §8(c)): GDN's NonNegativeParametrizer
    (pedestal 2^-36, LowerBound sqrt(minimum + pedestal), beta_min 1e-6), EntropyBottleneck.target
    (tail_mass 1e-9), EntropyModel's likelihood LowerBound (1e-9), GaussianConditional's scale
    bound (0.11). Suffix -> expected value."""
    ped = 2.0 ** -36
    t = float(np.log(2 / 1e-9 - 1))
    return {
        "beta_reparam.pedestal": [ped], "beta_reparam.lower_bound.bound": [(1e-6 + ped) ** 0.5],
        "gamma_reparam.pedestal": [ped], "gamma_reparam.lower_bound.bound": [ped ** 0.5],
        "entropy_bottleneck.entropy_bottleneck.target": [-t, 0.0, t],
        "likelihood_lower_bound.bound": [1e-9],
        "gaussian_conditional.scale_bound": [0.11], "gaussian_conditional.lower_bound_scale.bound": [0.11],
    }


def load_state_dict_all(model, state_dict):
    """models.py:444-449: copy every entry of a reference state_dict into the model, skipping the
    coder tables. Like the reference, an entry the model does not have raises KeyError and a
    shape mismatch raises; compressai's derived constant buffers (``_derived_buffers``) are
    checked against their constants instead of stored. Returns the model's keys that the
    state_dict did not set."""
    own = model.state_dict()
    derived = _derived_buffers()
    seen = set()
    for name, param in state_dict.items():
        if name.endswith(_SKIPPED_SUFFIXES):
            continue
        param = torch.as_tensor(param)
        if name in own:
            if tuple(own[name].shape) != tuple(param.shape):
                raise ValueError(f"{name}: shape {tuple(param.shape)} != {tuple(own[name].shape)}")
            with torch.no_grad():
                own[name].copy_(param)
            seen.add(name)
            continue
        suffix = next((k for k in derived if name.endswith("." + k)), None)
        if suffix is None:
            raise KeyError(name)
        want = torch.tensor(derived[suffix], dtype=torch.float64)
        got = param.detach().double().reshape(-1).cpu()
        if got.shape != want.shape or not torch.allclose(got, want, rtol=1e-5, atol=0.0):
            raise ValueError(f"{name}: {got.tolist()} differs from compressai's constant {want.tolist()}")
    model.invalidate()
    return sorted(set(own) - seen)


def get_rlvc_model(seed: int = 20261016, device="cuda", checkpoint=None):
    """RLVC with seeded weights, or a reference checkpoint: a path (``torch.load`` with
    ``weights_only=True``), a state_dict, or a dict holding one under 'state_dict' -- loaded with
    the reference's ``load_state_dict_all`` semantics (models.py:444-449)."""
    m = RLVC()
    if checkpoint is not None:
        ck = checkpoint
        if isinstance(ck, (str, bytes, os.PathLike)):
            ck = torch.load(ck, map_location="cpu", weights_only=True)
        if isinstance(ck, dict) and "state_dict" in ck and isinstance(ck["state_dict"], dict):
            ck = ck["state_dict"]
        m.missing_checkpoint_keys = load_state_dict_all(m, ck)
        m.weights_source = "checkpoint"
        return m.to(device).eval()
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in seeded_state_dict(seed).items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    if unexpected:
        raise KeyError(f"unexpected keys {unexpected[:5]}")
    bad = [k for k in missing if not k.endswith(("weight", "bias")) or "dec_lstm" not in k]
    if bad:
        raise KeyError(f"missing keys {bad[:5]}")
    m.weights_source = "seeded"
    return m.to(device).eval()
