"""ORACLE — test infrastructure only (tests/). CPU restatement of the reference's RLVC path
 in plain PyTorch fp32, functionally (state_dict in, tensors out):
``IterPredVideoCodecs.forward`` (models.py:982-1040, eval), ``Coder2D.forward`` (models.py:565-681,
keyword 'RLVC'), ``RecProbModel.forward`` (entropy_models.py:55-68), ``RPM`` (:328-357) and
``ConvLSTM`` (:359-378); SpyNet / Warp_net / warp come from oracle/dvc_ref.py (same modules).

compressai (absent) parts restated from its 1.2.x semantics: ``layers.GDN`` (x * rsqrt(beta +
gamma . x^2); inverse x * sqrt), ``EntropyBottleneck`` (filters (3,3,3,3): _logits_cumulative,
_likelihood with the sign trick, quantize 'dequantize' around the medians) and
``GaussianConditional`` with means (likelihood from 0.5 erfc, scale bound 0.11), each with the
1e-9 likelihood lower bound; ``get_estimate_bits`` = sum clamp(-log2(l + 1e-5), 0, 50).
Parity pin: ConvLSTM and RPM are checked against the reference itself
(tests/golden/rlvc_rpm.npz, tests/golden/gen_rlvc_golden.py); the compressai parts are
unpinned (no compressai here), as SURVEY §8(c) records for the coder.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

import dvc_ref as D

FILTERS = (3, 3, 3, 3)


def gdn_cai(sd, prefix, x, inverse):
    pedestal = (2.0 ** -18) ** 2
    beta = torch.clamp_min(sd[f"{prefix}.beta"], (1e-6 + pedestal) ** 0.5) ** 2 - pedestal
    C = x.shape[1]
    gamma = (torch.clamp_min(sd[f"{prefix}.gamma"], pedestal ** 0.5) ** 2 - pedestal).view(C, C, 1, 1)
    norm = F.conv2d(x ** 2, gamma, beta)
    return x * torch.sqrt(norm) if inverse else x * torch.rsqrt(norm)


def conv_lstm(sd, prefix, x, state, forget_bias=1.0):
    C = x.shape[1]
    c, h = torch.split(state, C, dim=1)
    y = F.conv2d(torch.cat((x, h), 1), sd[f"{prefix}.conv.weight"], sd[f"{prefix}.conv.bias"], 1, 1)
    j, i, f, o = torch.split(y, C, dim=1)
    f = torch.sigmoid(f + forget_bias)
    i = torch.sigmoid(i)
    c = c * f + i * F.relu(j)
    o = torch.sigmoid(o)
    h = o * F.relu(c)
    return h, torch.cat((c, h), 1)


def rpm(sd, prefix, x, hidden):
    conv = lambda i, v: F.conv2d(v, sd[f"{prefix}.conv{i}.weight"], sd[f"{prefix}.conv{i}.bias"], 1, 1)
    for i in range(1, 5):
        x = F.relu(conv(i, x))
    x, hidden = conv_lstm(sd, f"{prefix}.lstm", x, hidden)
    for i in range(5, 8):
        x = F.relu(conv(i, x))
    sm = F.relu(conv(8, x))
    C = x.shape[1]
    sigma, mu = torch.split(sm, C, dim=1)
    return sigma, mu, hidden


def eb_logits(sd, prefix, inputs):
    logits = inputs
    for i in range(len(FILTERS) + 1):
        logits = torch.matmul(F.softplus(sd[f"{prefix}._matrix{i}"]), logits)
        logits = logits + sd[f"{prefix}._bias{i}"]
        if i < len(FILTERS):
            logits = logits + torch.tanh(sd[f"{prefix}._factor{i}"]) * torch.tanh(logits)
    return logits


def eb_forward(sd, prefix, x):
    """EntropyBottleneck.forward(x, training=False): (outputs, likelihood) in NCHW."""
    C = x.shape[1]
    v = x.permute(1, 0, 2, 3).contiguous()
    shape = v.shape
    values = v.reshape(C, 1, -1)
    med = sd[f"{prefix}.quantiles"][:, :, 1:2]
    outputs = torch.round(values - med) + med
    lower = eb_logits(sd, prefix, outputs - 0.5)
    upper = eb_logits(sd, prefix, outputs + 0.5)
    sign = -torch.sign(lower + upper)
    lik = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))
    lik = torch.clamp_min(lik, 1e-9)
    back = lambda t: t.reshape(shape).permute(1, 0, 2, 3).contiguous()
    return back(outputs), back(lik)


def eb_aux_loss(sd, prefix, tail_mass=1e-9):
    """compressai EntropyBottleneck.loss(): sum |logits_cumulative(quantiles) - (-t, 0, t)|,
    t = log(2 / tail_mass - 1) (called by RecProbModel.loss, entropy_models.py:50-53)."""
    t = math.log(2 / tail_mass - 1)
    logits = eb_logits(sd, prefix, sd[f"{prefix}.quantiles"])
    return torch.abs(logits - torch.tensor([-t, 0.0, t])).sum()


def gc_forward(x, scales, means):
    outputs = torch.round(x - means) + means
    values = torch.abs(outputs - means)
    s = torch.clamp_min(scales, 0.11)
    cum = lambda t: 0.5 * torch.erfc(-(2 ** -0.5) * t)
    lik = cum((0.5 - values) / s) - cum((-0.5 - values) / s)
    return outputs, torch.clamp_min(lik, 1e-9)


def estimate_bits(lik):
    return torch.sum(torch.clamp(-1.0 * torch.log(lik + 1e-5) / math.log(2.0), 0, 50))


def rec_prob_model(sd, prefix, x, rpm_hidden, RPM_flag, prior_latent):
    """RecProbModel.forward (eval) -> (x_hat, likelihood, rpm_hidden, prior_latent, sigma, mu)."""
    sigma = mu = None
    if RPM_flag:
        sigma, mu, rpm_hidden = rpm(sd, f"{prefix}.RPM", prior_latent, rpm_hidden)
        sigma = torch.exp(torch.maximum(sigma, torch.tensor(-7.0))) / 10
        x_hat, lik = gc_forward(x, sigma, mu)
    else:
        x_hat, lik = eb_forward(sd, f"{prefix}.entropy_bottleneck", x)
    return x_hat, lik, rpm_hidden, torch.round(x), sigma, mu


def coder2d_decode(sd, prefix, latent_hat, state_dec, padding):
    """Coder2D's synthesis half (models.py:655-664): deconv + IGDN x3 with the recurrent cell
    (enc_lstm, models.py:661) after the second, then deconv4 -> (hat, new decoder state)."""
    deconv = lambda i, v: F.conv_transpose2d(v, sd[f"{prefix}.dec_conv{i}.weight"], sd[f"{prefix}.dec_conv{i}.bias"],
                                             2, padding, 1)
    x = gdn_cai(sd, f"{prefix}.igdn1", deconv(1, latent_hat), True)
    x = gdn_cai(sd, f"{prefix}.igdn2", deconv(2, x), True)
    x, state_dec = conv_lstm(sd, f"{prefix}.enc_lstm", x, state_dec)  # models.py:661: enc_lstm
    x = gdn_cai(sd, f"{prefix}.igdn3", deconv(3, x), True)
    return deconv(4, x), state_dec


def coder2d(sd, prefix, x, rae_hidden, rpm_hidden, RPM_flag, prior_latent, padding):
    """Coder2D.forward (eval, 'RLVC'); returns a dict of outputs and intermediates."""
    C = rae_hidden.shape[1] // 4
    state_enc, state_dec = torch.split(rae_hidden, 2 * C, dim=1)
    conv = lambda i, v: F.conv2d(v, sd[f"{prefix}.enc_conv{i}.weight"], sd.get(f"{prefix}.enc_conv{i}.bias"), 2,
                                 padding)
    x = gdn_cai(sd, f"{prefix}.gdn1", conv(1, x), False)
    x = gdn_cai(sd, f"{prefix}.gdn2", conv(2, x), False)
    x, state_enc = conv_lstm(sd, f"{prefix}.enc_lstm", x, state_enc)
    x = gdn_cai(sd, f"{prefix}.gdn3", conv(3, x), False)
    latent = conv(4, x)
    latent_hat, lik, rpm_hidden, prior_latent, sigma, mu = rec_prob_model(
        sd, f"{prefix}.entropy_bottleneck", latent, rpm_hidden, RPM_flag, prior_latent)
    bits_est = estimate_bits(lik)
    hat, state_dec = coder2d_decode(sd, prefix, latent_hat, state_dec, padding)
    aux = torch.zeros(()) if RPM_flag else eb_aux_loss(sd, f"{prefix}.entropy_bottleneck.entropy_bottleneck")
    return dict(hat=hat, rae_hidden=torch.cat((state_enc, state_dec), 1), rpm_hidden=rpm_hidden,
                bits_est=bits_est, prior_latent=prior_latent, latent=latent, latent_hat=latent_hat,
                sigma=sigma, mu=mu, aux=aux)


def init_hidden(h, w, C=128, batch=1):
    return (torch.zeros(batch, 4 * C, h // 4, w // 4), torch.zeros(batch, 4 * C, h // 4, w // 4),
            torch.zeros(batch, 2 * C, h // 16, w // 16), torch.zeros(batch, 2 * C, h // 16, w // 16))


def forward(sd, Y0_com, Y1_raw, hidden, RPM_flag, mv_prior_latent, res_prior_latent):
    """IterPredVideoCodecs.forward (eval, models.py:982-1040) without real-bit strings;
    returns a dict (Y1_com, hidden, bpp_est, img_loss, psnr, priors, intermediates)."""
    rae_mv, rae_res, rpm_mv, rpm_res = hidden
    B, _, H, W = Y1_raw.shape
    mv = D.me_spynet(sd, Y1_raw, Y0_com)
    m = coder2d(sd, "mv_codec", mv, rae_mv, rpm_mv, RPM_flag, mv_prior_latent, 1)
    Y1_MC, Y1_warp = D.motion_compensation(sd, Y0_com, m["hat"])
    res = Y1_raw - Y1_MC
    r = coder2d(sd, "res_codec", res, rae_res, rpm_res, RPM_flag, res_prior_latent, 2)
    Y1_com = torch.clip(r["hat"] + Y1_MC, min=0, max=1)
    bpp_est = (m["bits_est"] + r["bits_est"]) / (H * W * B)
    img_loss = torch.mean((Y1_raw - Y1_com) ** 2)
    psnr = 10.0 * torch.log(1 / img_loss) / math.log(10.0)
    aux_loss = m["aux"] + r["aux"] / 2  # models.py:1030-1031, stage 'REC'
    return dict(Y1_com=Y1_com, hidden=(m["rae_hidden"], r["rae_hidden"], m["rpm_hidden"], r["rpm_hidden"]),
                bpp_est=bpp_est, img_loss=img_loss, psnr=psnr, aux_loss=aux_loss, mv_prior_latent=m["prior_latent"],
                res_prior_latent=r["prior_latent"], mv=mv, mv_hat=m["hat"], Y1_MC=Y1_MC, mv_codec=m, res_codec=r)
