"""ORACLE — test infrastructure only. CPU restatement of the reference DVC P-frame forward.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the reported CPU baseline. The product path
(``fastvideocodec_amd``) never calls it.

It restates ``DVC/net.py:VideoCompressor.forward`` (net.py:70-220) in plain PyTorch CPU
fp32 ops, functionally (a state_dict in, tensors out), one function per reference module.
Every function cites the reference lines it follows. Exact resampling semantics follow
SURVEY.md Appendix B; ``warp`` is the closed form of ``torch_warp`` (endecoder.py:52-67)
without its ``.cuda()``/device-indexed grid cache.

Parity pin: ``tests/golden/*.npz`` were produced by running the reference itself
(imported from /root/reference in the build container, see tests/golden/gen_golden.py);
``tests/test_oracle_golden.py`` checks this restatement against them.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _p(sd, name):
    return sd[name]


# ---------------------------------------------------------------- resampling (Appendix B)
def warp(im: torch.Tensor, flow: torch.Tensor) -> torch.Tensor:
    """torch_warp / flow_warp (endecoder.py:52-67, 116-119): an align_corners=True grid
    (linspace(-1,1)) plus flow/((n-1)/2), sampled by grid_sample(bilinear, border,
    align_corners=False)."""
    B, _, H, W = flow.shape
    gx = torch.linspace(-1.0, 1.0, W).view(1, 1, 1, W).expand(B, -1, H, -1)
    gy = torch.linspace(-1.0, 1.0, H).view(1, 1, H, 1).expand(B, -1, -1, W)
    grid = torch.cat([gx, gy], 1)
    f = torch.cat([flow[:, 0:1] / ((im.size(3) - 1.0) / 2.0),
                   flow[:, 1:2] / ((im.size(2) - 1.0) / 2.0)], 1)
    return F.grid_sample(im, (grid + f).permute(0, 2, 3, 1), mode="bilinear",
                         padding_mode="border", align_corners=False)


def up2(x: torch.Tensor, align_corners: bool) -> torch.Tensor:
    """bilinearupsacling (ac=False, endecoder.py:173-179) / bilinearupsacling2 (ac=True, :180-184)."""
    H, W = x.shape[-2:]
    return F.interpolate(x, (H * 2, W * 2), mode="bilinear", align_corners=align_corners)


# ---------------------------------------------------------------- SpyNet (endecoder.py)
def me_basic(sd, prefix, x):
    """MEBasic.forward (endecoder.py:162-168): 5x conv7x7 p3, ReLU between."""
    for i in range(1, 6):
        x = F.conv2d(x, _p(sd, f"{prefix}.conv{i}.weight"), _p(sd, f"{prefix}.conv{i}.bias"), 1, 3)
        if i < 5:
            x = F.relu(x)
    return x


def me_spynet(sd, im1, im2):
    """ME_Spynet.forward (endecoder.py:337-356)."""
    L = 4
    im1l, im2l = [im1], [im2]
    for lvl in range(L - 1):
        im1l.append(F.avg_pool2d(im1l[lvl], kernel_size=2, stride=2))
        im2l.append(F.avg_pool2d(im2l[lvl], kernel_size=2, stride=2))
    sh = im2l[L - 1].shape
    flow = torch.zeros(sh[0], 2, sh[2] // 2, sh[3] // 2)
    for lvl in range(L):
        fup = up2(flow, False) * 2.0
        x = torch.cat([im1l[L - 1 - lvl], warp(im2l[L - 1 - lvl], fup), fup], 1)
        flow = fup + me_basic(sd, f"opticFlow.moduleBasic.{lvl}", x)
    return flow


# ---------------------------------------------------------------- MV codec
def mv_encoder(sd, x):
    """Analysis_mv_net.forward (analysis_mv.py:58-66): conv3x3 s(2,1)x4, LeakyReLU(0.1)."""
    for i in range(1, 9):
        s = 2 if i % 2 == 1 else 1
        x = F.conv2d(x, _p(sd, f"mvEncoder.conv{i}.weight"), _p(sd, f"mvEncoder.conv{i}.bias"), s, 1)
        if i < 8:
            x = F.leaky_relu(x, 0.1)
    return x


def mv_decoder(sd, x):
    """Synthesis_mv_net.forward (synthesis_mv.py:59-79): deconv3x3 s2 p1 op1 / conv3x3."""
    for i in range(1, 9):
        w, b = _p(sd, f"mvDecoder.deconv{i}.weight"), _p(sd, f"mvDecoder.deconv{i}.bias")
        if i % 2 == 1:
            x = F.conv_transpose2d(x, w, b, 2, 1, 1)
        else:
            x = F.conv2d(x, w, b, 1, 1)
        if i < 8:
            x = F.leaky_relu(x, 0.1)
    return x


# ---------------------------------------------------------------- motion compensation
def res_block(sd, prefix, x):
    """ResBlock.forward (endecoder.py:252-260), pre-activation, identity skip."""
    y = F.conv2d(F.relu(x), _p(sd, f"{prefix}.conv1.weight"), _p(sd, f"{prefix}.conv1.bias"), 1, 1)
    y = F.conv2d(F.relu(y), _p(sd, f"{prefix}.conv2.weight"), _p(sd, f"{prefix}.conv2.bias"), 1, 1)
    return x + y


def warp_net(sd, x):
    """Warp_net.forward (endecoder.py:281-296)."""
    fe = F.relu(F.conv2d(x, _p(sd, "warpnet.feature_ext.weight"), _p(sd, "warpnet.feature_ext.bias"), 1, 1))
    c0 = res_block(sd, "warpnet.conv0", fe)
    c1 = res_block(sd, "warpnet.conv1", F.avg_pool2d(c0, 2, 2))
    c2 = res_block(sd, "warpnet.conv2", F.avg_pool2d(c1, 2, 2))
    c3 = res_block(sd, "warpnet.conv3", c2)
    c3u = c1 + up2(c3, True)
    c4 = res_block(sd, "warpnet.conv4", c3u)
    c4u = c0 + up2(c4, True)
    c5 = res_block(sd, "warpnet.conv5", c4u)
    return F.conv2d(c5, _p(sd, "warpnet.conv6.weight"), _p(sd, "warpnet.conv6.bias"), 1, 1)


def motion_compensation(sd, ref, mv):
    """VideoCompressor.motioncompensation (net.py:64-68)."""
    warpframe = warp(ref, mv)
    prediction = warp_net(sd, torch.cat((warpframe, ref), 1)) + warpframe
    return prediction, warpframe


# ---------------------------------------------------------------- GDN + residual codec
def gdn(sd, prefix, x, inverse):
    """GDN.forward (GDN.py:63-93): beta/gamma reparametrised with LowerBound, 1x1 conv on x^2."""
    pedestal = (2.0 ** -18) ** 2
    beta_bound = (1e-6 + pedestal) ** 0.5
    gamma_bound = 2.0 ** -18
    C = x.shape[1]
    beta = torch.clamp_min(_p(sd, f"{prefix}.beta"), beta_bound) ** 2 - pedestal
    gamma = (torch.clamp_min(_p(sd, f"{prefix}.gamma"), gamma_bound) ** 2 - pedestal).view(C, C, 1, 1)
    norm = torch.sqrt(F.conv2d(x ** 2, gamma, beta))
    return x * norm if inverse else x / norm


def res_encoder(sd, x):
    """Analysis_net.forward (analysis.py:44-48)."""
    for i in range(1, 5):
        x = F.conv2d(x, _p(sd, f"resEncoder.conv{i}.weight"), _p(sd, f"resEncoder.conv{i}.bias"), 2, 2)
        if i < 4:
            x = gdn(sd, f"resEncoder.gdn{i}", x, False)
    return x


def res_decoder(sd, x):
    """Synthesis_net.forward (synthesis.py:42-58)."""
    for i in range(1, 5):
        x = F.conv_transpose2d(x, _p(sd, f"resDecoder.deconv{i}.weight"), _p(sd, f"resDecoder.deconv{i}.bias"), 2, 2, 1)
        if i < 4:
            x = gdn(sd, f"resDecoder.igdn{i}", x, True)
    return x


def prior_encoder(sd, x):
    """Analysis_prior_net.forward (analysis_prior.py:40-56)."""
    x = torch.abs(x)
    x = F.relu(F.conv2d(x, _p(sd, "respriorEncoder.conv1.weight"), _p(sd, "respriorEncoder.conv1.bias"), 1, 1))
    x = F.relu(F.conv2d(x, _p(sd, "respriorEncoder.conv2.weight"), _p(sd, "respriorEncoder.conv2.bias"), 2, 2))
    return F.conv2d(x, _p(sd, "respriorEncoder.conv3.weight"), _p(sd, "respriorEncoder.conv3.bias"), 2, 2)


def prior_decoder(sd, x):
    """Synthesis_prior_net.forward (synthesis_prior.py:42-58)."""
    x = F.relu(F.conv_transpose2d(x, _p(sd, "respriorDecoder.deconv1.weight"), _p(sd, "respriorDecoder.deconv1.bias"), 2, 2, 1))
    x = F.relu(F.conv_transpose2d(x, _p(sd, "respriorDecoder.deconv2.weight"), _p(sd, "respriorDecoder.deconv2.bias"), 2, 2, 1))
    x = F.conv_transpose2d(x, _p(sd, "respriorDecoder.deconv3.weight"), _p(sd, "respriorDecoder.deconv3.bias"), 1, 1)
    return torch.exp(x)


# ---------------------------------------------------------------- bit estimates
def bit_estimator(sd, prefix, x):
    """BitEstimator.forward (bitEstimator.py:36-42) with Bitparm (:6-25)."""
    for f in range(1, 4):
        h, b, a = (_p(sd, f"{prefix}.f{f}.{n}") for n in "hba")
        x = x * F.softplus(h) + b
        x = x + torch.tanh(x) * torch.tanh(a)
    h, b = _p(sd, f"{prefix}.f4.h"), _p(sd, f"{prefix}.f4.b")
    return torch.sigmoid(x * F.softplus(h) + b)


def bits_laplace(feature, sigma):
    """feature_probs_based_sigma (net.py:121-151), estimate branch."""
    mu = torch.zeros_like(sigma)
    sigma = sigma.clamp(1e-5, 1e10)
    lap = torch.distributions.laplace.Laplace(mu, sigma)
    probs = lap.cdf(feature + 0.5) - lap.cdf(feature - 0.5)
    return torch.sum(torch.clamp(-1.0 * torch.log(probs + 1e-5) / math.log(2.0), 0, 50))


def bits_factorized(sd, prefix, v):
    """iclr18_estrate_bits_z / _mv (net.py:153-205), estimate branch."""
    prob = bit_estimator(sd, prefix, v + 0.5) - bit_estimator(sd, prefix, v - 0.5)
    return torch.sum(torch.clamp(-1.0 * torch.log(prob + 1e-5) / math.log(2.0), 0, 50))


# ---------------------------------------------------------------- the forward
def forward(sd, input_image, referframe, return_intermediates=False):
    """VideoCompressor.forward (net.py:70-220), eval mode (torch.round quantisation)."""
    with torch.no_grad():
        estmv = me_spynet(sd, input_image, referframe)
        mvfeature = mv_encoder(sd, estmv)
        quant_mv = torch.round(mvfeature)
        quant_mv_upsample = mv_decoder(sd, quant_mv)
        prediction, warpframe = motion_compensation(sd, referframe, quant_mv_upsample)
        input_residual = input_image - prediction
        feature = res_encoder(sd, input_residual)
        z = prior_encoder(sd, feature)
        compressed_z = torch.round(z)
        recon_sigma = prior_decoder(sd, compressed_z)
        compressed_feature = torch.round(feature)
        recon_res = res_decoder(sd, compressed_feature)
        recon_image = prediction + recon_res
        clipped = recon_image.clamp(0.0, 1.0)
        mse_loss = torch.mean((recon_image - input_image).pow(2))
        warploss = torch.mean((warpframe - input_image).pow(2))
        interloss = torch.mean((prediction - input_image).pow(2))
        bits_feature = bits_laplace(compressed_feature, recon_sigma)
        bits_z = bits_factorized(sd, "bitEstimator_z", compressed_z)
        bits_mv = bits_factorized(sd, "bitEstimator_mv", quant_mv)
        B, _, H, W = input_image.shape
        bpp_feature = bits_feature / (B * H * W)
        bpp_z = bits_z / (B * H * W)
        bpp_mv = bits_mv / (B * H * W)
        bpp = bpp_feature + bpp_z + bpp_mv
    out = (clipped, mse_loss, warploss, interloss, bpp_feature, bpp_z, bpp_mv, bpp)
    if not return_intermediates:
        return out
    inter = dict(estmv=estmv, mvfeature=mvfeature, quant_mv=quant_mv,
                 quant_mv_upsample=quant_mv_upsample, warpframe=warpframe,
                 prediction=prediction, feature=feature, z=z, compressed_z=compressed_z,
                 recon_sigma=recon_sigma, compressed_feature=compressed_feature,
                 recon_res=recon_res)
    return out, inter


def decode(sd, referframe, quant_mv, compressed_z, compressed_feature):
    """Decoder-side reconstruction from the three quantised latents (net.py:77-105 restricted
    to what a decoder can compute): mv -> MC prediction; z -> sigma; feature -> residual."""
    with torch.no_grad():
        mv = mv_decoder(sd, quant_mv)
        prediction, _ = motion_compensation(sd, referframe, mv)
        sigma = prior_decoder(sd, compressed_z)
        recon = prediction + res_decoder(sd, compressed_feature)
        return recon.clamp(0.0, 1.0), sigma


def psnr(a, b):
    """PSNR (models.py:460-473): 10*ln(1/mse)/ln(10) over the whole tensor."""
    mse = torch.mean(torch.pow(a - b, 2))
    return 10.0 * torch.log(1 / mse) / math.log(10.0)
