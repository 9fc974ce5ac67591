"""ORACLE — test infrastructure only (tests/). numpy restatement of the I-frame transform the
build uses in place of BPG (the reference codes I-frames with `bpgenc`/`bpgdec` through
os.system, models.py:412-429; those binaries are absent):

* 8-bit samples q = clamp(round(x * 255), 0, 255) (frames in the reference are PIL images
  through ToTensor, i.e. exactly k/255: dataset.py:58-86);
* JPEG 2000 reversible colour transform (RCT): Y = floor((R + 2G + B) / 4), U = B - G, V = R - G;
* L levels of the JPEG 2000 reversible LeGall 5/3 lifting wavelet, rows then columns, symmetric
  extension, Mallat layout (LL top-left);
* optional dead-zone quantisation of the high-pass subbands with step Q (lossy mode): c -> sign(c)
  floor(|c| / Q), reconstructed as sign(c) (|c| * Q + Q // 2) (c != 0); Q = 1 is lossless.
The device implementation (fastvideocodec_amd/iframe.py, csrc/fvc_iframe.hip) must match these
integers exactly (tests/test_gpu_iframe.py).
"""
from __future__ import annotations

import numpy as np


def to_u8(x):
    return np.clip(np.rint(np.asarray(x, np.float32) * np.float32(255.0)), 0, 255).astype(np.int32)


def rct_forward(q):
    r, g, b = q[0], q[1], q[2]
    return np.stack([(r + 2 * g + b) >> 2, b - g, r - g])


def rct_inverse(c):
    y, u, v = c[0], c[1], c[2]
    g = y - ((u + v) >> 2)
    return np.stack([v + g, g, u + g])


def lift53_1d(x, axis):
    """One 5/3 analysis step along axis (even length): returns [low | high] along that axis."""
    x = np.moveaxis(x, axis, -1)
    e, o = x[..., 0::2], x[..., 1::2]
    e_next = np.concatenate([e[..., 1:], e[..., -1:]], -1)  # x[2n+2], symmetric at the end
    d = o - ((e + e_next) >> 1)
    d_prev = np.concatenate([d[..., :1], d[..., :-1]], -1)   # d[n-1], symmetric at the start
    s = e + ((d_prev + d + 2) >> 2)
    return np.moveaxis(np.concatenate([s, d], -1), -1, axis)


def unlift53_1d(y, axis):
    y = np.moveaxis(y, axis, -1)
    n = y.shape[-1] // 2
    s, d = y[..., :n], y[..., n:]
    d_prev = np.concatenate([d[..., :1], d[..., :-1]], -1)
    e = s - ((d_prev + d + 2) >> 2)
    e_next = np.concatenate([e[..., 1:], e[..., -1:]], -1)
    o = d + ((e + e_next) >> 1)
    x = np.empty(y.shape, y.dtype)
    x[..., 0::2] = e
    x[..., 1::2] = o
    return np.moveaxis(x, -1, axis)


def dwt_forward(c, levels):
    c = c.copy()
    h, w = c.shape[-2:]
    for _ in range(levels):
        sub = c[..., :h, :w]
        sub = lift53_1d(sub, -1)
        sub = lift53_1d(sub, -2)
        c[..., :h, :w] = sub
        h, w = h // 2, w // 2
    return c


def dwt_inverse(c, levels):
    c = c.copy()
    H, W = c.shape[-2:]
    for lv in reversed(range(levels)):
        h, w = H >> lv, W >> lv
        sub = c[..., :h, :w]
        sub = unlift53_1d(sub, -2)
        sub = unlift53_1d(sub, -1)
        c[..., :h, :w] = sub
    return c


def highpass_mask(H, W, levels):
    m = np.ones((H, W), bool)
    m[: H >> levels, : W >> levels] = False
    return m


def quantize(c, q, levels):
    if q <= 1:
        return c.copy()
    m = highpass_mask(*c.shape[-2:], levels)
    out = c.copy()
    a = np.abs(c[..., m]) // q
    out[..., m] = np.sign(c[..., m]) * a
    return out


def dequantize(c, q, levels):
    if q <= 1:
        return c.copy()
    m = highpass_mask(*c.shape[-2:], levels)
    out = c.copy()
    v = c[..., m]
    out[..., m] = np.where(v == 0, 0, np.sign(v) * (np.abs(v) * q + q // 2))
    return out


def encode_coeffs(x, levels, q=1):
    """frame [3,H,W] in [0,1] -> quantised wavelet coefficients [3,H,W] int32."""
    return quantize(dwt_forward(rct_forward(to_u8(x)), levels), q, levels)


def decode_coeffs(c, levels, q=1):
    """quantised coefficients -> frame [3,H,W] float32 (k/255)."""
    rgb = rct_inverse(dwt_inverse(dequantize(c, q, levels), levels))
    return (np.clip(rgb, 0, 255).astype(np.float32) / np.float32(255.0))


def block_index(c, scale_table, bs=32):
    """Per (plane, bs x bs block) Laplace table index of the block's mean |coefficient| (the
    scale compressai's build_indexes maps it to, lower bound 0.11)."""
    P, H, W = c.shape
    a = np.abs(c.astype(np.int64)).reshape(P, H // bs, bs, W // bs, bs).sum(axis=(2, 4))
    m = np.maximum((a / float(bs * bs)).astype(np.float32), np.float32(0.11))
    st = np.asarray(scale_table, np.float32)
    idx = np.full(m.shape, len(st) - 1, np.int32)
    for t in st[:-1]:
        idx -= (m <= t).astype(np.int32)
    return idx.astype(np.uint8)
