"""Seeded synthetic GOP generator (stands in for ``dataset.py:VideoDataset``, which needs
cv2 + video files; see SURVEY.md §8(d) "Synthetic inputs").

* base frame: 3-channel sum of 8 random 2-D sinusoids (1-32 cycles/frame) plus
  U(-0.02, 0.02) noise, normalised to [0, 1];
* P-frame t: bilinear shift of the base by (1.25 t, 0.5 t) px plus a smooth local
  displacement field (<= 2 px) plus N(0, 0.01^2) noise, clamped and quantised to k/255
  (what ``transforms.ToTensor`` of an 8-bit frame gives, ``dataset.py:58-86``);
* frames are generated at the source size and replicate-padded to multiples of 64
  (the reference forward needs H, W % 64 == 0, SURVEY.md §7 "Size constraint").

Seed convention: ``seed = 20261015 + 1000 * gop + view``.
"""
from __future__ import annotations

import numpy as np


def gop_seed(gop: int = 0, view: int = 0) -> int:
    return 20261015 + 1000 * gop + view


def _bilinear_sample(img: np.ndarray, sx: np.ndarray, sy: np.ndarray) -> np.ndarray:
    """Sample img [C,H,W] at float coords (x=col, y=row), edge-clamped."""
    C, H, W = img.shape
    sx = np.clip(sx, 0, W - 1)
    sy = np.clip(sy, 0, H - 1)
    x0 = np.floor(sx).astype(np.int64)
    y0 = np.floor(sy).astype(np.int64)
    x1 = np.minimum(x0 + 1, W - 1)
    y1 = np.minimum(y0 + 1, H - 1)
    wx = (sx - x0).astype(np.float32)
    wy = (sy - y0).astype(np.float32)
    out = np.empty_like(img)
    for c in range(C):
        p = img[c]
        out[c] = ((p[y0, x0] * (1 - wx) + p[y0, x1] * wx) * (1 - wy)
                  + (p[y1, x0] * (1 - wx) + p[y1, x1] * wx) * wy)
    return out


def pad_to_multiple(frames: np.ndarray, m: int = 64) -> np.ndarray:
    """Replicate-pad [..., H, W] up to multiples of m."""
    H, W = frames.shape[-2:]
    Hp = (H + m - 1) // m * m
    Wp = (W + m - 1) // m * m
    if (Hp, Wp) == (H, W):
        return frames
    pad = [(0, 0)] * (frames.ndim - 2) + [(0, Hp - H), (0, Wp - W)]
    return np.pad(frames, pad, mode="edge")


def make_gop(height: int, width: int, gop_size: int, seed: int, pad: int = 64) -> np.ndarray:
    """Return a float32 array [gop_size, 3, Hp, Wp] in [0, 1] (k/255 values)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    H, W = height, width
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    base = np.zeros((3, H, W), np.float32)
    for c in range(3):
        for _ in range(8):
            fx = rng.uniform(1, 32) / W
            fy = rng.uniform(1, 32) / H
            ph = rng.uniform(0, 2 * np.pi)
            amp = rng.uniform(0.2, 1.0)
            base[c] += (amp * np.sin(2 * np.pi * (fx * xx + fy * yy) + ph)).astype(np.float32)
    base += rng.uniform(-0.02, 0.02, size=base.shape).astype(np.float32) * (base.max() - base.min())
    base = (base - base.min()) / (base.max() - base.min())
    # smooth local displacement field, <= 2 px
    fxl, fyl = rng.uniform(1, 3, size=2)
    phl = rng.uniform(0, 2 * np.pi, size=2)
    dxl = 2.0 * np.sin(2 * np.pi * fxl * yy / H + phl[0]).astype(np.float32)
    dyl = 2.0 * np.sin(2 * np.pi * fyl * xx / W + phl[1]).astype(np.float32)
    frames = np.empty((gop_size, 3, H, W), np.float32)
    for t in range(gop_size):
        s = t / max(gop_size - 1, 1)
        sx = xx - 1.25 * t - s * dxl
        sy = yy - 0.5 * t - s * dyl
        f = _bilinear_sample(base, sx, sy)
        if t > 0:
            f = f + rng.normal(0.0, 0.01, size=f.shape).astype(np.float32)
        f = np.clip(f, 0.0, 1.0)
        frames[t] = np.round(f * 255.0).astype(np.float32) / np.float32(255.0)
    if pad:
        frames = pad_to_multiple(frames, pad)
    return np.ascontiguousarray(frames, dtype=np.float32)


def make_pair(height: int, width: int, seed: int):
    """(input_image, referframe) pair, each [1,3,H,W]: ref = frame 0, cur = frame 1."""
    g = make_gop(height, width, 2, seed)
    return g[1:2].copy(), g[0:1].copy()
