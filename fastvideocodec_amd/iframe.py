"""I-frame codec on the GPU, replacing the reference's BPG I-frame
(``models.py:412-429`` I_compression: ``bpgenc -q I_level`` / ``bpgdec`` through os.system; the
binaries are not in the reference tree or this image).

Pipeline (csrc/fvc_iframe.hip; numpy restatement oracle/iframe_ref.py):
  8-bit samples -> JPEG 2000 reversible colour transform -> LEVELS levels of the reversible
  LeGall 5/3 lifting wavelet -> dead-zone quantisation of the high-pass subbands with step q
  (q = 1: lossless) -> device rANS of every coefficient under the codec's Laplace tables, the
  table of each 32 x 32 block chosen from its mean |coefficient| (the block indexes travel in
  the bitstream) -> one stream per BAND_ROWS rows of a plane.
The quantiser step follows the BPG/HEVC QP convention the reference's I_level uses (step doubles
every 6 levels): q = round(2^((I_level - 6) / 6)), so level 2's I_level 27 gives q = 11;
I_level <= 6 (or q=1) is lossless. Integer arithmetic throughout: the encoder's reconstruction
is bit-identical to the decoder's.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from . import kernels as K
from .entropy_models import EncodedStreams, LaplaceTables, RangeCoder

LEVELS = 4
BLOCK = 32
BAND_ROWS = 4


def iframe_step(I_level) -> int:
    """Quantiser step for a BPG-style I_level (models.py:1439 _I_LVL_LIST: 37 .. 7)."""
    if I_level is None:
        return 1
    return max(1, int(round(2.0 ** ((float(I_level) - 6.0) / 6.0))))


class IFrameBitstream:
    """An I-frame batch: geometry, quantiser, per-block table indexes (uint8, host) and the range
    coded coefficient streams (one per BAND_ROWS rows of each plane)."""

    def __init__(self, batch, h, w, levels, q, block_index, streams: EncodedStreams):
        self.batch, self.h, self.w, self.levels, self.q = batch, h, w, levels, q
        self.block_index = block_index
        self.streams = streams

    def nbytes(self) -> int:
        return int(self.streams.pack_off[-1].item()) * 4 + int(np.asarray(self.block_index).size)


_CODERS = {}


def _coder(device):
    key = str(device)
    if key not in _CODERS:
        t = LaplaceTables()
        _CODERS[key] = (RangeCoder(t.cdf, t.cdf_length, t.offset, device),
                        torch.from_numpy(t.scale_table).to(device))
    return _CODERS[key]


def _check(h, w, levels):
    if h % BLOCK or w % BLOCK or h % (1 << levels) or w % (1 << levels) or h % BAND_ROWS:
        raise ValueError(f"I-frame size {h}x{w} must be a multiple of {max(BLOCK, 1 << levels)}")


def _dwt(c, levels, inverse):
    P, h, w = c.shape[0] * c.shape[1], c.shape[2], c.shape[3]
    tmp = torch.empty_like(c)
    _lib.call("fvc_iframe_dwt53", c.data_ptr(), tmp.data_ptr(), P, h, w, levels, int(inverse), K.stream_handle())


def _reconstruct(coef, levels, q):
    """quantised coefficients [B,3,h,w] int32 (consumed) -> frames [B,3,h,w] float32."""
    B, _, h, w = coef.shape
    _lib.call("fvc_iframe_quant", coef.data_ptr(), 3 * B, h, w, levels, q, 1, K.stream_handle())
    _dwt(coef, levels, True)
    out = torch.empty(coef.shape, dtype=torch.float32, device=coef.device)
    _lib.call("fvc_iframe_rct_inv", coef.data_ptr(), out.data_ptr(), B, h, w, K.stream_handle())
    return out


def encode(frames: torch.Tensor, q: int = 1, levels: int = LEVELS):
    """frames [B,3,h,w] device float in [0,1] -> (IFrameBitstream, reconstruction [B,3,h,w])."""
    K._chk(frames, name="frames")
    B, C, h, w = frames.shape
    if C != 3:
        raise ValueError("I-frames are [B,3,H,W]")
    _check(h, w, levels)
    if q < 1:
        raise ValueError("quantiser step must be >= 1")
    coder, table = _coder(frames.device)
    st = K.stream_handle()
    coef = torch.empty((B, 3, h, w), dtype=torch.int32, device=frames.device)
    with torch.no_grad():
        _lib.call("fvc_iframe_rct_fwd", frames.data_ptr(), coef.data_ptr(), B, h, w, st)
        _dwt(coef, levels, False)
        _lib.call("fvc_iframe_quant", coef.data_ptr(), 3 * B, h, w, levels, q, 0, st)
        bidx = torch.empty((3 * B, h // BLOCK, w // BLOCK), dtype=torch.uint8, device=frames.device)
        idx = torch.empty_like(coef)
        _lib.call("fvc_iframe_block_index", coef.data_ptr(), table.data_ptr(), table.numel(), bidx.data_ptr(),
                  idx.data_ptr(), 3 * B, h, w, BLOCK, st)
        S = 3 * B * h // BAND_ROWS
        enc = coder.encode(coef.view(S, BAND_ROWS * w), idx.view(S, BAND_ROWS * w))
        recon = _reconstruct(coef.clone(), levels, q)
    return IFrameBitstream(B, h, w, levels, q, bidx.cpu().numpy(), enc), recon


def decode(bs: IFrameBitstream, device=None, check=True) -> torch.Tensor:
    """IFrameBitstream -> frames [B,3,h,w] float32 on the device (bit-identical to the encoder's
    reconstruction)."""
    dev = bs.streams.packed.device if device is None else torch.device(device)
    coder, _ = _coder(dev)
    B, h, w = bs.batch, bs.h, bs.w
    with torch.no_grad():
        bidx = torch.from_numpy(np.ascontiguousarray(bs.block_index, np.uint8)).to(dev)
        idx = torch.empty((B, 3, h, w), dtype=torch.int32, device=dev)
        _lib.call("fvc_iframe_expand_index", bidx.data_ptr(), idx.data_ptr(), 3 * B, h, w, BLOCK, K.stream_handle())
        S = 3 * B * h // BAND_ROWS
        coef = coder.decode(bs.streams, idx.view(S, BAND_ROWS * w), check).view(B, 3, h, w)
        return _reconstruct(coef, bs.levels, bs.q)


def psnr(a: torch.Tensor, b: torch.Tensor) -> float:
    mse = float(torch.mean((a.double() - b.double()) ** 2))
    return float("inf") if mse == 0 else 10.0 * math.log10(1.0 / mse)
