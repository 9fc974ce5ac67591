"""GOP driver for real encode+decode (the bitstream counterpart of models.parallel_compression,
models.py:368-383): the I-frame passes through (BPG out of scope), every P-frame is encoded
against the previous *decoded* frame and decoded from its bitstream.

G GOPs are processed together as a batch (frame t of every GOP in one forward), which
raises occupancy on the small late layers; GOPs are independent, so this is the per-GPU
analogue of sharding GOPs across ranks.
"""
from __future__ import annotations

import torch


def encode_decode_gop(model, frames: torch.Tensor, check=False):
    """frames: [G, T, 3, H, W] device tensor. Returns (bitstreams, decoded [G,T-1,3,H,W] list,
    sse list, encoder recon list)."""
    G, T = frames.shape[:2]
    x_prev = frames[:, 0].contiguous()
    bitstreams, decoded, sses, enc_recons = [], [], [], []
    for t in range(1, T):
        cur = frames[:, t].contiguous()
        bs, rec_enc, sse = model.compress(cur, x_prev, return_sse=True)
        rec_dec = model.decompress(bs, x_prev, check=check)
        bitstreams.append(bs)
        decoded.append(rec_dec)
        enc_recons.append(rec_enc)
        sses.append(sse)
        x_prev = rec_dec
    return bitstreams, decoded, sses, enc_recons
