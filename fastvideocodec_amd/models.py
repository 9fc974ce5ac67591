"""Drop-in mirror of the reference ``models.py`` surface for the DVC-pretrained path.

``get_codec_model('DVC-pretrained', ...)`` (models.py:32-36 -> get_DVC_pretrained 1432-1445)
returns a ``VideoCompressor`` carrying the attributes the reference GOP driver reads
(``name``, ``compression_level``, ``loss_type``, ``I_level``, ``r``). ``parallel_compression``
(models.py:233-410, DVC-pretrained branch 368-383) and ``PSNR`` (460-473) keep the reference
signatures and return values, so ``eval.py``'s ``static_simulation_model`` can call them
unchanged.

The I-frame codec (BPG via ``os.system``, models.py:412-429) is replaced by a pass-through:
``I_compression`` returns the I-frame losslessly with bpp 0 / PSNR inf, and
``parallel_compression`` leaves a pass-through I-frame out of its aggregates even when
``compressI`` is set (an infinite PSNR would otherwise swamp ``psnr``), so eval.py's averages
stay finite (documented in DESIGN.md).
"""
from __future__ import annotations

import math
import os
import warnings

import torch

from .net import VideoCompressor
from .weights import seeded_torch_state_dict

_RATIO_LIST = [256, 512, 1024, 2048, 2048 * 2, 2048 * 4, 2048 * 8]
_I_LVL_LIST = [37, 32, 27, 22, 17, 12, 7]


class SeededWeightsWarning(UserWarning):
    """The codec runs on the build's seeded (untrained) weights, not a DVC snapshot."""


def get_DVC_pretrained(level, checkpoint=None, seed=20261015, device=None):
    """models.py:1432-1445. The reference loads DVC/snapshot/{r}.model through
    DVC/net.py:21-34 load_model (the snapshots are absent from the reference tree). Here:
    checkpoint=path loads a state_dict the same way (keys the model does not have are dropped,
    as load_model does; they are listed in ``model.dropped_checkpoint_keys``) and a missing file
    raises FileNotFoundError like load_model's open(); checkpoint=None uses the build's seeded
    weights, flagged by ``model.weights_source == 'seeded'`` and a SeededWeightsWarning."""
    model = VideoCompressor()
    model.name = "DVC-pretrained"
    model.compression_level = level
    model.loss_type = "P"
    model.I_level = _I_LVL_LIST[level]
    model.r = _RATIO_LIST[level]
    if checkpoint is not None:
        if not os.path.isfile(checkpoint):
            raise FileNotFoundError(f"DVC checkpoint not found: {checkpoint}")
        sd = torch.load(checkpoint, map_location="cpu", weights_only=True)
        own = model.state_dict()
        model.dropped_checkpoint_keys = sorted(k for k in sd if k not in own)
        missing = sorted(k for k in own if k not in sd)
        own.update({k: v for k, v in sd.items() if k in own})  # net.py:21-34 load_model semantics
        model.load_state_dict(own)
        if model.dropped_checkpoint_keys or missing:
            warnings.warn(f"checkpoint {checkpoint}: {len(model.dropped_checkpoint_keys)} unknown keys dropped, "
                          f"{len(missing)} model keys kept at their initial values", stacklevel=2)
        model.weights_source = checkpoint
    else:
        model.load_state_dict(seeded_torch_state_dict(seed))
        model.dropped_checkpoint_keys = []
        model.weights_source = "seeded"
        warnings.warn(f"DVC-pretrained level {level}: no checkpoint given, using seeded weights (seed {seed}); "
                      "rate-distortion figures are not those of a trained DVC", SeededWeightsWarning, stacklevel=2)
    dev = device if device is not None else (torch.device("cuda") if torch.cuda.is_available() else None)
    if dev is not None:
        model = model.to(dev)
    return model


def get_codec_model(name, loss_type="P", compression_level=2, noMeasure=True, use_split=True, num_views=0,
                    resilience=0, use_attn=True, load_with_copy=False, **kw):
    """models.py:32-66 — the codecs this build implements: 'DVC-pretrained' (the hot path) and
    'RLVC' (IterPredVideoCodecs, models.py:954-1051, eval forward: rlvc.py)."""
    if name in ["DVC-pretrained"]:
        return get_DVC_pretrained(compression_level, **kw)
    if name == "RLVC":
        from .rlvc import get_rlvc_model
        m = get_rlvc_model(**kw)
        m.name, m.loss_type, m.compression_level = name, loss_type, compression_level
        return m
    raise NotImplementedError(f"codec {name!r} is outside this build's scope (DVC-pretrained, RLVC)")


class AverageMeter(object):
    """models.py:1414-1430."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def PSNR(Y1_raw, Y1_com, use_list=False):
    """models.py:460-473 (10*ln(1/mse)/ln(10))."""
    Y1_com = Y1_com.to(Y1_raw.device)
    log10 = math.log(10.0)
    if not use_list:
        train_mse = torch.mean(torch.pow(Y1_raw - Y1_com, 2))
        return 10.0 * torch.log(1 / train_mse) / log10
    out = []
    for i in range(Y1_raw.size(0)):
        train_mse = torch.mean(torch.pow(Y1_raw[i:i + 1] - Y1_com[i:i + 1], 2))
        out.append(10.0 * torch.log(1 / train_mse) / log10)
    return out


def I_compression(Y1_raw, I_level, model_name="", codec=None):
    """models.py:412-429: code the I-frame, return (Y1_com, bpp, psnr). The reference runs
    bpgenc/bpgdec at quality I_level (binaries absent). codec=None (default): lossless
    pass-through (bpp 0, PSNR inf), which the golden GOP fixtures assume; codec="dwt53": the
    build's GPU I-frame codec (fastvideocodec_amd/iframe.py) at the BPG-style step for I_level,
    which reconstructs k/255 frames exactly when the step is 1."""
    if codec is None:
        return Y1_raw, torch.zeros((), device=Y1_raw.device), torch.full((), float("inf"), device=Y1_raw.device)
    if codec != "dwt53":
        raise ValueError(f"unknown I-frame codec {codec!r}")
    from . import iframe as IF
    B, _, H, W = Y1_raw.shape
    bs, Y1_com = IF.encode(Y1_raw.float().contiguous(), IF.iframe_step(I_level))
    bpp = torch.tensor(bs.nbytes() * 8.0 / (B * H * W), device=Y1_raw.device)
    psnr = torch.tensor(IF.psnr(Y1_raw, Y1_com), device=Y1_raw.device)
    return Y1_com, bpp, psnr


def _psnr_from_mse(m):
    return 10.0 * torch.log(1 / m) / math.log(10.0)


def parallel_compression(args, model, data, compressI=False, level=0, batch_idx=0):
    """models.py:233-410 restricted to the DVC-pretrained branch (368-383).

    Returns the reference 11-tuple:
    (x_hat, loss, img_loss, be_loss, be_res_loss, psnr, psnr_list, aux_loss, aux2, aux3, aux4)."""
    if model.name != "DVC-pretrained":
        raise NotImplementedError(model.name)
    img_loss_list, bpp_list, psnr_list = [], [], []
    aux_loss_list, aux2_loss_list = [], []
    x_hat, bpp_i, psnr_i = I_compression(data[0:1], model.I_level, codec=getattr(model, "iframe_codec", None))
    data[0:1] = x_hat
    if compressI and bool(torch.isfinite(psnr_i)):
        # models.py:251-253; a lossless pass-through I-frame (PSNR inf, bpp 0) is left out of
        # the aggregates instead: it would make psnr infinite and bias be_loss towards 0
        bpp_list += [bpp_i]
        psnr_list += [psnr_i]
    B = data.size(0)
    x_prev = data[0:1]
    x_hat_list = []
    for i in range(1, B):
        x_prev, mseloss, warploss, interloss, bpp_feature, bpp_z, bpp_mv, bpp = model(data[i:i + 1], x_prev)
        x_prev = x_prev.detach()
        img_loss_list += [model.r * mseloss]
        aux_loss_list += [_psnr_from_mse(warploss)]
        bpp_list += [bpp]
        psnr_list += [_psnr_from_mse(mseloss)]
        aux2_loss_list += [_psnr_from_mse(interloss)]
        x_hat_list.append(x_prev)
    x_hat = torch.cat(x_hat_list, dim=0) if x_hat_list else data[0:0]
    be_loss = torch.stack(bpp_list, 0).mean(0).cpu().item() if bpp_list else 0
    img_loss = 0  # reference: only set when all_loss_list is non-empty (never for DVC-pretrained)
    psnr = torch.stack(psnr_list, 0).mean(0).cpu().item() if psnr_list else 0
    aux_loss = torch.stack(aux_loss_list, 0).mean(0).cpu().item() if aux_loss_list else 0
    aux2_loss = torch.stack(aux2_loss_list, 0).mean(0).cpu().item() if aux2_loss_list else 0
    psnrs = torch.stack(psnr_list, 0).tolist() if psnr_list else []
    return x_hat, 0, img_loss, be_loss, 0, psnr, psnrs, aux_loss, aux2_loss, 0, 0
