"""Seeded weights for the DVC P-frame codec (no trained checkpoint exists offline).

The reference's trained snapshots ``DVC/snapshot/{256,512,1024,2048}.model`` are not in
the repository (``models.py:1443``), so every parity fixture and every benchmark uses a
seeded state_dict whose keys and shapes are exactly those of the reference
``DVC/net.py:VideoCompressor`` (so a real checkpoint drops in via ``load_state_dict``).

* SpyNet levels L1-L4 carry the reference's pretrained numpy weights
  (``DVC/flow_pretrain_np``, loaded by ``endecoder.py:122-140``), shipped as data in
  ``data/spynet_l1_l4.npz``.
* Every other tensor follows the reference initialiser of that layer (xavier-normal with
  the per-layer gains of ``analysis_mv.py:14-44``, ``synthesis_mv.py:15-42``,
  ``analysis.py:16-29``, ``synthesis.py:14-27``, ``analysis_prior.py:17-25``,
  ``synthesis_prior.py:17-25``; xavier-uniform for ``Warp_net``/``ResBlock``
  ``endecoder.py:232-240,267-279``; GDN init ``GDN.py:45-61``; BitEstimator
  ``N(0, 0.01)`` ``bitEstimator.py:13-17``), drawn from numpy PCG64 so the values are
  identical on every machine.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import numpy as np

_DATA = os.path.join(os.path.dirname(__file__), "data", "spynet_l1_l4.npz")

# channel constants, DVC/subnet/basics.py:23-27
OUT_CHANNEL_N = 64
OUT_CHANNEL_M = 96
OUT_CHANNEL_MV = 128


def _xavier_normal(rng, shape, gain, transposed=False):
    rf = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    # torch computes fan_in from dim 1 and fan_out from dim 0 for both conv and deconv
    fan_in = shape[1] * rf
    fan_out = shape[0] * rf
    std = gain * math.sqrt(2.0 / float(fan_in + fan_out))
    return (rng.standard_normal(shape) * std).astype(np.float32)


def _xavier_uniform(rng, shape, gain=1.0):
    rf = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    fan_in = shape[1] * rf
    fan_out = shape[0] * rf
    bound = gain * math.sqrt(6.0 / float(fan_in + fan_out))
    return rng.uniform(-bound, bound, size=shape).astype(np.float32)


def _gdn(ch):
    pedestal = (2.0 ** -18) ** 2
    beta = np.sqrt(np.ones(ch, np.float32) + np.float32(pedestal)).astype(np.float32)
    gamma = np.sqrt(np.float32(0.1) * np.eye(ch, dtype=np.float32) + np.float32(pedestal)).astype(np.float32)
    return beta, gamma


def seeded_state_dict(seed: int = 20261015) -> "OrderedDict[str, np.ndarray]":
    """Return a reference-keyed state_dict of float32 numpy arrays."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    spy = np.load(_DATA)
    for lvl in range(4):
        for f in range(1, 6):
            sd[f"opticFlow.moduleBasic.{lvl}.conv{f}.weight"] = spy[f"modelL{lvl+1}_F-{f}-weight"].astype(np.float32)
            sd[f"opticFlow.moduleBasic.{lvl}.conv{f}.bias"] = spy[f"modelL{lvl+1}_F-{f}-bias"].astype(np.float32)

    mv = OUT_CHANNEL_MV
    # Analysis_mv_net (analysis_mv.py:14-44)
    for i in range(1, 9):
        cin = 2 if i == 1 else mv
        gain = math.sqrt(2 * (2 + mv) / 4) if i == 1 else math.sqrt(2)
        sd[f"mvEncoder.conv{i}.weight"] = _xavier_normal(rng, (mv, cin, 3, 3), gain)
        sd[f"mvEncoder.conv{i}.bias"] = np.full(mv, 0.01, np.float32)
    # Synthesis_mv_net (synthesis_mv.py:15-42); odd layers are ConvTranspose2d [Cin,Cout,k,k]
    for i in range(1, 9):
        cout = 2 if i == 8 else mv
        gain = math.sqrt(2 * 1 * (mv + 2) / (mv + mv)) if i == 8 else math.sqrt(2)
        shape = (mv, cout, 3, 3) if i % 2 == 1 else (cout, mv, 3, 3)
        sd[f"mvDecoder.deconv{i}.weight"] = _xavier_normal(rng, shape, gain)
        sd[f"mvDecoder.deconv{i}.bias"] = np.full(cout, 0.01, np.float32)
    # Warp_net (endecoder.py:262-279), ResBlock (228-246): xavier_uniform, zero bias
    sd["warpnet.feature_ext.weight"] = _xavier_uniform(rng, (64, 6, 3, 3))
    sd["warpnet.feature_ext.bias"] = np.zeros(64, np.float32)
    for r in range(6):
        for c in (1, 2):
            sd[f"warpnet.conv{r}.conv{c}.weight"] = _xavier_uniform(rng, (64, 64, 3, 3))
            sd[f"warpnet.conv{r}.conv{c}.bias"] = np.zeros(64, np.float32)
    sd["warpnet.conv6.weight"] = _xavier_uniform(rng, (3, 64, 3, 3))
    sd["warpnet.conv6.bias"] = np.zeros(3, np.float32)
    N, M = OUT_CHANNEL_N, OUT_CHANNEL_M
    # Analysis_net (analysis.py:16-29)
    gains = [math.sqrt(2 * (3 + N) / 6), math.sqrt(2), math.sqrt(2), math.sqrt(2 * (M + N) / (N + N))]
    cins = [3, N, N, N]
    couts = [N, N, N, M]
    for i in range(4):
        sd[f"resEncoder.conv{i+1}.weight"] = _xavier_normal(rng, (couts[i], cins[i], 5, 5), gains[i])
        sd[f"resEncoder.conv{i+1}.bias"] = np.full(couts[i], 0.01, np.float32)
        if i < 3:
            b, g = _gdn(N)
            sd[f"resEncoder.gdn{i+1}.beta"] = b
            sd[f"resEncoder.gdn{i+1}.gamma"] = g
    # Synthesis_net (synthesis.py:14-27): ConvTranspose2d weights [Cin,Cout,5,5]
    gains = [math.sqrt(2 * (N + M) / (M + M)), math.sqrt(2), math.sqrt(2), math.sqrt(2 * (N + 3) / (N + N))]
    cins = [M, N, N, N]
    couts = [N, N, N, 3]
    for i in range(4):
        sd[f"resDecoder.deconv{i+1}.weight"] = _xavier_normal(rng, (cins[i], couts[i], 5, 5), gains[i])
        sd[f"resDecoder.deconv{i+1}.bias"] = np.full(couts[i], 0.01, np.float32)
        if i < 3:
            b, g = _gdn(N)
            sd[f"resDecoder.igdn{i+1}.beta"] = b
            sd[f"resDecoder.igdn{i+1}.gamma"] = g
    # Analysis_prior_net (analysis_prior.py:17-25)
    sd["respriorEncoder.conv1.weight"] = _xavier_normal(rng, (N, M, 3, 3), math.sqrt(2 * (M + N) / (M + M)))
    sd["respriorEncoder.conv1.bias"] = np.full(N, 0.01, np.float32)
    for i in (2, 3):
        sd[f"respriorEncoder.conv{i}.weight"] = _xavier_normal(rng, (N, N, 5, 5), math.sqrt(2))
        sd[f"respriorEncoder.conv{i}.bias"] = np.full(N, 0.01, np.float32)
    # Synthesis_prior_net (synthesis_prior.py:17-25)
    for i in (1, 2):
        sd[f"respriorDecoder.deconv{i}.weight"] = _xavier_normal(rng, (N, N, 5, 5), math.sqrt(2))
        sd[f"respriorDecoder.deconv{i}.bias"] = np.full(N, 0.01, np.float32)
    sd["respriorDecoder.deconv3.weight"] = _xavier_normal(rng, (N, M, 3, 3), math.sqrt(2 * (N + M) / (N + N)))
    sd["respriorDecoder.deconv3.bias"] = np.full(M, 0.01, np.float32)
    # BitEstimator (bitEstimator.py:6-42)
    for name, ch in (("bitEstimator_z", N), ("bitEstimator_mv", mv)):
        for f in range(1, 5):
            for p in (("h", "b", "a") if f < 4 else ("h", "b")):
                sd[f"{name}.f{f}.{p}"] = (rng.standard_normal((1, ch, 1, 1)) * 0.01).astype(np.float32)
    return sd


def seeded_torch_state_dict(seed: int = 20261015):
    import torch
    return OrderedDict((k, torch.from_numpy(np.ascontiguousarray(v))) for k, v in seeded_state_dict(seed).items())
