"""Generate golden fixtures by running the REFERENCE DVC forward (build container only).

Run from the repo root:  python tests/golden/gen_golden.py

It imports ``DVC.net.VideoCompressor`` from /root/reference (read-only) with three shims
(SURVEY.md §8(c)): empty stub modules for the absent ``torchvision``/``torchac`` imports
(``basics.py:14``, ``GDN.py:5``, ``net.py:4,15``; neither is called on this path), cwd set
to /root/reference (relative npy path, ``endecoder.py:9``), and ``torch_warp`` replaced by
the same math without ``.cuda()`` (``endecoder.py:52-67`` indexes a cache list with
``device.index`` and moves the grid to CUDA). Weights are the build's seeded state_dict
(``fastvideocodec_amd.weights.seeded_state_dict``), inputs the build's synthetic GOPs.

Outputs ``tests/golden/dvc_<H>x<W>.npz`` (per-stage tensors + the 8 forward outputs) and
``tests/golden/dvc_chain_256x256.npz`` (a 4-frame GOP through the ``parallel_compression``
DVC-pretrained loop, ``models.py:368-383``). The reference never leaves this container;
only these data files are committed.
"""
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "tests", "golden")
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

from fastvideocodec_amd.synthetic import gop_seed, make_gop  # noqa: E402
from fastvideocodec_amd.weights import seeded_torch_state_dict  # noqa: E402

for _n in ["torchvision", "torchvision.models", "torchvision.utils", "torchac"]:
    sys.modules[_n] = types.ModuleType(_n)
sys.modules["torchvision"].models = sys.modules["torchvision.models"]
sys.modules["torchvision"].utils = sys.modules["torchvision.utils"]
sys.modules["torchvision.utils"].save_image = lambda *a, **k: None
sys.path.insert(0, "/root/reference")
os.chdir("/root/reference")

import torch  # noqa: E402
import DVC.subnet.endecoder as E  # noqa: E402


def _cpu_torch_warp(x, flow):
    B, _, H, W = flow.shape
    gh = torch.linspace(-1.0, 1.0, W).view(1, 1, 1, W).expand(B, -1, H, -1)
    gv = torch.linspace(-1.0, 1.0, H).view(1, 1, H, 1).expand(B, -1, -1, W)
    grid = torch.cat([gh, gv], 1)
    f = torch.cat([flow[:, 0:1] / ((x.size(3) - 1.0) / 2.0), flow[:, 1:2] / ((x.size(2) - 1.0) / 2.0)], 1)
    return torch.nn.functional.grid_sample(x, (grid + f).permute(0, 2, 3, 1), mode="bilinear",
                                           padding_mode="border", align_corners=False)


E.torch_warp = _cpu_torch_warp
from DVC.net import VideoCompressor  # noqa: E402

torch.set_num_threads(8)


def build():
    m = VideoCompressor()
    m.load_state_dict(seeded_torch_state_dict())
    m.eval()
    return m


def run_pair(m, cur, ref):
    acts = {}

    def hook(name):
        def f(mod, inp, out):
            acts[name] = out
        return f

    hs = []
    for n, key in [("opticFlow", "estmv"), ("mvEncoder", "mvfeature"), ("mvDecoder", "quant_mv_upsample"),
                   ("resEncoder", "feature"), ("respriorEncoder", "z"), ("respriorDecoder", "recon_sigma"),
                   ("resDecoder", "recon_res")]:
        hs.append(getattr(m, n).register_forward_hook(hook(key)))
    orig_mc = m.motioncompensation

    def mc(refr, mv):
        p, w = orig_mc(refr, mv)
        acts["prediction"], acts["warpframe"] = p, w
        return p, w

    m.motioncompensation = mc
    with torch.no_grad():
        out = m(torch.from_numpy(cur), torch.from_numpy(ref))
    m.motioncompensation = orig_mc
    for h in hs:
        h.remove()
    d = {k: v.numpy().astype(np.float32) for k, v in acts.items()}
    d["quant_mv"] = np.round(d["mvfeature"]).astype(np.float32)
    d["compressed_z"] = np.round(d["z"]).astype(np.float32)
    d["compressed_feature"] = np.round(d["feature"]).astype(np.float32)
    names = ["clipped", "mse_loss", "warploss", "interloss", "bpp_feature", "bpp_z", "bpp_mv", "bpp"]
    for n, o in zip(names, out):
        d[n] = o.numpy().astype(np.float32)
    return d


def main():
    m = build()
    for (H, W) in [(64, 64), (128, 192), (256, 256)]:
        g = make_gop(H, W, 2, gop_seed(0))
        cur, ref = g[1:2].copy(), g[0:1].copy()
        d = run_pair(m, cur, ref)
        d["input_image"], d["referframe"] = cur, ref
        path = os.path.join(OUT, f"dvc_{H}x{W}.npz")
        np.savez_compressed(path, **d)
        print(path, os.path.getsize(path))
    # 4-frame GOP chain at 256x256 (models.py:368-383 loop; frame 0 passed through as the I-frame)
    g = make_gop(256, 256, 4, gop_seed(1))
    x_prev = g[0:1].copy()
    chain = {"gop": g}
    for i in range(1, 4):
        d = run_pair(m, g[i:i + 1].copy(), x_prev)
        for k in ["mse_loss", "warploss", "interloss", "bpp_feature", "bpp_z", "bpp_mv", "bpp",
                  "quant_mv", "compressed_z", "compressed_feature"]:
            chain[f"f{i}_{k}"] = d[k]
        chain[f"f{i}_clipped"] = d["clipped"]
        x_prev = d["clipped"]
    path = os.path.join(OUT, "dvc_chain_256x256.npz")
    np.savez_compressed(path, **chain)
    print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
