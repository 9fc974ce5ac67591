"""Tiny Winograd-kernel cases against a float64 conv, with the error's location (debug aid).
   FVC_LIB_PATH selects an experiment library."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import torch.nn.functional as F
from fastvideocodec_amd import kernels as K

dev = torch.device("cuda")
torch.manual_seed(0)
for (B, H, W) in [(1, 2, 30), (1, 4, 32), (1, 40, 72), (2, 37, 70)]:
    w = torch.randn(64, 64, 3, 3) * 0.05
    b = torch.randn(64) * 0.1
    pc = K.PackedConv(w, b, 3, 1, False, dev)
    assert pc.wino, "not on the Winograd kernel"
    x = torch.randn(B, H, W, 64, device=dev)
    y = pc(x)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double().permute(0, 3, 1, 2).cpu(), w.double(), b.double(), padding=1).permute(0, 2, 3, 1)
    d = (y.double().cpu() - ref).abs()
    bad = ~(d <= 1e-4)
    print(f"B{B} {H}x{W}: max err {float(d[~torch.isnan(d)].max()) if (~torch.isnan(d)).any() else float('nan'):.3e}, "
          f"bad {int(bad.sum())} of {bad.numel()}, nan {int(torch.isnan(y).sum())}", flush=True)
    if bad.any():
        idx = bad.nonzero()
        rows = sorted(set(idx[:, 1].tolist()))
        cols = sorted(set(idx[:, 2].tolist()))
        chs = sorted(set(idx[:, 3].tolist()))
        print("  bad rows", rows[:20], "cols", cols[:40], "chans", chs[:64], flush=True)
        print("  sample y", y[0, 0, 0, :8].tolist(), "ref", ref[0, 0, 0, :8].tolist(), flush=True)
