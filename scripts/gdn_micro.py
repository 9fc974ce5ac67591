"""GDN kernel timing at the DVC residual-codec resolutions (64 channels)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
beta = torch.rand(64, device=dev) + 0.5
gamma = torch.rand(64, 64, device=dev) * 0.1
for h, w in ((544, 960), (272, 480), (136, 240)):
    x = torch.randn(1, h, w, 64, device=dev)
    y = K.gdn(x, beta, gamma, False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        y = K.gdn(x, beta, gamma, False)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    gb = 2 * x.numel() * 4 / 1e9
    print(f"gdn {h}x{w}x64: {ms:.4f} ms  {gb / ms * 1e3:.0f} GB/s", flush=True)
