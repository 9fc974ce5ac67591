"""Micro-benchmark of the HBM-bound kernels at the bench's sizes (8 images of 1920x1088), with the
env switch of an A/B given on the command line: prints GB/s of algorithmic bytes per kernel and
checks the two variants give identical bits.

usage: python scripts/hbm_micro.py VAR   (runs each kernel with VAR=0 and VAR=1)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402

var = sys.argv[1] if len(sys.argv) > 1 else "FVC_UP2_Q16"
dev = torch.device("cuda")
B = 8
g = torch.Generator(device=dev).manual_seed(1)


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


cases = {
    "up2_add_full": (544, 960, 64),
    "up2_add_half": (272, 480, 64),
}
for name, (h, w, c) in cases.items():
    src = torch.randn(B, h, w, c, device=dev, generator=g)
    skip = torch.randn(B, 2 * h, 2 * w, c, device=dev, generator=g)
    outs = []
    for v in (("1", "0") if os.environ.get("ORDER") == "rev" else ("0", "1")):
        os.environ[var] = v
        ms = timeit(lambda: K.upsample2x_add(src, skip))
        outs.append(K.upsample2x_add(src, skip))
        nb = 4 * (src.numel() + 2 * skip.numel())
        print(f"{name:14s} {var}={v} {ms:7.3f} ms {nb / ms / 1e6:8.1f} GB/s", flush=True)
    torch.cuda.synchronize()
    print(f"{name:14s} identical: {torch.equal(outs[0], outs[1])}")
