"""Micro A/B of Warp_net's upsample-add + ResBlock conv1 (endecoder.py:288-293): the standalone
upsample2x_add kernel then the Winograd conv, against the fused form (fvc_conv2d_nhwc_wino_up:
the conv forms skip + up(low) in its staging and writes it once). Batch = the bench's 16 GOPs.
Prints ms per call of each and whether X and y are bit-identical."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--sizes", default="1088x1920,544x960")
ap.add_argument("--order", default="fwd", choices=["fwd", "rev"])
args = ap.parse_args()
dev = torch.device("cuda")
g = torch.Generator().manual_seed(1)
w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
pc = K.PackedConv(w, torch.randn(64, generator=g) * 0.1, 3, 1, False, dev, precision="x3")
assert pc.wino and pc.up_fusable()


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.iters


for hw in args.sizes.split(","):
    H, W = map(int, hw.split("x"))
    B = args.batch
    skip = torch.randn(B, H, W, 64, device=dev)
    low = torch.randn(B, H // 2, W // 2, 64, device=dev)

    def unfused():
        xs = K.upsample2x_add(low, skip=skip, align_corners=True)
        return pc(xs, in_op=K.IN_RELU, act=K.ACT_RELU), xs

    def fused():
        return pc.call_up(skip, low, in_op=K.IN_RELU, act=K.ACT_RELU)

    def up_only():
        return K.upsample2x_add(low, skip=skip, align_corners=True)

    xs0 = up_only()

    def conv_only():
        return pc(xs0, in_op=K.IN_RELU, act=K.ACT_RELU)

    order = [("unfused", unfused), ("fused", fused), ("up_only", up_only), ("conv_only", conv_only)]
    if args.order == "rev":
        order = order[::-1]
    res = {name: timeit(fn) for name, fn in order}
    (yu, xu), (yf, xf) = unfused(), fused()
    torch.cuda.synchronize()
    same = torch.equal(yu, yf) and torch.equal(xu, xf)
    print(f"{H}x{W} b{B}: " + "  ".join(f"{k} {v:.3f} ms" for k, v in res.items()) +
          f"  gain {res['unfused'] - res['fused']:.3f} ms  identical: {same}", flush=True)
    del skip, low, xs0
