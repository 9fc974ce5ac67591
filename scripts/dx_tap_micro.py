"""Micro-benchmark of mvDecoder deconv7 -> deconv8 as the bench runs it: the stride-2 transposed
3x3 128->128 conv on conv_dx_kernel with deconv8's (3x3 128->2) tap partials in its epilogue
(synthesis_mv.py:41-43), at 544x960 -> 1088x1920, then the tap gather. FVC_LIB_PATH selects an
experiment library (e.g. a -DFVC_DX_KO knock-out build)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402
from fastvideocodec_amd.profiling import conv_flops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--h", type=int, default=544)
ap.add_argument("--w", type=int, default=960)
args = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(0)
w7 = torch.randn(128, 128, 3, 3) * 0.03
w8 = torch.randn(2, 128, 3, 3) * 0.03
pc = K.PackedConv(w7, torch.zeros(128), 3, 2, True, dev)
tap = K.TapConsumer(w8, torch.zeros(2), 3, 1, False, dev)
assert pc.tap_fusable(tap)
B, H, W = args.batch, args.h, args.w
x = torch.randn(B, H, W, 128, device=dev)
P = pc.call_tap(x, tap, act=K.ACT_RELU)
torch.cuda.synchronize()
e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
e0.record()
for _ in range(args.iters):
    P = pc.call_tap(x, tap, act=K.ACT_RELU)
e1.record()
for _ in range(args.iters):
    tap.gather(P)
e2.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / args.iters
msg = e1.elapsed_time(e2) / args.iters
fl = conv_flops(128, 128, 3, 2, True, B, H, W)
print(f"deconv7+tap  {ms:8.3f} ms  {fl / ms / 1e9:8.2f} TF/s (deconv FLOP)   gather {msg:.3f} ms", flush=True)
