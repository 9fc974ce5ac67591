"""Micro-benchmark of single conv geometries at 1080p (for rocprofv3 --pmc / timing)."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402
from fastvideocodec_amd.profiling import conv_flops  # noqa: E402

CASES = {
    "c3_64_full": (64, 64, 3, 1, False, 1088, 1920),
    "c3_128_half": (128, 128, 3, 1, False, 544, 960),
    "c7_32_64_full": (32, 64, 7, 1, False, 1088, 1920),
    "d3_128_half": (128, 128, 3, 2, True, 544, 960),
    "d3_128_quarter": (128, 128, 3, 2, True, 272, 480),
    "d3_128_eighth": (128, 128, 3, 2, True, 136, 240),
    "d3_128_full": (128, 128, 3, 2, True, 1088, 1920),
    "c3_128_2_full": (128, 2, 3, 1, False, 1088, 1920),
    "d5_64_quarter": (64, 64, 5, 2, True, 272, 480),
    "d5_96_64_16": (96, 64, 5, 2, True, 136, 240),
    "c7_32_16_full": (32, 16, 7, 1, False, 1088, 1920),
    "c7_64_32_full": (64, 32, 7, 1, False, 1088, 1920),
    "c3_64_half": (64, 64, 3, 1, False, 544, 960),
    "c3_128_quarter": (128, 128, 3, 1, False, 272, 480),
    "c3_128_eighth": (128, 128, 3, 1, False, 136, 240),
    "c7_8_32_full": (8, 32, 7, 1, False, 1088, 1920),
    "c3_6_64_full": (6, 64, 3, 1, False, 1088, 1920),
    "c3s2_2_128_full": (2, 128, 3, 2, False, 1088, 1920),   # mvEncoder conv1
    "c5s2_3_64_full": (3, 64, 5, 2, False, 1088, 1920),     # resEncoder conv1
    "c3s2_128_half": (128, 128, 3, 2, False, 544, 960),
    "c3_64_3_full": (64, 3, 3, 1, False, 1088, 1920),
    "d5_64_3_half": (64, 3, 5, 2, True, 1088, 1920),
    "c7_16_2_full": (16, 2, 7, 1, False, 1088, 1920),
    # tap-partial GEMMs of the cout <= 4 layers (kernels.PackedConv tap path)
    "c1_128_18_full": (128, 18, 1, 1, False, 1088, 1920),
    "c1_64_27_full": (64, 27, 1, 1, False, 1088, 1920),
    "c1_64_75_half": (64, 75, 1, 1, False, 544, 960),
    # Warp_net ResBlock second conv: relu on the input, residual add in the epilogue
    "c3_64_full_res": (64, 64, 3, 1, False, 1088, 1920, "res"),
    "c3_64_full_relu": (64, 64, 3, 1, False, 1088, 1920, "relu"),   # ResBlock conv1: ReLU in, ReLU act
    "c3_64_half_relu": (64, 64, 3, 1, False, 544, 960, "relu"),
    "c3_64_half_res": (64, 64, 3, 1, False, 544, 960, "res"),
}

ap = argparse.ArgumentParser()
ap.add_argument("--cases", default=",".join(CASES))
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--batch", type=int, default=1)
args = ap.parse_args()
dev = torch.device("cuda")
for name in args.cases.split(","):
    cin, cout, k, s, tr, H, W = CASES[name][:7]
    form = CASES[name][7] if len(CASES[name]) > 7 else ""
    with_res = form == "res"
    if tr:
        H, W = H // 2, W // 2
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k)) * 0.05
    pc = K.PackedConv(w, torch.zeros(cout), k, s, tr, dev)
    B = args.batch
    x = torch.randn(B, H, W, K.cp4(cin), device=dev)
    kw = {}
    if with_res:
        kw = dict(in_op=K.IN_RELU, res=torch.randn(B, *pc.out_hw(H, W), K.cp4(cout), device=dev))
    elif form == "relu":
        kw = dict(in_op=K.IN_RELU, act=K.ACT_RELU)
    y = pc(x, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        pc(x, out=y, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    fl = conv_flops(cin, cout, k, s, tr, B, H, W)
    print(f"{name:16s} {ms:8.3f} ms  {fl / ms / 1e9:8.2f} TF/s", flush=True)
