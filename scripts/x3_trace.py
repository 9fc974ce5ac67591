"""Segment shares of conv_x3_kernel waves from a -D FVC_X3_TRACE=1 build (diagnostic only).

Run with FVC_LIB_PATH pointing at the trace library; prints, per geometry, the share of each
k-loop segment in the waves' cycles (sums over all waves of the last launch)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import _lib, kernels as K  # noqa: E402

CASES = {  # subset of scripts/conv_micro.py
    "c3_64_full": (64, 64, 3, 1, False, 1088, 1920),
    "c3_128_half": (128, 128, 3, 1, False, 544, 960),
    "c7_32_64_full": (32, 64, 7, 1, False, 1088, 1920),
    "d3_128_half": (128, 128, 3, 2, True, 544, 960),
}

NAMES = ["prologue", "load issue", "mfma", "stage store", "chunk end", "epilogue"]
lib = _lib.load()
fn = lib.fvc_x3_trace_read
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
slots = 1 << 16
buf = np.zeros((slots, 8), np.uint64)
dev = torch.device("cuda")
for name in os.environ.get("TRACE_CASES", "c3_64_full").split(","):
    cin, cout, k, s, tr, H, W = CASES[name][:7]
    if tr:
        H, W = H // 2, W // 2
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k)) * 0.05
    pc = K.PackedConv(w, torch.zeros(cout), k, s, tr, dev)
    x = torch.randn(4, H, W, K.cp4(cin), device=dev)
    for _ in range(3):
        y = pc(x)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, slots)  # clear
    y = pc(x)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, slots) == 0
    used = buf[buf[:, 7] > 0].astype(np.float64)
    tot = used[:, 6].sum()
    seg = used[:, :6].sum(0)
    print(f"{name}: waves {len(used)}, mean wave cycles {used[:, 6].mean():.0f}, "
          + ", ".join(f"{n} {v / tot * 100:.1f}%" for n, v in zip(NAMES, seg))
          + f", unaccounted {(tot - seg.sum()) / tot * 100:.1f}%", flush=True)
