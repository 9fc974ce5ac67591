"""r6: conv_wr7_kernel time per SpyNet layer and pyramid level at batch B for each work-item
height (FVC_WR7_ROWS = 128 / 64 / 32 / 16, and 0 = the launch's own choice): the data behind
wr7_rows()'s prologue estimate. Also checks that every item height gives bit-identical output."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402
from fastvideocodec_amd.weights import seeded_torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
sd = seeded_torch_state_dict()
levels = [(1088 >> i, 1920 >> i) for i in range(5)]
packs = {}
for name in ("conv2", "conv3", "conv4"):
    w = sd[f"opticFlow.moduleBasic.3.{name}.weight"]
    b = sd[f"opticFlow.moduleBasic.3.{name}.bias"]
    packs[name] = (K.PackedConv(w, b, 7, 1, False, dev, precision="x3"), w.shape[1], w.shape[0])
for B in [int(v) for v in os.environ.get("BATCHES", "1 16").split()]:
    for (H, W) in levels:
        line = [f"B={B:2d} {H}x{W}"]
        for name, (p, cin, cout) in packs.items():
            x = torch.relu(torch.randn(B, H, W, cin, device=dev))
            outs, ts = {}, {}
            for rows in ("128", "64", "32", "16", "0"):
                os.environ["FVC_WR7_ROWS"] = rows
                outs[rows] = p(x, act=K.ACT_RELU)
                torch.cuda.synchronize()
                n = 20 if B * H * W < 4e6 else 5
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(n):
                    p(x, act=K.ACT_RELU)
                e1.record()
                torch.cuda.synchronize()
                ts[rows] = e0.elapsed_time(e1) / n
            os.environ.pop("FVC_WR7_ROWS")
            same = all(torch.equal(outs["128"], o) for o in outs.values())
            line.append(f"{name} {cin}->{cout}: " + " ".join(f"{r}:{ts[r]:.3f}" for r in ts) + ("" if same else " MISMATCH"))
        print(" | ".join(line), flush=True)
