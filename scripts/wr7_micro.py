"""Time the Winograd-rows 7x7 conv alone (SpyNet level-4 layers at 1088x1920, 16 frames per
launch, as the bench batches them) against the direct split kernel: algorithmic TF/s per layer.
Libraries: FVC_LIB_PATH selects an experiment build (python -m fastvideocodec_amd.build --variant)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402
from fastvideocodec_amd.weights import seeded_torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
sd = seeded_torch_state_dict()
B, H, W = int(os.environ.get("B", "16")), 1088, 1920
for name in ("conv2", "conv3", "conv4"):
    w = sd[f"opticFlow.moduleBasic.3.{name}.weight"]
    b = sd[f"opticFlow.moduleBasic.3.{name}.bias"]
    cout, cin = w.shape[:2]
    x = torch.relu(torch.randn(B, H, W, cin, device=dev))
    res = {}
    for tag in ("wr7", "x3"):
        if tag == "x3":
            os.environ["FVC_WR7"] = "0"
        p = K.PackedConv(w, b, 7, 1, False, dev, precision="x3")
        os.environ.pop("FVC_WR7", None)
        p(x, act=K.ACT_RELU)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            p(x, act=K.ACT_RELU)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        res[tag] = (ms, 2.0 * B * H * W * cin * cout * 49 / (ms * 1e-3) / 1e12)
    print(f"{os.environ.get('FVC_LIB_PATH', 'product').split('/')[-1]:24s} {name} {cin}->{cout}: "
          f"wr7 {res['wr7'][0]:.3f} ms {res['wr7'][1]:.1f} TF/s | x3 {res['x3'][0]:.3f} ms {res['x3'][1]:.1f} TF/s",
          flush=True)
    del x
