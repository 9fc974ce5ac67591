"""Debug aid (r5): SpyNet's first layer (7x7 8 -> 32) on conv_stem_kernel (-DFVC_STEM_K7 library via
FVC_LIB_PATH) against the direct x3 kernel at pyramid sizes, batch 1 / 16: max difference of scale,
determinism, overflow flag."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402
from fastvideocodec_amd.weights import seeded_torch_state_dict  # noqa: E402

dev = torch.device("cuda")
sd = seeded_torch_state_dict()
w = sd["opticFlow.moduleBasic.3.conv1.weight"]
b = sd["opticFlow.moduleBasic.3.conv1.bias"]
os.environ["FVC_STEM"] = "1"
ps = K.PackedConv(w, b, 7, 1, False, dev, precision="x3")
os.environ["FVC_STEM"] = "0"
pd = K.PackedConv(w, b, 7, 1, False, dev, precision="x3")
print("stem path:", ps.stem is not None, flush=True)
g = torch.Generator().manual_seed(0)
for B, H, W in [(1, 136, 240), (1, 1088, 1920), (16, 1088, 1920), (1, 2176, 3840)]:
    x = torch.rand(B, H, W, 8, generator=g) * 2 - 1
    x[..., 6:] *= 20.0  # flow channels
    xd = x.to(dev)
    K.x3_overflow(reset=True)
    ys, yd = ps(xd, act=K.ACT_RELU), pd(xd, act=K.ACT_RELU)
    ys2 = ps(xd, act=K.ACT_RELU)
    torch.cuda.synchronize()
    ovf = K.x3_overflow(reset=True)
    d = float((ys - yd).abs().max() / yd.abs().max())
    print(f"B{B} {H}x{W}: diff {d:.2e} det {torch.equal(ys, ys2)} ovf {ovf} nan {int(torch.isnan(ys).sum())}", flush=True)
