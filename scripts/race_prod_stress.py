"""r6: does any PRODUCTION conv kernel disturb the warp gathers the way the 7x7 stem experiment does
(profiles/r6/race/README.md)? Stream A runs one production conv geometry back to back at 4K; stream B
runs the production motion-compensation warp (fvc_mc_assemble) on fixed inputs and compares every
output with a golden one made while stream A was idle (a device-side count, no host sync per
launch). Prints the mismatching pixel count per antagonist. FVC_LIB_PATH=.../libfvc_k7.so adds the
7x7 8->32 layer on the stem kernel (the experiment that shows the fault) as a positive control."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
H, W = 2176, 3840
ITERS = int(os.environ.get("ITERS", "40"))
# (name, cin, cout, k, stride, transposed, h, w, in_op, act): every split family's production shapes
CASES = [
    ("7x7 8->32 (x3; the stem in a K7 lib)", 8, 32, 7, 1, False, H, W, K.IN_NONE, K.ACT_RELU),
    ("f32 7x7 16->2", 16, 2, 7, 1, False, H, W, K.IN_NONE, K.ACT_NONE),
    ("x3 3x3 s2 128->128", 128, 128, 3, 2, False, H // 2, W // 2, K.IN_NONE, K.ACT_LRELU),
    ("wino 3x3 64->64", 64, 64, 3, 1, False, H, W, K.IN_RELU, K.ACT_RELU),
    ("wr7 7x7 32->64", 32, 64, 7, 1, False, H, W, K.IN_NONE, K.ACT_RELU),
    ("dx deconv 3x3 s2 128->128", 128, 128, 3, 2, True, H // 2, W // 2, K.IN_NONE, K.ACT_LRELU),
    ("stem 3x3 6->64", 6, 64, 3, 1, False, H, W, K.IN_NONE, K.ACT_RELU),
    ("stem 5x5 s2 3->64", 3, 64, 5, 2, False, H, W, K.IN_NONE, K.ACT_NONE),
]
g = torch.Generator().manual_seed(3)
ref = torch.rand(1, H, W, 4, generator=g)
ref[..., 3] = 0
mv = (torch.rand(1, H, W, 4, generator=g) - 0.5) * 6
mv[..., 2:] = 0
ref, mv = ref.to(dev), mv.to(dev)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
with torch.cuda.stream(sb):
    gold, _ = K.mc_assemble(ref, mv)
torch.cuda.synchronize()
only = os.environ.get("CASES")
for name, cin, cout, k, s, tr, h, w, iop, act in CASES:
    if only and not any(o in name for o in only.split(",")):
        continue
    wt = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), generator=g) * (1.0 / (cin * k * k) ** 0.5)
    p = K.PackedConv(wt, torch.zeros(cout), k, s, tr, dev, precision="x3")
    fam = "stem" if p.stem is not None else ("wr7" if p.wr7 else ("wino" if p.wino else ("dx" if p.dx else (
        "x3" if p.x3 else "f32"))))
    x = torch.rand(1, h, w, K.cp4(cin), device=dev)
    x[..., cin:] = 0
    bad = torch.zeros((), dtype=torch.int64, device=dev)
    with torch.cuda.stream(sa):
        p(x, in_op=iop, act=act)  # warm (packs, attributes)
    torch.cuda.synchronize()
    for it in range(ITERS):
        with torch.cuda.stream(sa):
            for _ in range(2):
                p(x, in_op=iop, act=act)
        with torch.cuda.stream(sb):
            for _ in range(4):
                wf, _ = K.mc_assemble(ref, mv)
                bad += (wf != gold).any(-1).sum()
    torch.cuda.synchronize()
    print(f"{name:36s} [{fam:4s}]: {ITERS * 4} warp launches beside {ITERS * 2} conv launches -> mismatching px {int(bad)}",
          flush=True)
