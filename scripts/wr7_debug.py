import os, sys, torch
sys.path.insert(0, os.getcwd())
from fastvideocodec_amd import kernels as K
dev = torch.device("cuda:0")
def packs(w, b):
    pw = K.PackedConv(w, b, 7, 1, False, dev, precision="x3")
    os.environ["FVC_WR7"] = "0"; pd = K.PackedConv(w, b, 7, 1, False, dev, precision="x3"); del os.environ["FVC_WR7"]
    return pw, pd
for (cin, cout, B, H, W) in [(32, 64, 4, 600, 640), (64, 32, 4, 600, 640), (32, 64, 16, 1088, 1920)]:
    g = torch.Generator().manual_seed(1)
    x = torch.relu(torch.randn(B, H, W, cin, generator=g)).to(dev)
    w = torch.randn(cout, cin, 7, 7, generator=g) * (1.0 / (cin * 49) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    pw, pd = packs(w, b)
    K.x3_overflow(reset=True)
    y1 = pw(x, act=K.ACT_RELU); y2 = pw(x, act=K.ACT_RELU); yd = pd(x, act=K.ACT_RELU)
    torch.cuda.synchronize()
    ovf = K.x3_overflow(reset=True)
    d = (y1 - yd).abs()
    print(cin, cout, B, H, W, "det", torch.equal(y1, y2), "ndiff", int((y1 != y2).sum()), "max|wr7-direct|/scale",
          float(d.max() / yd.abs().max()), "nan", bool(torch.isnan(y1).any()), "ovf", ovf, flush=True)
    if d.max() / yd.abs().max() > 1e-5:
        idx = (d > 1e-5 * yd.abs().max()).nonzero()
        print("bad count", idx.shape[0], "first", idx[:10].tolist(), flush=True)
        rows = idx[:, 1].unique()
        print("bad rows", rows[:40].tolist(), "row mod 128", (rows % 128).unique()[:40].tolist(), flush=True)
        cols = idx[:, 2].unique(); print("bad cols", cols[:40].tolist(), flush=True)
