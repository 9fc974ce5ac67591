"""Micro-benchmark of the LDS tap gathers (fvc_tap_gather_nhwc) at the bench's sizes: Warp_net
conv6 (3x3 64 -> 3, stride 1, + warpframe residual; endecoder.py:278-279) and mvDecoder deconv8
(3x3 transposed 128 -> 2, stride 2; synthesis_mv.py:41-43), 8 frames of 1088x1920. A/B of an env
switch (0 vs 1; ORDER=rev measures 1 first) with a bit-identity check. r5 used it for
FVC_GATHER_NT, non-temporal P staging, since reverted (profiles/r5/gather_nt).

usage: python scripts/gather_micro.py VAR"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import kernels as K  # noqa: E402

var = sys.argv[1] if len(sys.argv) > 1 else "FVC_GATHER_NT"
dev = torch.device("cuda")
B = 8
g = torch.Generator(device=dev).manual_seed(3)


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
    "conv6_s1": (torch.randn(3, 64, 3, 3) * 0.05, 3, 1, False, (1088, 1920), True),
    "deconv8_t2": (torch.randn(128, 2, 3, 3) * 0.05, 3, 2, True, (544, 960), False),
}
for name, (w, k, s, tr, (h, wd), with_res) in cases.items():
    cout = w.shape[1] if tr else w.shape[0]
    tap = K.TapConsumer(w, torch.zeros(cout), k, s, tr, dev)
    P = torch.randn(B, h, wd, tap.pcp, device=dev, generator=g)
    ho, wo = (2 * h, 2 * wd) if tr else (h, wd)
    res = torch.randn(B, ho, wo, 4, device=dev, generator=g) if with_res else None
    outs = []
    for v in (("1", "0") if os.environ.get("ORDER") == "rev" else ("0", "1")):
        os.environ[var] = v
        ms = timeit(lambda: tap.gather(P, res=res))
        outs.append(tap.gather(P, res=res))
        nb = 4 * (P.numel() + B * ho * wo * 4 * (2 if with_res else 1))
        print(f"{name:12s} {var}={v} {ms:7.3f} ms {nb / ms / 1e6:8.1f} GB/s", flush=True)
    torch.cuda.synchronize()
    print(f"{name:12s} identical: {torch.equal(outs[0], outs[1])}", flush=True)
