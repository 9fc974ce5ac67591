"""Micro-benchmark of the device rANS coder on 1080p-shaped latents (96 feature channels with
Laplace scale tables, 128 mv channels with factorized tables): encode / decode time per launch,
and a byte-equality + round-trip check."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastvideocodec_amd import entropy_models as EM  # noqa: E402

dev = torch.device("cuda")
rng = np.random.default_rng(5)
n = 68 * 120
lt = EM.LaplaceTables()
coder = EM.RangeCoder(lt.cdf, lt.cdf_length, lt.offset, dev)
S = 96
idx = rng.integers(0, lt.cdf.shape[0], size=(S, n)).astype(np.int32)
sig = lt.scale_table[idx]
sym = np.round(rng.laplace(0, sig)).astype(np.int32)
sym_d = torch.from_numpy(sym).to(dev)
idx_d = torch.from_numpy(idx).to(dev)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enc = coder.encode(sym_d, idx_d)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    out = coder.decode(enc, idx_d, check=False)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
ok = torch.equal(out, sym_d)
nbytes = int(enc.pack_off[-1].item()) * 4
print(f"feature-like {S}x{n}: encode {1e3 * (t1 - t0):.2f} ms  decode {1e3 * (t2 - t1):.2f} ms  "
      f"bytes {nbytes}  roundtrip {ok}", flush=True)
