"""SURVEY.md §5 race detection: the four-stream GOP pipeline (gop.encode_decode_gop, overlap=True:
encoder, two coder streams and the reconstruction stream in flight together, cross-stream
tensors record_stream'ed) run in a child process with every launch serialised by the runtime
(AMD_SERIALIZE_KERNEL=3: wait before and after each kernel; HIP_LAUNCH_BLOCKING=1) must produce the
same bytes and reconstructions as the same pipeline running concurrently in this process. A
missing stream dependency would show up as a difference between the two (the serialised run
cannot race)."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r'''
import hashlib, json, sys
sys.path.insert(0, {repo!r})
import numpy as np, torch
from fastvideocodec_amd.gop import encode_decode_gop
from fastvideocodec_amd.models import get_codec_model
from fastvideocodec_amd.synthetic import make_gop
dev = torch.device("cuda:0")
model = get_codec_model("DVC-pretrained", compression_level=2, device=dev)
frames = torch.from_numpy(np.stack([make_gop(128, 192, 5, 900 + g) for g in range(3)])).to(dev)
bss, dec, _, enc = encode_decode_gop(model, frames, check=True, overlap=True)
torch.cuda.synchronize()
h = hashlib.sha256()
for bs in bss:
    for part in (bs.mv, bs.z, bs.feature):
        for s in part.to_bytes_list():
            h.update(s)
for d, e in zip(dec, enc):
    h.update(d.cpu().numpy().tobytes()); h.update(e.cpu().numpy().tobytes())
print(json.dumps({{"digest": h.hexdigest()}}))
'''


def _digest(out):
    for line in out.splitlines()[::-1]:
        if line.startswith("{"):
            return json.loads(line)["digest"]
    raise AssertionError(out[-2000:])


@pytest.mark.timeout(300)
def test_pipeline_equals_serialised_launches(dev):
    code = _CHILD.format(repo=REPO)
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3", HIP_LAUNCH_BLOCKING="1")
    ser = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert ser.returncode == 0, ser.stderr[-3000:]
    conc = subprocess.run([sys.executable, "-c", code], env=dict(os.environ), capture_output=True, text=True,
                          timeout=240)
    assert conc.returncode == 0, conc.stderr[-3000:]
    assert _digest(ser.stdout) == _digest(conc.stdout)


# Production conv families at 4K as antagonists of the warp gathers (profiles/r6/race/README.md: on
# gfx950 a kernel issuing dense MFMA chains beside a gather kernel can make lanes 48-63 of gathered
# loads return zeros; the 7x7 stem experiment does, none of these may)
_ANTAGONISTS = [
    # (cin, cout, k, stride, transposed, level shift, in_op, act)
    (8, 32, 7, 1, False, 0, "IN_NONE", "ACT_RELU"),      # SpyNet conv1 (direct x3)
    (32, 64, 7, 1, False, 0, "IN_NONE", "ACT_RELU"),     # SpyNet conv2 (wr7)
    (64, 64, 3, 1, False, 0, "IN_RELU", "ACT_RELU"),     # Warp_net ResBlock (Winograd)
    (128, 128, 3, 2, True, 1, "IN_NONE", "ACT_LRELU"),   # mvDecoder deconv (dx)
    (128, 128, 3, 2, False, 1, "IN_NONE", "ACT_LRELU"),  # mvEncoder conv (x3, stride 2)
    (6, 64, 3, 1, False, 0, "IN_NONE", "ACT_RELU"),      # Warp_net feature_ext (stem)
    (16, 2, 7, 1, False, 0, "IN_NONE", "ACT_NONE"),      # SpyNet conv5 (fp32 kernel)
]


@pytest.mark.timeout(300)
def test_production_convs_leave_warp_gathers_exact(dev):
    """Each production conv family runs back to back on one stream while the motion-compensation
    warp (fvc_mc_assemble, data-dependent 4-tap gathers) runs on another at 4K: every warp output
    equals the one made with the conv stream idle (on-device compare, no host sync per launch)."""
    from fastvideocodec_amd import kernels as K
    H, W = 2176, 3840
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
    bad = {}
    for cin, cout, k, s, tr, sh, iop, act in _ANTAGONISTS:
        wt = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), generator=g) * (1.0 / (cin * k * k) ** 0.5)
        p = K.PackedConv(wt, torch.zeros(cout), k, s, tr, dev, precision="x3")
        x = torch.rand(1, H >> sh, W >> sh, K.cp4(cin), device=dev)
        x[..., cin:] = 0
        n = torch.zeros((), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        for _ in range(16):
            with torch.cuda.stream(sa):
                for _ in range(2):
                    p(x, in_op=getattr(K, iop), act=getattr(K, act))
            with torch.cuda.stream(sb):
                for _ in range(4):
                    wf, _ = K.mc_assemble(ref, mv)
                    n += (wf != gold).any(-1).sum()
        torch.cuda.synchronize()
        bad[f"{cin}->{cout} k{k} s{s}{' T' if tr else ''}"] = int(n)
    assert all(v == 0 for v in bad.values()), bad
