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
