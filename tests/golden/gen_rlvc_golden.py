"""Generate RLVC golden fixtures by running the REFERENCE's recurrent modules (build container only).

Run from the repo root:  python tests/golden/gen_rlvc_golden.py

Imports ``entropy_models.RPM`` and ``entropy_models.ConvLSTM`` (entropy_models.py:328-378, plain
torch modules) from /root/reference. The module's import-time dependencies on the absent
compressai / torchac packages are satisfied by empty stand-in modules (never called by these two
classes). Weights are the build's seeded RLVC state (fastvideocodec_amd.rlvc.seeded_state_dict),
inputs seeded random tensors. Output: tests/golden/rlvc_rpm.npz (inputs, weights used, outputs).
The reference never leaves this container; only the data file is committed.
"""
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "tests", "golden", "rlvc_rpm.npz")
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from fastvideocodec_amd.rlvc import seeded_state_dict  # noqa: E402


class _Stub(nn.Module):
    def __init__(self, *a, **k):
        super().__init__()


for name in ["compressai", "compressai.entropy_models", "compressai.models", "compressai.layers", "torchac"]:
    sys.modules[name] = types.ModuleType(name)
sys.modules["compressai.entropy_models"].EntropyModel = _Stub
sys.modules["compressai.entropy_models"].GaussianConditional = _Stub
sys.modules["compressai.entropy_models"].EntropyBottleneck = _Stub
sys.modules["compressai.models"].CompressionModel = _Stub
sys.modules["compressai.layers"].AttentionBlock = _Stub
sys.path.insert(0, "/root/reference")

import entropy_models as EMR  # noqa: E402

torch.set_num_threads(8)


def main():
    sd = seeded_state_dict()
    g = torch.Generator().manual_seed(7)
    C, H, W = 128, 4, 6
    out = {}
    lstm = EMR.ConvLSTM(C)
    pre = "mv_codec.enc_lstm."
    lstm.load_state_dict({k[len(pre):]: torch.from_numpy(v) for k, v in sd.items() if k.startswith(pre)})
    x = torch.randn(1, C, H, W, generator=g)
    state = 0.5 * torch.randn(1, 2 * C, H, W, generator=g)
    with torch.no_grad():
        h, st = lstm(x, state)
    out.update(lstm_x=x.numpy(), lstm_state=state.numpy(), lstm_h=h.numpy(), lstm_state_out=st.numpy())
    rpm = EMR.RPM(C)
    pre = "mv_codec.entropy_bottleneck.RPM."
    rpm.load_state_dict({k[len(pre):]: torch.from_numpy(v) for k, v in sd.items() if k.startswith(pre)})
    prior = torch.round(3 * torch.randn(2, C, H, W, generator=g))
    hid = 0.5 * torch.randn(2, 2 * C, H, W, generator=g)
    with torch.no_grad():
        sigma, mu, hid2 = rpm(prior, hid)
    out.update(rpm_prior=prior.numpy(), rpm_hidden=hid.numpy(), rpm_sigma=sigma.numpy(), rpm_mu=mu.numpy(),
               rpm_hidden_out=hid2.numpy())
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
