"""Generate the committed segment-framed P-frame container fixture (CPU only).

Run from the repo root:  python tests/golden/gen_container_fixture.py

A decoder must keep reading files written earlier. This writes one FVC1 container holding one
P-frame record in the codec's default 'segment' framing, built without the GPU: the symbols come
from the oracle forward (oracle/dvc_ref.py) on a 1024x256 synthetic pair (H/16 x W/16 = 1024
symbols per channel row, so every mv / feature row is cut into 2 segments of 512), the tables
from the product's host table builders (equal to the oracle's, tests/test_coder_oracle.py), and
every stream from the C oracle coder (oracle/rans_ref.c, byte-equal to the device rANS).

Outputs tests/golden/pframe_segment_256x1024.fvc (the container) and
tests/golden/pframe_segment_256x1024.npz (the frame pair's seed, the coded symbols per latent and
the oracle's decoded reconstruction PSNR). tests/test_container.py reads both on CPU, and
tests/test_gpu_coder.py decodes the file on the GPU.
"""
import io
import os
import struct
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from fastvideocodec_amd import container as CT  # noqa: E402
from fastvideocodec_amd import entropy_models as EM  # noqa: E402
from fastvideocodec_amd.net import segments  # noqa: E402
from fastvideocodec_amd.synthetic import make_gop  # noqa: E402
from fastvideocodec_amd.weights import seeded_torch_state_dict  # noqa: E402
from oracle import coder_ref as R  # noqa: E402
from oracle import dvc_ref  # noqa: E402

H, W, SEED = 256, 1024, 20261015 + 11
OUT = os.path.join(REPO, "tests", "golden", f"pframe_segment_{H}x{W}")


def be_params(sd, name):
    rows = [sd[f"{name}.f{f}.{p}"].numpy().reshape(-1) for f in (1, 2, 3) for p in "hba"]
    rows += [sd[f"{name}.f4.h"].numpy().reshape(-1), sd[f"{name}.f4.b"].numpy().reshape(-1)]
    return np.stack(rows)


def encode_segments(sym, idx, tab):
    """[C, hw] symbols -> the segment framing's streams (channel-major, segments contiguous)."""
    C, hw = sym.shape
    s = segments(hw)
    sym, idx = sym.reshape(C * s, hw // s), idx.reshape(C * s, hw // s)
    return [R.CRef.encode(sym[i], idx[i], tab.cdf, tab.cdf_length, tab.offset) for i in range(C * s)]


def main():
    torch.set_num_threads(8)
    sd = seeded_torch_state_dict()
    g = make_gop(H, W, 2, SEED)
    cur, ref = torch.from_numpy(g[1:2].copy()), torch.from_numpy(g[0:1].copy())
    _, inter = dvc_ref.forward(sd, cur, ref, return_intermediates=True)
    tz, tmv = EM.FactorizedTables(be_params(sd, "bitEstimator_z")), EM.FactorizedTables(be_params(sd, "bitEstimator_mv"))
    tf = EM.LaplaceTables()
    sym = {k: inter[gk].numpy().reshape(c, -1).astype(np.int32) for k, gk, c in
           (("mv", "quant_mv", 128), ("z", "compressed_z", 64), ("feature", "compressed_feature", 96))}
    idx = {"mv": np.repeat(np.arange(128, dtype=np.int32)[:, None], sym["mv"].shape[1], 1),
           "z": np.repeat(np.arange(64, dtype=np.int32)[:, None], sym["z"].shape[1], 1),
           "feature": R.build_indexes(inter["recon_sigma"].numpy().reshape(96, -1), tf.scale_table)}
    streams = [encode_segments(sym[k], idx[k], t) for k, t in (("mv", tmv), ("z", tz), ("feature", tf))]
    head = struct.pack("<BBHHHH", 0, CT.FRAMINGS.index("segment"), H // 16, W // 16, H // 64, W // 64)
    payload = head + b"".join(CT._pack_streams(s) for s in streams)
    buf = io.BytesIO()
    w = CT.ContainerWriter(buf, {"codec": "DVC-pretrained", "level": 2, "height": H, "width": W, "gop": 2,
                                 "gops": 1, "tables_crc32": CT.tables_crc_of(tz, tmv, tf), "framing": "segment",
                                 "note": "fixture: one P record (frame 1), no I record; the reference frame is "
                                         f"make_gop({H}, {W}, 2, {SEED})[0]"})
    w.write_pframe(0, 0, 1, payload)
    w.close()
    with open(OUT + ".fvc", "wb") as f:
        f.write(buf.getvalue())
    clip, *_ = dvc_ref.decode(sd, ref, inter["quant_mv"], inter["compressed_z"], inter["compressed_feature"])
    mse = float(((clip.double() - cur.double()) ** 2).mean())
    np.savez_compressed(OUT + ".npz", seed=SEED, height=H, width=W,
                        sym_mv=sym["mv"].astype(np.int16), sym_z=sym["z"].astype(np.int16),
                        sym_feature=sym["feature"].astype(np.int16), idx_feature=idx["feature"].astype(np.int8),
                        streams_per_latent=np.array([len(s) for s in streams], np.int32),
                        oracle_decode_psnr_db=10 * np.log10(1.0 / mse))
    print(OUT + ".fvc", len(buf.getvalue()), "bytes;", [len(s) for s in streams], "streams")


if __name__ == "__main__":
    main()
