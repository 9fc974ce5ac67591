"""CPU: the container's byte layout (header, records, trailing index, random access)."""
import io
import os

import pytest

from fastvideocodec_amd import container as CT


def test_container_records_and_index():
    buf = io.BytesIO()
    w = CT.ContainerWriter(buf, {"codec": "DVC-pretrained", "gop": 3})
    payloads = {}
    for view in range(2):
        for t in range(3):
            p = bytes([view, t]) * (10 + t)
            payloads[(view, t)] = p
            w._record(b"I" if t == 0 else b"P", view, 5, t, p)
    w.close()
    data = buf.getvalue()
    r = CT.ContainerReader(data)
    assert r.header == {"codec": "DVC-pretrained", "gop": 3}
    assert r.gops() == [(0, 5), (1, 5)]
    recs = r.gop_records(1, 5)
    assert [e[0] for e in recs] == [b"I", b"P", b"P"]
    assert [r.record(e) for e in recs] == [payloads[(1, t)] for t in range(3)]
    with pytest.raises(ValueError):
        CT.ContainerReader(b"XXXX" + data[4:])
    with pytest.raises(ValueError):
        CT.ContainerReader(data[:-4] + b"NOPE")


def test_streams_packing():
    s = [b"", b"ab", b"x" * 9]
    buf = CT._pack_streams(s)
    out, pos = CT._unpack_streams(buf, 0)
    assert out == s and pos == len(buf)


FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "pframe_segment_256x1024")


def test_segment_framed_fixture_decodes_on_cpu(seeded_sd):
    """the committed segment-framed container (tests/golden/gen_container_fixture.py)
    stays readable. The P payload's stream counts fix the segment cut (net.bitstream_rows, not
    SEGMENT_MIN), the header's table CRC equals the product's host tables, and the C oracle coder
    decodes every stream back to the committed symbols."""
    import struct

    import numpy as np

    from fastvideocodec_amd import entropy_models as EM
    from fastvideocodec_amd.net import FRAMINGS, bitstream_rows
    from oracle import coder_ref as R

    g = np.load(FIXTURE + ".npz")
    with open(FIXTURE + ".fvc", "rb") as f:
        r = CT.ContainerReader(f.read())
    H, W = int(g["height"]), int(g["width"])
    assert r.header["framing"] == "segment" and (r.header["height"], r.header["width"]) == (H, W)
    rows = lambda name: np.stack([seeded_sd[f"{name}.f{i}.{p}"].numpy().reshape(-1) for i in (1, 2, 3) for p in "hba"]  # noqa: E731
                                 + [seeded_sd[f"{name}.f4.{p}"].numpy().reshape(-1) for p in "hb"])
    tz, tmv, tf = EM.FactorizedTables(rows("bitEstimator_z")), EM.FactorizedTables(rows("bitEstimator_mv")), EM.LaplaceTables()
    assert r.header["tables_crc32"] == CT.tables_crc_of(tz, tmv, tf)
    (entry,) = r.index
    payload = r.record(entry)
    prec, fr, H16, W16, H64, W64 = struct.unpack_from("<BBHHHH", payload, 0)
    assert FRAMINGS[fr] == "segment" and (H16, W16, H64, W64) == (H // 16, W // 16, H // 64, W // 64)
    pos = 10
    for name, C, hw, tab in (("mv", 128, H16 * W16, tmv), ("z", 64, H64 * W64, tz), ("feature", 96, H16 * W16, tf)):
        strings, pos = CT._unpack_streams(payload, pos)
        n, per = bitstream_rows("segment", 1, C, hw, len(strings))
        sym = g[f"sym_{name}"].astype(np.int32).reshape(n, per)
        if name == "feature":
            idx = g["idx_feature"].astype(np.int32).reshape(n, per)
        else:
            idx = np.repeat(np.arange(C, dtype=np.int32), hw).reshape(n, per)
        for i, s in enumerate(strings):
            assert (R.CRef.decode(s, idx[i], tab.cdf, tab.cdf_length, tab.offset) == sym[i]).all(), (name, i)
    assert pos == len(payload)
    assert g["streams_per_latent"].tolist() == [256, 64, 192]  # 2 segments per 1024-symbol mv / feature row


def test_bitstream_rows_rejects_bad_counts():
    from fastvideocodec_amd._lib import FvcError
    from fastvideocodec_amd.net import bitstream_rows
    assert bitstream_rows("segment", 2, 96, 8160, 2 * 96 * 8) == (1536, 1020)
    assert bitstream_rows("segment", 1, 64, 510, 64) == (64, 510)
    assert bitstream_rows("item", 3, 96, 100, 3) == (3, 9600)
    with pytest.raises(FvcError):
        bitstream_rows("segment", 1, 96, 8160, 96 * 7)   # 7 does not divide 8160
    with pytest.raises(FvcError):
        bitstream_rows("segment", 1, 96, 8160, 95)
    with pytest.raises(FvcError):
        bitstream_rows("channel", 1, 96, 8160, 97)
