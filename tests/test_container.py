"""CPU: the container's byte layout (header, records, trailing index, random access)."""
import io

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
