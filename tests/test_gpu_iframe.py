"""GPU I-frame codec (replacing BPG, models.py:412-429) against its numpy restatement
(oracle/iframe_ref.py), and the on-disk container (GOP/view muxing, random access, table CRC)."""
import io

import numpy as np
import pytest
import torch

from fastvideocodec_amd import container as CT
from fastvideocodec_amd import iframe as IF
from fastvideocodec_amd import kernels as K
from fastvideocodec_amd.entropy_models import LaplaceTables
from fastvideocodec_amd.models import get_codec_model, parallel_compression
from fastvideocodec_amd.synthetic import make_gop
from oracle import coder_ref as R
from oracle import iframe_ref as IR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(dev):
    return get_codec_model("DVC-pretrained", compression_level=2, device=dev)


def _coeffs(dev, x, q):
    B, _, h, w = x.shape
    c = torch.empty((B, 3, h, w), dtype=torch.int32, device=dev)
    from fastvideocodec_amd import _lib
    _lib.call("fvc_iframe_rct_fwd", x.data_ptr(), c.data_ptr(), B, h, w, K.stream_handle())
    IF._dwt(c, IF.LEVELS, False)
    _lib.call("fvc_iframe_quant", c.data_ptr(), 3 * B, h, w, IF.LEVELS, q, 0, K.stream_handle())
    return c


@pytest.mark.parametrize("q", [1, 3, 11])
@pytest.mark.parametrize("size", [(64, 64), (128, 192), (1088, 1920)])
def test_iframe_matches_oracle(dev, q, size):
    """Coefficients, block indexes, every coefficient stream (vs the C oracle coder) and the
    reconstruction equal the numpy restatement; q = 1 is lossless."""
    h, w = size
    x = make_gop(h, w, 1, 31)[0]
    xd = torch.from_numpy(x[None].copy()).to(dev)
    bs, rec = IF.encode(xd, q)
    c = _coeffs(dev, xd, q).cpu().numpy()[0]
    c_ref = IR.encode_coeffs(x, IF.LEVELS, q)
    assert (c == c_ref).all()
    lt = LaplaceTables()
    bidx = IR.block_index(c_ref, lt.scale_table, IF.BLOCK)
    assert (bs.block_index == bidx).all()
    strings = bs.streams.to_bytes_list()
    idx = np.repeat(np.repeat(bidx.astype(np.int32), IF.BLOCK, 1), IF.BLOCK, 2)
    S = 3 * h // IF.BAND_ROWS
    cs, ids = c_ref.reshape(S, -1), idx.reshape(S, -1)
    check = range(S) if h <= 128 else range(0, S, 37)
    for s in check:
        assert strings[s] == R.CRef.encode(cs[s], ids[s], lt.cdf, lt.cdf_length, lt.offset), s
    rec_np = rec.cpu().numpy()[0]
    assert (rec_np == IR.decode_coeffs(c_ref, IF.LEVELS, q)).all()
    if q == 1:
        assert (rec_np == x).all()  # k/255 frames come back exactly
    dec = IF.decode(bs)
    assert torch.equal(dec, rec)


def test_iframe_step_and_parallel_compression(model, dev):
    assert IF.iframe_step(27) == 11 and IF.iframe_step(7) == 1 and IF.iframe_step(None) == 1
    gop = torch.from_numpy(make_gop(128, 192, 4, 5)).to(dev)
    model.iframe_codec = "dwt53"
    try:
        out = parallel_compression(None, model, gop.clone(), True)
    finally:
        model.iframe_codec = None
    psnr, psnr_list = out[5], out[6]
    assert np.isfinite(psnr) and len(psnr_list) == 4 and all(np.isfinite(psnr_list))


def test_container_roundtrip_gop_view_muxing(model, dev):
    """Two GOPs as two views: write, read back by random access, decode bit-exactly to the
    encoder's reconstructions; a model with different tables is refused."""
    video = torch.from_numpy(np.stack([make_gop(64, 128, 4, 60 + g) for g in range(2)])).to(dev)
    buf = io.BytesIO()
    rec = CT.encode_video(model, video, buf, views=[0, 1])
    data = buf.getvalue()
    r = CT.ContainerReader(data)
    assert r.header["gop"] == 4 and r.header["height"] == 64 and r.gops() == [(0, 0), (1, 1)]
    assert [e[0] for e in r.gop_records(1, 1)] == [b"I", b"P", b"P", b"P"]
    dec = CT.decode_video(model, data)
    torch.cuda.synchronize()
    for n in range(2):
        assert torch.equal(dec[(n, n)], rec[n])
    # the P-frame records carry exactly the model's own bitstreams
    bs, _ = model.compress(video[0, 1:2], rec[0, 0:1])
    assert r.record(r.gop_records(0, 0)[1]) == CT.pframe_payload(bs)
    other = get_codec_model("DVC-pretrained", compression_level=2, device=dev, seed=7)
    with pytest.raises(ValueError):
        CT.decode_video(other, data)


@pytest.mark.parametrize("framing", ["segment", "channel", "item"])
def test_container_roundtrip_each_framing(model, dev, framing):
    """Every P-frame stream framing through the container (framing code 0 channel, 1 item,
    2 segment) at 512x512, where the 1024-symbol mv / feature rows really are cut in two
    segments: the decoder reproduces the encoder's reconstructions bit for bit and the record
    holds the framing's stream count."""
    from fastvideocodec_amd.net import FRAMINGS, stream_rows
    video = torch.from_numpy(np.stack([make_gop(512, 512, 3, 90)])).to(dev)
    buf = io.BytesIO()
    rec = CT.encode_video(model, video, buf, framing=framing)
    data = buf.getvalue()
    dec = CT.decode_video(model, data)
    torch.cuda.synchronize()
    assert torch.equal(dec[(0, 0)], rec[0])
    r = CT.ContainerReader(data)
    payload = r.record(r.gop_records(0, 0)[1])
    assert payload[1] == FRAMINGS.index(framing)
    n_mv = int.from_bytes(payload[10:14], "little")  # streams(mv) count after the 10-byte head
    assert n_mv == stream_rows(framing, 1, 128, 32 * 32)[0]

