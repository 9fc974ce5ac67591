"""Coder parity on the GPU: the device rANS against the oracle coders (C restatement and the
pure-Python one, oracle/coder_ref.py) on real latents, in both stream framings, plus the
compressai-framed API (entropy_models.py:26-94 surface) and the split-precision overflow
handling of the product path."""
import numpy as np
import pytest
import torch

from fastvideocodec_amd import entropy_models as EM
from fastvideocodec_amd import kernels as K
from fastvideocodec_amd.models import get_codec_model
from oracle import coder_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(dev):
    return get_codec_model("DVC-pretrained", compression_level=2, device=dev)


def _frame(dev, h, w, seed=7):
    from fastvideocodec_amd.synthetic import make_gop, gop_seed
    f = torch.from_numpy(make_gop(h, w, 2, gop_seed(seed))).to(dev)
    return f[1:2], f[0:1]


def _latent_symbols(model, t):
    """Symbols and table indexes of the three latents as numpy [C, HW] (B = 1), from the
    encoder's own tensors through the product's symbol / index kernels."""
    c = model._coders
    out = {}
    for name, key, C in (("mv", "mvfeature", 128), ("z", "z", 64), ("feature", "feature", 96)):
        sym = K.latent_to_symbols(t[key], C).cpu().numpy().reshape(C, -1)
        if name == "feature":
            idx = K.build_indexes(t["sigma"], c["scale_table"], C).cpu().numpy().reshape(C, -1)
        else:
            idx = np.repeat(np.arange(C, dtype=np.int32)[:, None], sym.shape[1], 1)
        out[name] = (sym, idx)
    return out


def _tables(model):
    tz, tmv, tf = model._coders["tables"]
    return {"z": tz, "mv": tmv, "feature": tf}


@pytest.mark.parametrize("framing", ["segment", "channel"])
def test_compress_1080p_every_stream_vs_oracle(model, dev, framing):
    """BASELINE configs[2]: one 1920x1080 P-frame compressed by the product path; each of its
    streams equals the C oracle coder's bytes on the same symbols / indexes / tables, the z
    streams also equal the pure-Python coder's, and the device decoder returns the encoder's
    symbols. 'channel': 288 streams (128 mv + 64 z + 96 feature rows of 8160 / 510 symbols);
    'segment' (the codec's default): every 8160-symbol mv / feature row cut into 8 streams of
    1020 symbols (1024 + 64 + 768 streams), z rows (510 symbols) left whole."""
    from fastvideocodec_amd.net import stream_rows
    cur, ref = _frame(dev, 1080, 1920)
    with torch.no_grad():
        t = model._encode_graph(cur, ref)
    bs = model.compress_tensors(t, framing=framing)
    assert bs.framing == framing
    lat = _latent_symbols(model, t)
    tabs = _tables(model)
    nbytes = 0
    expect = {"segment": {"mv": 1024, "z": 64, "feature": 768}, "channel": {"mv": 128, "z": 64, "feature": 96}}
    for name in ("mv", "z", "feature"):
        sym, idx = lat[name]
        C, hw = sym.shape
        shape = stream_rows(framing, 1, C, hw)
        assert shape[0] == expect[framing][name], shape
        sym, idx = sym.reshape(shape), idx.reshape(shape)
        tb = tabs[name]
        strings = getattr(bs, name).to_bytes_list()
        assert len(strings) == sym.shape[0]
        for c in range(sym.shape[0]):
            assert strings[c] == R.CRef.encode(sym[c], idx[c], tb.cdf, tb.cdf_length, tb.offset), (name, c)
            nbytes += len(strings[c])
        if name == "z":
            for c in range(sym.shape[0]):
                assert strings[c] == R.rans_encode_py(sym[c], idx[c], tb.cdf, tb.cdf_length, tb.offset), c
    assert nbytes == bs.nbytes()
    dl = model.decode_latents(bs)
    for name, key, C in (("mv", "mv", 128), ("z", "z", 64), ("feature", "feature", 96)):
        got = K.latent_to_symbols(dl[key], C).cpu().numpy().reshape(C, -1)
        assert (got == lat[name][0]).all(), name


@pytest.mark.parametrize("size", [(64, 64), (1080, 1920)], ids=["64x64", "1080p"])
def test_compress_item_framing_vs_oracle(model, dev, size):
    """compressai's framing (EntropyModel.compress: one string per batch item over (C,H,W) in C
    order): each latent's single stream equals the C oracle (and, at 64x64, the pure-Python
    coder) on the whole sequence, and decodes to the encoder's reconstruction bit-for-bit."""
    cur, ref = _frame(dev, *size)
    with torch.no_grad():
        t = model._encode_graph(cur, ref)
    bs = model.compress_tensors(t, framing="item")
    assert bs.framing == "item"
    lat = _latent_symbols(model, t)
    tabs = _tables(model)
    for name in ("mv", "z", "feature"):
        sym, idx = lat[name]
        tb = tabs[name]
        strings = getattr(bs, name).to_bytes_list()
        assert len(strings) == 1
        assert strings[0] == R.CRef.encode(sym.ravel(), idx.ravel(), tb.cdf, tb.cdf_length, tb.offset), name
        if size == (64, 64):
            assert strings[0] == R.rans_encode_py(sym.ravel(), idx.ravel(), tb.cdf, tb.cdf_length, tb.offset)
    bs2, rec_enc = model.compress(cur, ref, framing="item")
    rec_dec = model.decompress(bs2, ref)
    torch.cuda.synchronize()
    assert torch.equal(rec_enc, rec_dec)


def test_compressai_api_classes(model, dev):
    """EntropyBottleneck / ConditionalEntropyModel / RecProbModel (compressai surface) on a batch
    of 2: one string per item equal to the pure-Python coder over the item's (C,H,W) sequence,
    decompress == quantize (+ means), get_actual_bits == 8 x bytes."""
    g = torch.Generator().manual_seed(3)
    bz, bmv = model._be_params()
    eb = EM.EntropyBottleneck(bmv, dev)
    assert eb.update() and not eb.update()
    x = (torch.randn(2, 128, 4, 6, generator=g) * 3).to(dev)
    strings = eb.compress(x)
    assert len(strings) == 2
    tmv = _tables(model)["mv"]
    xr = torch.round(x).to(torch.int32).cpu().numpy()
    idx = np.repeat(np.arange(128, dtype=np.int32)[:, None], 24, 1).ravel()
    for i in range(2):
        assert strings[i] == R.rans_encode_py(xr[i].ravel(), idx, tmv.cdf, tmv.cdf_length, tmv.offset)
    y = eb.decompress(strings, (4, 6))
    assert torch.equal(y.cpu(), torch.round(x).cpu())
    for dist in ("laplace", "gaussian"):
        gc = EM.ConditionalEntropyModel(None, dist, dev)
        gc.update_scale_table(EM.get_scale_table())
        scales = (torch.rand(2, 8, 5, 7, generator=g) * 20 + 0.05).to(dev)
        means = (torch.randn(2, 8, 5, 7, generator=g)).to(dev)
        xv = (torch.randn(2, 8, 5, 7, generator=g) * 10).to(dev)
        ind = gc.build_indexes(scales)
        assert (ind.cpu().numpy() == R.build_indexes(scales.cpu().numpy(), gc.scale_table.numpy())).all()
        st = gc.compress(xv, ind, means=means)
        cdf = gc._quantized_cdf.cpu().numpy()
        ln = gc._cdf_length.cpu().numpy()
        off = gc._offset.cpu().numpy()
        symr = torch.round(xv - means).to(torch.int32).cpu().numpy()
        for i in range(2):
            assert st[i] == R.rans_encode_py(symr[i].ravel(), ind[i].cpu().numpy().ravel(), cdf, ln, off), dist
        back = gc.decompress(st, ind, means=means)
        assert torch.equal(back.cpu(), (torch.round(xv - means) + means).cpu())
    rpm = EM.RecProbModel(128, bmv, dist="gaussian", device=dev)
    rpm.update(force=True)
    s1 = rpm.compress(x)
    assert s1 == strings
    assert float(rpm.get_actual_bits(s1)) == 8 * sum(len(s) for s in s1)
    rpm.set_RPM(True)
    rpm.sigma = (torch.rand(2, 128, 4, 6, generator=g) * 5 + 0.2).to(dev)
    rpm.mu = torch.zeros(2, 128, 4, 6, device=dev)
    s2 = rpm.compress(x)
    assert torch.equal(rpm.decompress(s2, (4, 6)).cpu(), torch.round(x).cpu())


def test_rans_encoder_empty_stream_flushes_state(dev):
    """compressai flushes the initial state even for zero symbols: 8 bytes."""
    lap = EM.LaplaceTables()
    cdfs = [row[: n].tolist() for row, n in zip(lap.cdf, lap.cdf_length)]
    s = EM.RansEncoder(dev).encode_with_indexes([], [], cdfs, lap.cdf_length.tolist(), lap.offset.tolist())
    assert s == R.rans_encode_py([], [], lap.cdf, lap.cdf_length, lap.offset)
    assert len(s) == 8


def test_rans_decode_damaged_streams(dev):
    """Damaged input to the device decoder (compressai's RansDecoder has no error detection; this
    decoder bounds every read by the stream's own word count and reports ECORRUPT per stream):
    * a stream cut short by its last word fails with FvcError (the renorm that needs the word
      finds the stream exhausted), and so does an empty (0-word) stream;
    * words flipped inside one stream change only that stream's symbols: every other stream of
      the launch still decodes to its exact symbols, whatever the damaged one yields;
    * the launch completes either way (no fault, no hang: the decoder's reads never leave the
      packed buffer)."""
    from fastvideocodec_amd._lib import FvcError
    lap = EM.LaplaceTables()
    rc = EM.RangeCoder(lap.cdf, lap.cdf_length, lap.offset, dev)
    g = np.random.default_rng(5)
    S, n = 96, 1020
    idx = g.integers(0, lap.cdf.shape[0], (S, n)).astype(np.int32)
    sym = np.rint(g.laplace(0, 3, (S, n))).astype(np.int32)
    idx_d, sym_d = torch.from_numpy(idx).to(dev), torch.from_numpy(sym).to(dev)
    strings = rc.encode(sym_d, idx_d).to_bytes_list()
    assert torch.equal(rc.decode(EM.EncodedStreams.from_bytes_list(strings, dev), idx_d).cpu(), sym_d.cpu())
    for cut in (4, len(strings[17])):  # one word short; the whole stream gone
        bad = list(strings)
        bad[17] = strings[17][: len(strings[17]) - cut]
        with pytest.raises(FvcError):
            rc.decode(EM.EncodedStreams.from_bytes_list(bad, dev), idx_d)
        torch.cuda.synchronize()
    for victim in (0, 40, S - 1):
        bad = list(strings)
        w = bytearray(strings[victim])
        for k in range(8, len(w) - 4, 97):
            w[k] ^= 0xA5
        bad[victim] = bytes(w)
        out = rc.decode(EM.EncodedStreams.from_bytes_list(bad, dev), idx_d, check=False).cpu()
        torch.cuda.synchronize()
        keep = [i for i in range(S) if i != victim]
        assert torch.equal(out[keep], sym_d.cpu()[keep]), victim
        assert not torch.equal(out[victim], sym_d.cpu()[victim]), victim


def _overflowing_model(dev, policy):
    """Seeded weights with Warp_net's last ResBlock's first conv scaled by 1e7: its output (the
    next conv's input) leaves the split-precision range (|v| >= 65000)."""
    m = get_codec_model("DVC-pretrained", compression_level=2, device=dev)
    with torch.no_grad():
        m.warpnet.conv5.conv1.weight.mul_(1e7)
        m.warpnet.conv5.conv1.bias.mul_(1e7)
    m.invalidate()
    m.on_overflow = policy
    return m


def test_overflow_recompute_forward_and_compress(dev):
    """An activation >= 65000 through forward() and compress(): the frame is recomputed on the
    fp32 kernels (bit-identical to running the model in fp32), the bitstream records it, and
    the decoder reproduces the encoder's recon; with on_overflow='raise' FvcError is raised."""
    from fastvideocodec_amd._lib import FvcError
    cur, ref = _frame(dev, 128, 192)
    m = _overflowing_model(dev, "recompute")
    out = m(cur, ref)
    assert m.last_precision == "f32"
    with K.precision("f32"):
        exp = m(cur, ref)
    for a, b in zip(out, exp):
        assert torch.equal(a, b)
    bs, rec = m.compress(cur, ref)
    assert bs.precision == "f32" and m.last_precision == "f32"
    assert torch.equal(rec, out[0])
    assert torch.equal(m.decompress(bs, ref), rec)
    m.on_overflow = "raise"
    with pytest.raises(FvcError):
        m(cur, ref)
    with pytest.raises(FvcError):
        m.compress(cur, ref)
    # an unmodified model stays on the split-precision path
    ok = get_codec_model("DVC-pretrained", compression_level=2, device=dev)
    ok(cur, ref)
    assert ok.last_precision == "x3"


def test_overflow_recompute_gop(dev):
    """The GOP pipeline resolves its per-frame probes at join: the GOP is re-coded in fp32 and
    still decodes bit-exactly."""
    from fastvideocodec_amd.gop import encode_decode_gop
    from fastvideocodec_amd.synthetic import make_gop
    m = _overflowing_model(dev, "recompute")
    frames = torch.from_numpy(np.stack([make_gop(128, 192, 3, 11)])).to(dev)
    bss, dec, _, enc = encode_decode_gop(m, frames, check=True, overlap=True)
    torch.cuda.synchronize()
    assert all(b.precision == "f32" for b in bss)
    for a, b in zip(dec, enc):
        assert torch.equal(a, b)


def test_overflow_flag_is_stream_local(dev):
    """The overflow flag is per stream (the C-ABI keeps no global state): an overflow on a side
    stream does not show on the main stream."""
    w = torch.randn(64, 64, 3, 3) * 0.05
    pc = K.PackedConv(w, torch.zeros(64), 3, 1, False, dev, precision="x3")
    x = torch.zeros(1, 16, 32, 64, device=dev)
    x[0, 3, 7, 5] = 7.0e4
    K.x3_overflow(reset=True)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        K.x3_overflow(reset=True)
        pc(x)
        assert K.x3_overflow(reset=True)
    assert not K.x3_overflow(reset=True)


def test_segment_framed_container_fixture_decodes(model, dev):
    """the committed segment-framed container (written on CPU by the C oracle coder,
    tests/golden/gen_container_fixture.py) decodes on the device: the entropy decode gives the
    committed symbols exactly, and the reconstruction matches the oracle decoder's PSNR."""
    import os

    from fastvideocodec_amd import container as CT
    from fastvideocodec_amd.synthetic import make_gop

    base = os.path.join(os.path.dirname(__file__), "golden", "pframe_segment_256x1024")
    g = np.load(base + ".npz")
    with open(base + ".fvc", "rb") as f:
        r = CT.ContainerReader(f.read())
    assert r.header["tables_crc32"] == CT.tables_crc(model)
    bs = CT.pframe_from_payload(r.record(r.index[0]), dev)
    assert bs.framing == "segment" and (bs.mv.nstreams, bs.z.nstreams, bs.feature.nstreams) == (256, 64, 192)
    lat = model.decode_latents(bs)
    for name, key, C in (("mv", "mv", 128), ("z", "z", 64), ("feature", "feature", 96)):
        got = K.latent_to_symbols(lat[key], C).cpu().numpy().reshape(C, -1)
        assert (got == g[f"sym_{name}"].astype(np.int32)).all(), name
    H, W = int(g["height"]), int(g["width"])
    frames = make_gop(H, W, 2, int(g["seed"]))
    rec = model.decompress(bs, torch.from_numpy(frames[0:1].copy()).to(dev)).cpu().numpy().astype(np.float64)
    psnr = 10 * np.log10(1.0 / np.mean((rec - frames[1:2]) ** 2))
    assert abs(psnr - float(g["oracle_decode_psnr_db"])) <= 1e-4, (psnr, float(g["oracle_decode_psnr_db"]))
