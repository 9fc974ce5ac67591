"""CPU: the C-ABI library builds, loads, exports every symbol include/fvc.h declares, and its
host-side entry points (weight packing, CDF quantisation) behave. No device calls here."""
import os
import re

import numpy as np
import pytest
import torch

from fastvideocodec_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "fvc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fvc_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding():
    assert set(header_symbols()) == set(_lib.EXPORTED)


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.fvc_version() >= 1


def test_wpack_sizes_and_packing():
    lib = _lib.load()
    for cin, cout, k, s, tr in [(8, 32, 7, 1, 0), (128, 128, 3, 2, 1), (64, 3, 5, 2, 1), (64, 96, 3, 1, 1),
                                (96, 64, 3, 1, 0), (3, 64, 5, 2, 0)]:
        n = lib.fvc_conv_wpack_floats(cin, cout, k, s, tr)
        assert n > 0 and n % 128 == 0
        shape = (cin, cout, k, k) if tr else (cout, cin, k, k)
        w = torch.randn(shape)
        out = torch.empty(n)
        _lib.call("fvc_conv_pack_weight", w.data_ptr(), out.data_ptr(), cin, cout, k, s, tr)
        # every weight appears exactly once in the pack (the rest is zero padding)
        assert abs(float(out.abs().sum()) - float(w.abs().sum())) < 1e-3 * float(w.abs().sum())
        assert int((out != 0).sum()) == int((w != 0).sum())
    assert lib.fvc_conv_wpack_floats(8, 160, 3, 1, 0) == 0  # > 128 output channels unsupported
    assert lib.fvc_conv_wpack_floats(8, 16, 4, 1, 0) == 0   # even kernel unsupported


def test_pmf_to_quantized_cdf_abi():
    from fastvideocodec_amd import entropy_models as EM
    assert EM.pmf_to_quantized_cdf([0.25] * 4).tolist() == [0, 16384, 32768, 49152, 65536]
    with pytest.raises(_lib.FvcError):
        EM.pmf_to_quantized_cdf([0.0, 0.0])


def test_models_api_surface():
    from fastvideocodec_amd.models import get_codec_model
    m = get_codec_model("DVC-pretrained", compression_level=2, device=torch.device("cpu"))
    assert (m.name, m.compression_level, m.loss_type, m.I_level, m.r) == ("DVC-pretrained", 2, "P", 27, 1024)
    x = torch.rand(1, 3, 64, 64)
    with pytest.raises(ValueError):  # no CPU fallback: the product path is HIP-only
        m(x, x)
    with pytest.raises(NotImplementedError):
        get_codec_model("ELFVC")
    r = get_codec_model("RLVC", compression_level=2, device="cpu")  # models.py:33 IterPredVideoCodecs
    assert (r.name, r.compression_level, r.loss_type) == ("RLVC", 2, "P")


def test_state_dict_matches_reference_layout():
    from fastvideocodec_amd.net import VideoCompressor
    from fastvideocodec_amd.weights import seeded_state_dict
    m = VideoCompressor()
    sd = seeded_state_dict()
    own = m.state_dict()
    assert list(own.keys()) == list(sd.keys())
    for k, v in sd.items():
        assert tuple(own[k].shape) == v.shape, k


@pytest.mark.parametrize("geom", [(8, 32, 7, 1, 0), (32, 64, 7, 1, 0), (64, 64, 3, 1, 0), (128, 128, 3, 2, 1),
                                  (128, 128, 3, 2, 0), (96, 64, 5, 2, 1), (64, 96, 3, 1, 1), (6, 64, 3, 1, 0)])
def test_x3_pack_splits_every_weight_once(geom):
    """Split-precision pack (fvc_conv_x3.hip): every weight appears exactly once as a hi/lo fp16
    pair with hi + lo*2^-11 == w*2^kw to ~2^-22 relative, and max|w|*2^kw lies in [2^13, 2^14)."""
    import ctypes
    lib = _lib.load()
    cin, cout, k, s, tr = geom
    assert lib.fvc_conv_x3_supported(*geom) == 1
    nbytes = lib.fvc_conv_x3_wpack_bytes(*geom)
    assert nbytes > 0 and nbytes % 2048 == 0
    g = torch.Generator().manual_seed(sum(geom))
    w = torch.randn((cin, cout, k, k) if tr else (cout, cin, k, k), generator=g) * 0.03
    out = torch.empty(nbytes // 2, dtype=torch.float16)
    osc = ctypes.c_float(0)
    assert lib.fvc_conv_x3_pack_weight(w.data_ptr(), out.data_ptr(), ctypes.addressof(osc), cin, cout, k, s, tr) == 0
    frags = out.view(-1, 2, 64, 8).double()  # [k-step x N-tile][hi | lo * 2^11][lane][8]
    val = (frags[:, 0] + frags[:, 1] * 2.0 ** -11).flatten()
    hi = frags[:, 0].flatten()
    nz = hi != 0
    assert int(nz.sum()) == w.numel()
    rec = torch.sort(val[nz] * osc.value).values
    ref = torch.sort(w.flatten().double()).values
    # ~22 significant bits; weights below ~2^-17 of the layer max keep an absolute error ~2^-37 of it
    assert torch.allclose(rec, ref, rtol=2 ** -20, atol=float(w.abs().max()) * 2 ** -32)
    scaled = float(w.abs().max()) / osc.value
    assert 2 ** 13 <= scaled < 2 ** 14


@pytest.mark.parametrize("np_cin", [(18, 128), (27, 64), (32, 32), (5, 60)])
def test_x3_tap_pack_layout(np_cin):
    """Fused tap epilogue weights (fvc_x3_tap_pack_weight): block kb, lane (li, lh), element t
    holds row li and channel 16 kb + 4 lh + {0,1,2,3,8,9,10,11}[t] -- the producing tile's
    accumulator order -- as a hi / lo*2^11 fp16 pair of w*2^kt; rows >= np and channels >= cin
    are zero. Also the C-ABI support predicate for the two fused pairs and the refusals."""
    import ctypes
    lib = _lib.load()
    npart, cin = np_cin
    nbytes = lib.fvc_x3_tap_wpack_bytes(npart, cin)
    nkb = 2 * -(-((cin + 3) // 4 * 4) // 32)  # two k16 blocks per 32-channel N-tile of the producer
    assert nbytes == nkb * 2 * 64 * 16
    g = torch.Generator().manual_seed(npart * cin)
    w = torch.randn(npart, cin, generator=g) * 0.05
    out = torch.empty(nbytes // 2, dtype=torch.float16)
    osc = ctypes.c_float(0)
    assert lib.fvc_x3_tap_pack_weight(w.data_ptr(), out.data_ptr(), ctypes.addressof(osc), npart, cin) == 0
    fr = out.view(nkb, 2, 64, 8).double()
    val = (fr[:, 0] + fr[:, 1] * 2.0 ** -11) * osc.value          # [kb][lane][t]
    perm = [0, 1, 2, 3, 8, 9, 10, 11]
    expect = torch.zeros(nkb, 64, 8, dtype=torch.float64)
    for kb in range(nkb):
        for lane in range(64):
            li, lh = lane & 31, lane >> 5
            for t in range(8):
                ci = 16 * kb + 4 * lh + perm[t]
                if li < npart and ci < cin:
                    expect[kb, lane, t] = float(w[li, ci])
    assert torch.allclose(val, expect, rtol=2 ** -20, atol=float(w.abs().max()) * 2 ** -32)
    assert lib.fvc_x3_tap_wpack_bytes(33, cin) == 0  # more partials than one P tile
    assert lib.fvc_conv_x3_tap_supported(128, 128, 3, 2, 1, 20) == 1  # mvDecoder deconv7 -> deconv8
    assert lib.fvc_conv_x3_tap_supported(64, 64, 3, 1, 0, 28) == 1    # Warp_net conv5 -> conv6
    assert lib.fvc_conv_x3_tap_supported(64, 64, 3, 1, 0, 30) == 0    # P channels must be a multiple of 4
    assert lib.fvc_conv_x3_pool_supported(64, 64, 3) == 1
    assert lib.fvc_conv_x3_pool_supported(128, 128, 3) == 0           # two N-groups: pool needs one wave per pixel


def test_x3_rejects_unsupported_layers():
    lib = _lib.load()
    assert lib.fvc_conv_x3_supported(2, 128, 3, 2, 0) == 1  # cin padded to 4: one zero-extended octet
    assert lib.fvc_conv_x3_supported(3, 64, 5, 2, 0) == 1   # resEncoder conv1
    assert lib.fvc_conv_x3_supported(16, 2, 7, 1, 0) == 0   # 7x7 cout <= 4: VALU small-N kernel
    assert lib.fvc_conv_x3_wpack_bytes(16, 2, 7, 1, 0) == 0
    assert lib.fvc_conv_x3_supported(64, 3, 3, 1, 0) == 1   # 3x3 cout <= 4: N padded to one MFMA tile


def test_checkpoint_loading_semantics(tmp_path, seeded_sd):
    """DVC/net.py:21-34 load_model: unknown keys are dropped, a missing file raises; seeded
    weights are flagged."""
    import warnings
    from fastvideocodec_amd.models import SeededWeightsWarning, get_DVC_pretrained
    with pytest.raises(FileNotFoundError):
        get_DVC_pretrained(2, checkpoint=str(tmp_path / "nope.model"), device=torch.device("cpu"))
    sd = dict(seeded_sd)
    sd["imageCompressor.extra"] = torch.zeros(3)
    sd["mvEncoder.conv1.bias"] = torch.full_like(sd["mvEncoder.conv1.bias"], 0.5)
    path = tmp_path / "1024.model"
    torch.save(sd, path)
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        m = get_DVC_pretrained(2, checkpoint=str(path), device=torch.device("cpu"))
    assert m.dropped_checkpoint_keys == ["imageCompressor.extra"] and m.weights_source == str(path)
    assert float(m.mvEncoder.conv1.bias[0]) == 0.5
    with pytest.warns(SeededWeightsWarning):
        m2 = get_DVC_pretrained(2, device=torch.device("cpu"))
    assert m2.weights_source == "seeded"


def test_bench_bookkeeping():
    import bench
    e, d = bench.tflop_per_pframe(1088, 1920)
    assert abs(e + d - 4.226) < 1e-9
    e4, d4 = bench.tflop_per_pframe(2176, 3840)
    assert abs((e4 + d4) / (e + d) - 4.0) < 1e-12
    assert bench.metric_name(1080, 1920) == "1080p frames/sec encode+decode at λ=1024; bpp/PSNR parity vs CPU ref"
    assert bench.metric_name(2160, 3840).startswith("3840x2160 ")
    assert 1 <= bench.cpu_cores() <= len(os.sched_getaffinity(0))


def test_x3_dispatch_count_mirrors_the_batch_split(monkeypatch):
    """The timer's dispatch count follows run_x3's recursive halving at 4 GB of output / residual
    (so bench avg_launch_us is per kernel dispatch, as rocprofv3 counts)."""
    from fastvideocodec_amd.kernels import x3_dispatches
    monkeypatch.delenv("FVC_X3_SPLIT_BYTES", raising=False)
    full64 = 1088 * 1920 * 64 * 4
    assert x3_dispatches(8, full64) == 1          # 4.28 GB < 4 GB - 4 KB: one launch
    assert x3_dispatches(16, full64) == 2
    assert x3_dispatches(3, 2176 * 3840 * 64 * 4) == 2
    assert x3_dispatches(1, 1 << 40) == 1         # one image never splits (the C side refuses it)
    assert x3_dispatches(4, 100, res_image_bytes=1 << 31) == 4
    monkeypatch.setenv("FVC_X3_SPLIT_BYTES", "1000")
    assert x3_dispatches(5, 300) == 2             # 1500 B -> 2 + 3 images (600, 900 B): two launches
    assert x3_dispatches(8, 300) == 4             # 2400 -> 4 + 4 (1200 each) -> 2 + 2 + 2 + 2


def test_x3_layout_id_tracks_layout_switches(monkeypatch):
    """the env switches that change an x3 pack's layout change its layout id (which
    PackedConv records at pack time and compares before every launch); other knobs do not."""
    lib = _lib.load()
    for k in ("FVC_DX", "FVC_X3_PT", "FVC_X3_CC", "FVC_X3_CIN4", "FVC_X3_SMALLN", "FVC_X3_WM"):
        monkeypatch.delenv(k, raising=False)
    dx = lib.fvc_conv_x3_layout_id(128, 128, 3, 2, 1)
    pt = lib.fvc_conv_x3_layout_id(32, 16, 7, 1, 0)
    c4 = lib.fvc_conv_x3_layout_id(3, 64, 5, 2, 0)
    wide = lib.fvc_conv_x3_layout_id(64, 64, 3, 1, 0)
    assert 0 not in (dx, pt, c4, wide)
    assert lib.fvc_conv_x3_layout_id(8, 160, 3, 1, 0) == 0  # not an x3 geometry
    monkeypatch.setenv("FVC_X3_WM", "1")  # block shape only: same pack
    assert lib.fvc_conv_x3_layout_id(64, 64, 3, 1, 0) == wide
    monkeypatch.setenv("FVC_DX", "0")
    assert lib.fvc_conv_x3_layout_id(128, 128, 3, 2, 1) not in (0, dx)
    monkeypatch.setenv("FVC_X3_PT", "0")
    assert lib.fvc_conv_x3_layout_id(32, 16, 7, 1, 0) not in (0, pt)
    monkeypatch.setenv("FVC_X3_CC", "8")
    assert lib.fvc_conv_x3_layout_id(64, 64, 3, 1, 0) not in (0, wide)
    monkeypatch.setenv("FVC_X3_CIN4", "0")
    assert lib.fvc_conv_x3_layout_id(3, 64, 5, 2, 0) == 0  # back on the fp32 kernels


def test_layout_check_refuses_on_every_call(monkeypatch):
    """PackedConv._check_layout caches the env snapshot it last accepted; a snapshot it
    refused must be refused again on the next call, not remembered as checked."""
    from fastvideocodec_amd import kernels as K
    for k in K._LAYOUT_ENV:
        monkeypatch.delenv(k, raising=False)
    pc = object.__new__(K.PackedConv)  # host-side state only: no device pack needed for the check
    pc.cin, pc.cout, pc.ksize, pc.stride, pc.transposed = 128, 128, 3, 2, True
    pc.layout = int(_lib.load().fvc_conv_x3_layout_id(128, 128, 3, 2, 1))
    pc._check_layout()
    monkeypatch.setenv("FVC_DX", "0")
    for _ in range(3):
        with pytest.raises(_lib.FvcError):
            pc._check_layout()
    monkeypatch.setenv("FVC_DX", "1")
    pc._check_layout()


def test_segment_framing_rows():
    """'segment' framing (the codec's default stream cut): >= 512 symbols per stream, a power-of-two
    count of equal contiguous segments per (frame, channel) row; the other framings unchanged."""
    from fastvideocodec_amd.net import segments, stream_rows
    assert segments(8160) == 8 and segments(32640) == 32 and segments(510) == 1 and segments(256) == 1
    assert segments(1024) == 2 and segments(1 << 20) == 64
    assert stream_rows("segment", 2, 128, 8160) == (2 * 128 * 8, 1020)
    assert stream_rows("channel", 2, 128, 8160) == (256, 8160)
    assert stream_rows("item", 2, 128, 8160) == (2, 128 * 8160)
