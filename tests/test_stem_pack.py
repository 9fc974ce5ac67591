"""CPU: the stem kernel's weight pack (fvc_conv_stem_pack_weight, host C++ in libfvc) and the
kernel's reduction dataflow restated in float64 numpy: per k-step, lane (li, lh) holds the 8 K
values 16 step + 8 lh .. + 7 of its pixel li (K = tap * cinp + channel; one tap of 8 channels when
cinp = 8, two taps of 4 when cinp = 4), the A fragment of lane l is output channel 32 n + (l & 31)
with the same K values. Summing A x B over the steps with the pack's values (hi + lo * 2^-11,
descaled) must equal the direct conv, which pins the pack layout and the kernel's tap indexing
without a GPU."""
import ctypes

import numpy as np
import pytest

from fastvideocodec_amd import _lib


def _pack(w):
    cout, cin, k, _ = w.shape
    lib = _lib.load()
    nb = lib.fvc_conv_stem_wpack_bytes(cin, cout, k)
    assert nb > 0
    wp = np.zeros(nb // 2, np.float16)
    osc = ctypes.c_float(0.0)
    wc = np.ascontiguousarray(w, np.float32)
    _lib.call("fvc_conv_stem_pack_weight", wc.ctypes.data, cin, cout, k, wp.ctypes.data, ctypes.addressof(osc))
    return wp, osc.value


@pytest.mark.parametrize("cin,cout,k,s", [(6, 64, 3, 1), (2, 128, 3, 2), (3, 64, 5, 2), (8, 128, 5, 2), (1, 64, 3, 1)])
def test_stem_pack_and_dataflow_equal_direct_conv(cin, cout, k, s):
    rng = np.random.default_rng(cin * 100 + cout + k)
    w = rng.normal(0, 0.1, (cout, cin, k, k))
    wp, osc = _pack(w)
    cinp = 4 if cin <= 4 else 8
    tpl = 1 if cinp == 8 else 2           # taps per lane per step
    tps = 2 * tpl
    kt = k * k
    ns = (kt + tps - 1) // tps
    nt = cout // 32
    a = wp.reshape(ns, nt, 2, 64, 8).astype(np.float64)
    A = (a[:, :, 0] + a[:, :, 1] / 2048.0) * osc       # [step][n][lane][8]
    H, W = 7, 10
    x = np.zeros((H, W, cinp))
    x[..., :cin] = rng.normal(0, 1, (H, W, cin))
    Ho, Wo = H // s, W // s
    p = k // 2
    y = np.zeros((Ho, Wo, cout))
    for oy in range(Ho):
        for ox in range(Wo):
            for st in range(ns):
                for lh in range(2):
                    # the lane's 8 K values (the kernel's tap loads)
                    bvals = np.zeros(8)
                    for t in range(tpl):
                        tap = st * tps + lh * tpl + t
                        if tap >= kt:
                            continue
                        ky, kx = divmod(tap, k)
                        iy, ix = oy * s + ky - p, ox * s + kx - p
                        if 0 <= iy < H and 0 <= ix < W:
                            bvals[t * cinp if cinp == 4 else 0:(t + 1) * cinp if cinp == 4 else 8] = x[iy, ix]
                    for n in range(nt):
                        for li in range(32):
                            y[oy, ox, 32 * n + li] += A[st, n, lh * 32 + li] @ bvals
    ref = np.zeros((Ho, Wo, cout))
    xpad = np.pad(x[..., :cin], ((p, p), (p, p), (0, 0)))
    for oy in range(Ho):
        for ox in range(Wo):
            patch = xpad[oy * s:oy * s + k, ox * s:ox * s + k, :]          # [ky][kx][ci]
            ref[oy, ox] = np.einsum("oikl,kli->o", w, patch)
    err = np.abs(y - ref).max() / np.abs(ref).max()
    assert err < 1e-6, err  # only the weight split's rounding (~2^-22 relative) remains


def test_stem_supported_geometries():
    lib = _lib.load()
    ok = [(6, 64, 3, 1), (2, 128, 3, 2), (3, 64, 5, 2), (8, 128, 3, 1), (4, 64, 5, 2)]
    for cin, cout, k, s in ok:
        assert lib.fvc_conv_stem_supported(cin, cout, k, s, 0) == 1, (cin, cout, k, s)
        assert lib.fvc_conv_stem_wpack_bytes(cin, cout, k) > 0
    for cin, cout, k, s, tr in [(9, 64, 3, 1, 0), (6, 32, 3, 1, 0), (6, 64, 5, 1, 0), (6, 64, 7, 1, 0), (8, 32, 7, 1, 0),
                                (6, 64, 3, 2, 1), (0, 64, 3, 1, 0)]:
        assert lib.fvc_conv_stem_supported(cin, cout, k, s, tr) == 0, (cin, cout, k, s, tr)
