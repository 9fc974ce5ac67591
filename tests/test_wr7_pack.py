"""CPU: the Winograd-rows F(2,7) weight pack (fvc_conv_wr7_pack_weight, host C++ in libfvc) and
the kernel's dataflow restated in float64 numpy: B^T rows as the kernel's per-wave even / odd
coefficients, its position pairs and output-transform partials, U from the pack (hi + lo * 2^-11,
descaled). The restated pipeline must equal a direct 7x7 correlation, which pins the pack layout,
G, and the constants hard-coded in the kernel without a GPU."""
import ctypes

import numpy as np
import pytest

from fastvideocodec_amd import _lib

# the kernel's per-wave constants (fvc_conv_wr7.hip): positions, even / odd column weights (x 2^4),
# V_a = e + qa o, V_b = pb e + qb o, and the output partials Y_i += ya_i M_a + yb_i M_b
WAVES = [((1, 2), (0, 1, -4.25, 1), (1, -4.25, 1, 0), (1, 1, -1), ((1, 1), (1, -1))),
         ((3, 4), (0, .25, -1.25, 1), (.5, -2.5, 2, 0), (1, 1, -1), ((1, 1), (2, -2))),
         ((5, 6), (0, 4, -5, 1), (2, -2.5, .5, 0), (1, 1, -1), ((1, 1), (.5, -.5))),
         ((0, 7), (-1, 5.25, -5.25, 1), (-1, 5.25, -5.25, 1), (0, 0, 1), ((1, 0), (0, 1)))]


def _unpack(up, nt, osc):
    """packed fp16 [wave][pp][dy][n][plane][lane][8] -> U[position][dy][co][ci] (float64, true scale
    incl. the kernel's 2^-4 V scale folded back)."""
    a = up.reshape(4, 2, 7, nt, 2, 64, 8).astype(np.float64)
    val = a[:, :, :, :, 0] + a[:, :, :, :, 1] / 2048.0          # [w][pp][dy][n][lane][8]
    U = np.zeros((8, 7, 16 * nt, 32))
    for w, (pos, *_rest) in enumerate(WAVES):
        for pp in range(2):
            for n in range(nt):
                for lane in range(64):
                    co = 16 * n + (lane & 15)
                    U[pos[pp], :, co, 8 * (lane >> 4):8 * (lane >> 4) + 8] = val[w, pp, :, n, lane, :]
    return U * osc / 16.0  # osc = 2^(4 - kw)


def _pack(w, cin, cout, ci0, co0, nt):
    lib = _lib.load()
    up = np.zeros(lib.fvc_conv_wr7_wpack_bytes(nt) // 2, np.float16)
    osc = ctypes.c_float(0.0)
    wc = np.ascontiguousarray(w, np.float32)
    _lib.call("fvc_conv_wr7_pack_weight", wc.ctypes.data, cin, cout, ci0, co0, nt, up.ctypes.data,
              ctypes.addressof(osc))
    return up, osc.value


@pytest.mark.parametrize("cin,cout,ci0,co0,nt", [(32, 64, 0, 32, 2), (64, 32, 32, 0, 2), (32, 16, 0, 0, 1)])
def test_wr7_pack_and_dataflow_equal_direct_conv(cin, cout, ci0, co0, nt):
    rng = np.random.default_rng(cin + cout)
    w = rng.normal(0, 0.05, (cout, cin, 7, 7))
    up, osc = _pack(w, cin, cout, ci0, co0, nt)
    U = _unpack(up, nt, osc)
    H, Wd = 9, 14
    x = rng.normal(0, 1, (32, H, Wd))                     # this launch's 32 input channels
    xp = np.pad(x, ((0, 0), (3, 3), (3, 4)))              # zero padding (+1 column: 2-px tiles)
    T = (Wd + 1) // 2
    Y = np.zeros((16 * nt, H, 2 * T))
    for w_, (pos, E, O, (qa, pb, qb), (y0c, y1c)) in enumerate(WAVES):
        M = {}
        for pp in range(2):
            M[pos[pp]] = np.zeros((16 * nt, H, T))
        for yy in range(H):
            for dy in range(7):
                row = xp[:, yy + dy, :]                       # [32, Wd + 7]
                for t in range(T):
                    xs = row[:, 2 * t:2 * t + 8] / 16.0           # the kernel's 2^-4 V scale
                    e = sum(E[k] * xs[:, 2 * k] for k in range(4))
                    o = sum(O[k] * xs[:, 2 * k + 1] for k in range(4))
                    va, vb = e + qa * o, pb * e + qb * o
                    M[pos[0]][:, yy, t] += U[pos[0], dy] @ va * 16.0
                    M[pos[1]][:, yy, t] += U[pos[1], dy] @ vb * 16.0
        for i, (ca, cb) in enumerate((y0c, y1c)):
            Y[:, :, i::2] += ca * M[pos[0]] + cb * M[pos[1]]
    ref = np.zeros((16 * nt, H, Wd))
    xq = np.pad(x, ((0, 0), (3, 3), (3, 3)))
    wb = w[co0:co0 + 16 * nt, ci0:ci0 + 32]
    for dy in range(7):
        for dx in range(7):
            ref += np.einsum("oc,chw->ohw", wb[:, :, dy, dx], xq[:, dy:dy + H, dx:dx + Wd])
    err = np.abs(Y[:, :, :Wd] - ref).max() / np.abs(ref).max()
    assert err < 2e-6, err   # the fp16 hi / lo split of U (~2^-22) bounds it


def test_wr7_supported_geometries():
    lib = _lib.load()
    ok = [(c, o) for c in (8, 16, 32, 64, 128) for o in (2, 16, 32, 64) if lib.fvc_conv_wr7_supported(c, o, 7, 1, 0)]
    assert ok == [(32, 16), (32, 32), (32, 64), (64, 16), (64, 32)]
    assert not lib.fvc_conv_wr7_supported(32, 64, 3, 1, 0) and not lib.fvc_conv_wr7_supported(32, 64, 7, 2, 0)
