"""Host side of the torchac-compatible coder (fvc_torchac_encode / fvc_torchac_decode in
libfvc.so: plain CPU code, no GPU needed) against the restated torchac algorithm
(oracle/torchac_ref.py). torchac itself is absent: parity unpinned against it (see the oracle)."""
import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import torchac_ref as T  # noqa: E402

from fastvideocodec_amd import _lib  # noqa: E402


def _random_case(rng, N, Lp, peaked=False):
    pmf = rng.random((N, Lp - 1)) ** (8 if peaked else 2) + 1e-7
    cdf = np.concatenate([np.zeros((N, 1)), np.cumsum(pmf, 1) / pmf.sum(1, keepdims=True)], 1)
    cdf = np.minimum(cdf, 1).astype(np.float32)
    sym = np.array([rng.choice(Lp - 1, p=pmf[i] / pmf[i].sum()) for i in range(N)], np.int16)
    return cdf, sym


def _c_encode(rows, sym):
    Lp = rows.shape[-1]
    rows = rows.astype(np.int64)
    s = sym.astype(np.int64)
    lo = rows[np.arange(len(s)), s].astype(np.uint32)
    hi = np.where(s == Lp - 2, 1 << 16, rows[np.arange(len(s)), np.minimum(s + 1, Lp - 1)]).astype(np.uint32)
    lib = _lib.load()
    cap = lib.fvc_torchac_max_bytes(len(s))
    out = np.empty(cap, np.uint8)
    n_out = ctypes.c_size_t(0)
    _lib.call("fvc_torchac_encode", lo.ctypes.data, hi.ctypes.data, len(s), out.ctypes.data, cap, ctypes.addressof(n_out))
    return out[:n_out.value].tobytes()


def _c_decode(rows, data, n, row_index=None):
    Lp = rows.shape[-1]
    rows = np.ascontiguousarray(rows, np.uint16)
    sym = np.empty(max(n, 1), np.int16)
    buf = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    ri = None if row_index is None else np.ascontiguousarray(row_index, np.int32)
    _lib.call("fvc_torchac_decode", rows.ctypes.data, Lp, None if ri is None else ri.ctypes.data, rows.shape[0], n,
              buf.ctypes.data, len(data), sym.ctypes.data)
    return sym[:n]


@pytest.mark.parametrize("N,Lp,peaked", [(1, 3, False), (7, 4, True), (200, 17, False), (500, 300, True),
                                         (300, 2 * 150, False)])
def test_encode_decode_vs_oracle(N, Lp, peaked):
    rng = np.random.default_rng(N * 1000 + Lp)
    cdf, sym = _random_case(rng, N, Lp, peaked)
    rows = T.normalize(cdf)
    ref = T.encode_int16_normalized_cdf(rows, sym)
    got = _c_encode(rows, sym)
    assert got == ref
    assert np.array_equal(_c_decode(rows, got, N), sym)
    assert np.array_equal(T.decode_int16_normalized_cdf(rows, got), sym)


def test_shared_rows_and_edges():
    # per-channel rows shared by many elements (the BitEstimator case), the max symbol (Lp - 2),
    # whose upper bound is 2^16, and a degenerate row concentrated on one bin
    rng = np.random.default_rng(3)
    Lp, C = 300, 4
    cdf = np.zeros((C, Lp), np.float32)
    for c in range(C):
        p = rng.random(Lp - 1) ** 6
        cdf[c, 1:] = np.cumsum(p) / p.sum()
    cdf[3] = 0
    cdf[3, 151:] = 1  # all mass on symbol 150
    rows = T.normalize(np.minimum(cdf, 1))
    row_index = rng.integers(0, C, 2000).astype(np.int32)
    sym = np.array([rng.integers(0, Lp - 1) if r < 3 else 150 for r in row_index], np.int16)
    sym[:5] = Lp - 2
    full = rows[row_index]
    data = _c_encode(full, sym)
    assert data == T.encode_int16_normalized_cdf(full, sym)
    assert np.array_equal(_c_decode(rows, data, len(sym), row_index), sym)


def test_normalization_matches_torchac_rule():
    # torchac: round(cdf * (2^16 - (Lp-1))) + k as int16 bits (the last entry may wrap)
    Lp = 300
    cdf = np.linspace(0, 1, Lp, dtype=np.float32)[None, :]
    rows = T.normalize(cdf)
    assert rows[0, 0] == 0 and rows[0, -2] == (round(float(np.float32(298 / 299)) * 65237) + 298) & 0xFFFF
    assert rows[0, -1] == (65237 + 299) & 0xFFFF  # 65536 wraps to 0


def test_bounds_errors_and_empty():
    with pytest.raises(ValueError):
        T.check_bounds(np.array([[0, 0.5, 1.2]], np.float32), np.array([0]))
    with pytest.raises(ValueError):
        T.check_bounds(np.array([[0, 0.5, 1.0]], np.float32), np.array([2]))  # symbols are 0 .. Lp - 2
    T.check_bounds(np.array([[0, 0.5, 1.0]], np.float32), np.array([1]))
    rows = T.normalize(np.array([[0, 0.5, 1.0]], np.float32))
    empty = np.zeros(0, np.int16)
    assert _c_encode(rows[:0], empty) == T.encode_int16_normalized_cdf(rows[:0], empty)
    with pytest.raises(_lib.FvcError):  # an empty interval (hi <= lo) is rejected, not coded
        lib_lo = np.array([5], np.uint32)
        out = np.empty(64, np.uint8)
        n_out = ctypes.c_size_t(0)
        _lib.call("fvc_torchac_encode", lib_lo.ctypes.data, lib_lo.ctypes.data, 1, out.ctypes.data, 64,
                  ctypes.addressof(n_out))
