"""ORACLE — test infrastructure only. Coder restatements used as the checker.

* ``pmf_to_quantized_cdf_py`` / ``rans_encode_py`` / ``rans_decode_py``: pure-Python
  restatements of compressai 1.2's C++ coder (cpp_exts/ops/ops.cpp, rans_interface.cpp,
  ryg_rans rans64.h) for small known-answer cases;
* ``pmf_to_quantized_cdf_np``: the quantiser restated on the frequency array (numpy), fast
  enough for every real table; the product's host quantiser edits the cumulative table in place
  instead, so the two are independent programs for one spec;
* ``CRef``: ctypes binding of ``oracle/build/librans_ref.so`` (oracle/rans_ref.c, the same
  algorithm in C) for full-size byte-exact checks and the CPU coder baseline;
* ``factorized_tables`` / ``laplace_tables``: restatements of EntropyBottleneck.update() /
  GaussianConditional.update() (compressai entropy_models.py) specialised to DVC's
  BitEstimator CDF (DVC/subnet/bitEstimator.py:27-42) and Laplace scales (net.py:138-141).

compressai is not installed and not vendored: the coder is "parity
unpinned" against compressai itself; it is pinned by Python == C == device byte equality,
round trips and hand-worked known answers (tests/test_coder_oracle.py).
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

PREC = 16
BYPASS_PREC = 4
MAX_BYPASS = (1 << BYPASS_PREC) - 1
RANS64_L = 1 << 31
MASK64 = (1 << 64) - 1


# ------------------------------------------------------------------ pure Python
def pmf_to_quantized_cdf_py(pmf, precision=PREC):
    """ops.cpp pmf_to_quantized_cdf (float32 products, std::round = half away from zero)."""
    pmf = np.asarray(pmf, np.float32)
    if np.any(pmf < 0) or not np.all(np.isfinite(pmf)):
        raise ValueError("invalid pmf")
    scale = np.float32(1 << precision)
    cdf = [0]
    for p in pmf:
        v = np.float32(p) * scale
        cdf.append(int(math.floor(float(v) + 0.5)) if v >= 0 else -int(math.floor(-float(v) + 0.5)))
    total = sum(cdf)
    if total == 0:
        raise ValueError("pmf sums to zero")
    cdf = [((1 << precision) * c) // total for c in cdf]
    for i in range(1, len(cdf)):
        cdf[i] += cdf[i - 1]
    cdf[-1] = 1 << precision
    n = len(cdf) - 1
    for i in range(n):
        if cdf[i] == cdf[i + 1]:
            best_freq, best_steal = None, -1
            for j in range(n):
                f = cdf[j + 1] - cdf[j]
                if f > 1 and (best_freq is None or f < best_freq):
                    best_freq, best_steal = f, j
            assert best_steal != -1
            if best_steal < i:
                for j in range(best_steal + 1, i + 1):
                    cdf[j] -= 1
            else:
                for j in range(i + 1, best_steal + 1):
                    cdf[j] += 1
    return np.asarray(cdf, np.uint32)


def pmf_to_quantized_cdf_np(pmf, precision=PREC):
    """The same spec (ops.cpp pmf_to_quantized_cdf) restated on the frequency array with numpy,
    fast enough for every real table (Laplace tables reach 10,611 bins with ~7,800 empty ones).
    An empty bin's repair changes exactly two frequencies (freq[i] += 1, freq[donor] -= 1; see
    oracle/rans_ref.c), so no cumulative-table edits are needed."""
    p = np.asarray(pmf, np.float32)
    if p.size == 0 or np.any(~(p >= 0)) or not np.all(np.isfinite(p)):
        raise ValueError("invalid pmf")
    one = 1 << precision
    v = (p * np.float32(one)).astype(np.float64)           # float32 product, exact in float64
    freq = np.floor(v + 0.5).astype(np.int64)              # std::round (v >= 0)
    total = int(freq.sum())
    if total == 0:
        raise ValueError("pmf sums to zero")
    freq = (one * freq) // total
    freq[-1] += one - int(freq.sum())
    for i in np.flatnonzero(freq == 0):                     # bins are repaired in index order
        if freq[i] != 0:
            continue
        cand = np.where(freq > 1, freq, np.iinfo(np.int64).max)
        donor = int(np.argmin(cand))                        # first minimum = ops.cpp's strict <
        if freq[donor] <= 1:
            raise ValueError("no bin to steal from")
        freq[donor] -= 1
        freq[i] += 1
    return np.concatenate([[0], np.cumsum(freq)]).astype(np.uint32)


def _push_symbols(symbols, indexes, cdfs, sizes, offsets):
    q = []
    for s, ci in zip(symbols, indexes):
        cdf = cdfs[ci]
        max_value = int(sizes[ci]) - 2
        value = int(s) - int(offsets[ci])
        raw = 0
        if value < 0:
            raw = -2 * value - 1
            value = max_value
        elif value >= max_value:
            raw = 2 * (value - max_value)
            value = max_value
        q.append((int(cdf[value]), int(cdf[value + 1]) - int(cdf[value]), False))
        if value == max_value:
            nb = 0
            while nb < 8 and (raw >> (nb * BYPASS_PREC)) != 0:
                nb += 1
            val = nb
            while val >= MAX_BYPASS:
                q.append((MAX_BYPASS, MAX_BYPASS + 1, True))
                val -= MAX_BYPASS
            q.append((val, val + 1, True))
            for j in range(nb):
                v = (raw >> (j * BYPASS_PREC)) & MAX_BYPASS
                q.append((v, v + 1, True))
    return q


def rans_encode_py(symbols, indexes, cdfs, sizes, offsets) -> bytes:
    """BufferedRansEncoder.encode_with_indexes + flush (single stream)."""
    q = _push_symbols(symbols, indexes, cdfs, sizes, offsets)
    out = []  # emitted words, in emission order (they end up reversed in memory)
    x = RANS64_L
    while q:
        start, rng, byp = q.pop()
        if not byp:
            x_max = ((RANS64_L >> PREC) << 32) * rng
            if x >= x_max:
                out.append(x & 0xFFFFFFFF)
                x >>= 32
            x = ((x // rng) << PREC) + (x % rng) + start
        else:
            freq = 1 << (16 - BYPASS_PREC)
            x_max = ((RANS64_L >> 16) << 32) * freq
            if x >= x_max:
                out.append(x & 0xFFFFFFFF)
                x >>= 32
            x = ((x << BYPASS_PREC) | start) & MASK64
    words = [x & 0xFFFFFFFF, (x >> 32) & 0xFFFFFFFF] + out[::-1]
    return np.asarray(words, "<u4").tobytes()


def rans_decode_py(data: bytes, indexes, cdfs, sizes, offsets):
    """RansDecoder.decode_with_indexes (single stream)."""
    w = np.frombuffer(data, "<u4").astype(np.uint64).tolist()
    x = int(w[0]) | (int(w[1]) << 32)
    p = 2

    def renorm(x, p):
        if x < RANS64_L:
            x = ((x << 32) | int(w[p])) & MASK64
            p += 1
        return x, p

    out = []
    for ci in indexes:
        cdf = cdfs[ci]
        size = int(sizes[ci])
        max_value = size - 2
        cum = x & ((1 << PREC) - 1)
        s = 0
        while s + 1 < size and int(cdf[s + 1]) <= cum:
            s += 1
        start, freq = int(cdf[s]), int(cdf[s + 1]) - int(cdf[s])
        x = freq * (x >> PREC) + (x & ((1 << PREC) - 1)) - start
        x, p = renorm(x, p)
        value = s
        if value == max_value:
            val = x & MAX_BYPASS
            x >>= BYPASS_PREC
            x, p = renorm(x, p)
            nb = val
            while val == MAX_BYPASS:
                val = x & MAX_BYPASS
                x >>= BYPASS_PREC
                x, p = renorm(x, p)
                nb += val
            raw = 0
            for j in range(nb):
                val = x & MAX_BYPASS
                x >>= BYPASS_PREC
                x, p = renorm(x, p)
                raw |= val << (j * BYPASS_PREC)
            value = raw >> 1
            value = -value - 1 if raw & 1 else value + max_value
        out.append(value + int(offsets[ci]))
    return out


# ------------------------------------------------------------------ C restatement
class CRef:
    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "librans_ref.so")
            if not os.path.exists(path):
                import subprocess
                # oracle/build/ does not exist in a fresh clone: run make in oracle/ itself
                subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(path))], check=True)
            lib = ctypes.CDLL(path)
            vp, ci = ctypes.c_void_p, ctypes.c_int
            lib.ref_pmf_to_quantized_cdf.argtypes = [vp, ci, ci, vp]
            lib.ref_rans_encode.argtypes = [vp, vp, ci, vp, ci, vp, vp, vp, ci]
            lib.ref_rans_decode.argtypes = [vp, ci, vp, ci, vp, ci, vp, vp, vp]
            cls._lib = lib
        return cls._lib

    @classmethod
    def pmf_to_quantized_cdf(cls, pmf, precision=PREC):
        p = np.ascontiguousarray(pmf, np.float32)
        out = np.empty(p.size + 1, np.uint32)
        if cls.lib().ref_pmf_to_quantized_cdf(p.ctypes.data, p.size, precision, out.ctypes.data) != 0:
            raise ValueError("invalid pmf")
        return out

    @classmethod
    def encode(cls, symbols, indexes, cdf, sizes, offsets) -> bytes:
        s = np.ascontiguousarray(symbols, np.int32)
        i = np.ascontiguousarray(indexes, np.int32)
        c = np.ascontiguousarray(cdf, np.int32)
        z = np.ascontiguousarray(sizes, np.int32)
        o = np.ascontiguousarray(offsets, np.int32)
        cap = 2 * s.size + 16
        out = np.empty(cap, np.uint32)
        nw = cls.lib().ref_rans_encode(s.ctypes.data, i.ctypes.data, s.size, c.ctypes.data, c.shape[1],
                                       z.ctypes.data, o.ctypes.data, out.ctypes.data, cap)
        if nw < 0:
            raise RuntimeError("encode overflow")
        return out[:nw].astype("<u4").tobytes()

    @classmethod
    def decode(cls, data: bytes, indexes, cdf, sizes, offsets):
        w = np.frombuffer(data, "<u4").astype(np.uint32)
        i = np.ascontiguousarray(indexes, np.int32)
        c = np.ascontiguousarray(cdf, np.int32)
        z = np.ascontiguousarray(sizes, np.int32)
        o = np.ascontiguousarray(offsets, np.int32)
        out = np.empty(i.size, np.int32)
        if cls.lib().ref_rans_decode(w.ctypes.data, w.size, i.ctypes.data, i.size, c.ctypes.data, c.shape[1],
                                     z.ctypes.data, o.ctypes.data, out.ctypes.data) != 0:
            raise RuntimeError("corrupt stream")
        return out


# ------------------------------------------------------------------ table restatements
def _pack(pmfs, tails, lengths, quantize=None):
    """EntropyModel._pmf_to_cdf; quantize defaults to the numpy restatement (the C one is
    compared against it in tests)."""
    quantize = quantize or pmf_to_quantized_cdf_np
    max_len = int(max(lengths))
    cdf = np.zeros((len(lengths), max_len + 2), np.int32)
    for i, (p, t, n) in enumerate(zip(pmfs, tails, lengths)):
        prob = np.append(np.asarray(p[:n], np.float64), t).astype(np.float32)
        q = quantize(prob)
        cdf[i, : q.size] = q
    return cdf


def _be_logits(prm, x):
    prm = prm.astype(np.float64)
    softplus = lambda v: np.where(v > 20.0, v, np.log1p(np.exp(np.minimum(v, 20.0))))
    for f in range(3):
        x = x * softplus(prm[3 * f][:, None]) + prm[3 * f + 1][:, None]
        x = x + np.tanh(x) * np.tanh(prm[3 * f + 2][:, None])
    return x * softplus(prm[9][:, None]) + prm[10][:, None]


def _sig(v):
    return 0.5 * (1.0 + np.tanh(0.5 * v))


def factorized_tables(params, tail_mass=1e-9, max_half=150, quantize=None):
    """EntropyBottleneck.update() with the BitEstimator CDF and medians fixed at 0."""
    prm = np.asarray(params, np.float32)
    C = prm.shape[1]
    lo_t = math.log(tail_mass / 2) - math.log1p(-tail_mass / 2)
    qs = []
    for target in (lo_t, -lo_t):
        a, b = np.full(C, -1e4), np.full(C, 1e4)
        for _ in range(200):
            m = 0.5 * (a + b)
            below = _be_logits(prm, m[:, None])[:, 0] < target
            a, b = np.where(below, m, a), np.where(below, b, m)
        qs.append(0.5 * (a + b))
    minima = np.clip(np.ceil(-qs[0]), 0, max_half).astype(np.int64)
    maxima = np.clip(np.ceil(qs[1]), 0, max_half).astype(np.int64)
    lengths = maxima + minima + 1
    samples = np.arange(int(lengths.max()))[None, :] - minima[:, None]
    lower, upper = _be_logits(prm, samples - 0.5), _be_logits(prm, samples + 0.5)
    sign = -np.sign(lower + upper)
    pmf = np.abs(_sig(sign * upper) - _sig(sign * lower))
    tails = [_sig(lower[c, 0]) + _sig(-upper[c, lengths[c] - 1]) for c in range(C)]
    return _pack(pmf, tails, lengths, quantize), (lengths + 2).astype(np.int32), (-minima).astype(np.int32)


def laplace_tables(scale_table, tail_mass=1e-9, quantize=None):
    """GaussianConditional.update() with the Laplace CDF (multiplier -ln(tail_mass))."""
    st = np.asarray(scale_table, np.float32).astype(np.float64)
    center = np.ceil(st * -math.log(tail_mass)).astype(np.int64)
    lengths = 2 * center + 1
    samples = np.abs(np.arange(int(lengths.max()))[None, :] - center[:, None]).astype(np.float64)
    cdf = lambda v: 0.5 - 0.5 * np.sign(v) * np.expm1(-np.abs(v))
    upper = cdf((0.5 - samples) / st[:, None])
    lower = cdf((-0.5 - samples) / st[:, None])
    return (_pack(upper - lower, 2 * lower[:, 0], lengths, quantize), (lengths + 2).astype(np.int32),
            (-center).astype(np.int32))


def build_indexes(scales, scale_table):
    """GaussianConditional.build_indexes (lower bound 0.11)."""
    s = np.maximum(np.asarray(scales, np.float32), np.float32(0.11))
    idx = np.full(s.shape, len(scale_table) - 1, np.int32)
    for t in np.asarray(scale_table, np.float32)[:-1]:
        idx -= (s <= t).astype(np.int32)
    return idx


def gaussian_tables(scale_table, tail_mass=1e-9, quantize=None):
    """compressai GaussianConditional.update() (the table build RLVC's RecProbModel runs through
    update_scale_table, entropy_models.py:43-48). compressai evaluates the pmf with float32 torch
    ops (Phi(x) = 0.5 * erfc(-x / sqrt(2))), so this restatement does too; the multiplier is
    -Phi^-1(tail_mass / 2) (scipy.stats.norm.ppf, as compressai's _standardized_quantile)."""
    import scipy.stats
    import torch
    st = torch.as_tensor(np.asarray(scale_table, np.float32))
    mult = -float(scipy.stats.norm.ppf(tail_mass / 2))
    center = torch.ceil(st * mult).int()
    lengths = (2 * center + 1).numpy().astype(np.int64)
    samples = torch.abs(torch.arange(int(lengths.max())).int() - center[:, None]).float()
    phi = lambda v: 0.5 * torch.erfc(v * -(2 ** -0.5))
    upper = phi((0.5 - samples) / st[:, None])
    lower = phi((-0.5 - samples) / st[:, None])
    return (_pack((upper - lower).numpy(), (2 * lower[:, 0]).numpy(), lengths, quantize),
            (lengths + 2).astype(np.int32), (-center.numpy()).astype(np.int32))
