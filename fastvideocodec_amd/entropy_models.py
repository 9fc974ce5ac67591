"""Entropy models and the device range coder for the DVC latents.

Mirrors the coder API the reference reaches through ``entropy_models.py`` (compressai):

* ``get_scale_table`` — ``entropy_models.py:18-23``;
* ``FactorizedTables`` — ``EntropyBottleneck.update()`` semantics for DVC's per-channel
  ``BitEstimator`` CDF (``DVC/subnet/bitEstimator.py:27-42``). DVC has no learned quantiles, so
  the support is solved from the CDF itself: minima/maxima = ceil of the tail_mass/2 quantiles
  around the median 0 (DVC quantises by rounding at 0, ``net.py:76,91``), capped at ``max_half``;
* ``LaplaceTables`` — ``GaussianConditional.update()`` over the scale table with the Laplace
  CDF DVC estimates feature bits with (``net.py:138-141``); multiplier = -ln(tail_mass);
* ``build_indexes`` — ``GaussianConditional.build_indexes``;
* ``RangeCoder`` — batched device rANS, each stream byte-identical to compressai
  ``RansEncoder.encode_with_indexes`` on that stream's symbols;
* ``RansEncoder`` / ``RansDecoder`` — the compressai pybind11 call signatures
  (list in, bytes out), served by the device coder.

Tables are built once on the host (as compressai's ``update()`` does) with pmfs evaluated in
float64, cast to float32 and quantised by the C-ABI ``fvc_pmf_to_quantized_cdf``.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from . import kernels as K

SCALES_MIN = 0.11
SCALES_MAX = 256
SCALES_LEVELS = 64
PRECISION = 16
TAIL_MASS = 1e-9


def get_scale_table(min=SCALES_MIN, max=SCALES_MAX, levels=SCALES_LEVELS):
    """entropy_models.py:18-23 (float32, as torch computes it)."""
    return torch.exp(torch.linspace(math.log(min), math.log(max), levels))


def pmf_to_quantized_cdf(pmf, precision=PRECISION) -> np.ndarray:
    """compressai pmf_to_quantized_cdf via the C-ABI (host). Returns uint32 [len(pmf)+1]."""
    p = np.ascontiguousarray(np.asarray(pmf, dtype=np.float32))
    out = np.empty(p.size + 1, dtype=np.uint32)
    _lib.call("fvc_pmf_to_quantized_cdf", p.ctypes.data, p.size, precision, out.ctypes.data)
    return out


def _pack_tables(pmfs, tails, lengths):
    """EntropyModel._pmf_to_cdf: per table prob = cat(pmf[:len], tail) -> quantised cdf."""
    max_len = int(max(lengths))
    cdf = np.zeros((len(lengths), max_len + 2), dtype=np.int32)
    for i, (p, t, n) in enumerate(zip(pmfs, tails, lengths)):
        prob = np.concatenate([np.asarray(p[:n], np.float64), [t]]).astype(np.float32)
        q = pmf_to_quantized_cdf(prob)
        cdf[i, : q.size] = q.astype(np.int32)
    return cdf


# ------------------------------------------------------------------ factorized (BitEstimator)
def bitestimator_logits(params: np.ndarray, x: np.ndarray) -> np.ndarray:
    """Pre-sigmoid output of BitEstimator (bitEstimator.py:18-42), float64, per channel.

    params: [11, C] rows h1 b1 a1 h2 b2 a2 h3 b3 a3 h4 b4; x: [C, n]."""
    p = params.astype(np.float64)
    sp = lambda v: np.where(v > 20.0, v, np.log1p(np.exp(np.minimum(v, 20.0))))  # F.softplus
    x = x.astype(np.float64)
    for f in range(3):
        h, b, a = p[3 * f][:, None], p[3 * f + 1][:, None], p[3 * f + 2][:, None]
        x = x * sp(h) + b
        x = x + np.tanh(x) * np.tanh(a)
    return x * sp(p[9][:, None]) + p[10][:, None]


def _sigmoid(v):
    return 0.5 * (1.0 + np.tanh(0.5 * v))


class FactorizedTables:
    def __init__(self, params: np.ndarray, tail_mass: float = TAIL_MASS, max_half: int = 150):
        params = np.asarray(params, np.float32)
        C = params.shape[1]
        self.channels = C
        # quantiles of the monotone CDF by bisection on the logits
        target_lo = math.log(tail_mass / 2) - math.log1p(-tail_mass / 2)   # logit(tail/2)
        target_hi = -target_lo
        lo = np.full(C, -1e4)
        hi = np.full(C, 1e4)
        q = {}
        for name, target in (("q0", target_lo), ("q2", target_hi)):
            a, b = lo.copy(), hi.copy()
            for _ in range(200):
                m = 0.5 * (a + b)
                v = bitestimator_logits(params, m[:, None])[:, 0]
                a = np.where(v < target, m, a)
                b = np.where(v < target, b, m)
            q[name] = 0.5 * (a + b)
        minima = np.clip(np.ceil(0.0 - q["q0"]), 0, max_half).astype(np.int64)
        maxima = np.clip(np.ceil(q["q2"] - 0.0), 0, max_half).astype(np.int64)
        self.offset = (-minima).astype(np.int32)
        pmf_start = -minima
        lengths = (maxima + minima + 1).astype(np.int64)
        max_len = int(lengths.max())
        samples = np.arange(max_len)[None, :] + pmf_start[:, None]
        lower = bitestimator_logits(params, samples - 0.5)
        upper = bitestimator_logits(params, samples + 0.5)
        sign = -np.sign(lower + upper)
        pmf = np.abs(_sigmoid(sign * upper) - _sigmoid(sign * lower))
        tails = []
        for c in range(C):
            n = lengths[c]
            tails.append(_sigmoid(lower[c, 0]) + _sigmoid(-upper[c, n - 1]))
        self.cdf = _pack_tables(pmf, tails, lengths)
        self.cdf_length = (lengths + 2).astype(np.int32)


# ------------------------------------------------------------------ conditional Laplace
def _laplace_std_cdf(x):
    return 0.5 - 0.5 * np.sign(x) * np.expm1(-np.abs(x))


class LaplaceTables:
    def __init__(self, scale_table=None, tail_mass: float = TAIL_MASS):
        if scale_table is None:
            scale_table = get_scale_table()
        st = np.asarray(torch.as_tensor(scale_table, dtype=torch.float32).numpy(), np.float64)
        self.scale_table = st.astype(np.float32)
        multiplier = -math.log(tail_mass)  # -(Laplace standardized quantile at tail_mass/2)
        pmf_center = np.ceil(st * multiplier).astype(np.int64)
        lengths = 2 * pmf_center + 1
        max_len = int(lengths.max())
        samples = np.abs(np.arange(max_len)[None, :] - pmf_center[:, None]).astype(np.float64)
        s = st[:, None]
        upper = _laplace_std_cdf((0.5 - samples) / s)
        lower = _laplace_std_cdf((-0.5 - samples) / s)
        pmf = upper - lower
        tails = 2 * lower[:, 0]
        self.cdf = _pack_tables(pmf, tails, lengths)
        self.cdf_length = (lengths + 2).astype(np.int32)
        self.offset = (-pmf_center).astype(np.int32)


# ------------------------------------------------------------------ device range coder
class EncodedStreams:
    """Packed rANS output of S streams: words (uint32 little-endian) + offsets (in words)."""

    def __init__(self, packed: torch.Tensor, pack_off: torch.Tensor, nstreams: int):
        self.packed = packed
        self.pack_off = pack_off
        self.nstreams = nstreams

    def nbytes_device(self) -> torch.Tensor:
        return self.pack_off[-1] * 4

    def to_bytes_list(self):
        off = self.pack_off.cpu().numpy()
        words = self.packed[: int(off[-1])].cpu().numpy().view(np.uint32)
        return [words[off[i]: off[i + 1]].astype("<u4").tobytes() for i in range(self.nstreams)]

    @classmethod
    def from_bytes_list(cls, strings, device):
        lens = [len(s) // 4 for s in strings]
        off = np.zeros(len(strings) + 1, np.int64)
        off[1:] = np.cumsum(lens)
        buf = np.frombuffer(b"".join(strings), dtype="<u4").astype(np.uint32)
        packed = torch.from_numpy(buf.view(np.int32).copy()).to(device) if buf.size else torch.zeros(1, dtype=torch.int32, device=device)
        return cls(packed, torch.from_numpy(off).to(device), len(strings))


class RangeCoder:
    """rANS over a fixed table set (cdf [T, L] int32, cdf_length [T], offset [T])."""

    def __init__(self, cdf, cdf_length, offset, device):
        self.cdf = torch.as_tensor(np.ascontiguousarray(cdf, np.int32)).to(device)
        self.cdf_length = torch.as_tensor(np.ascontiguousarray(cdf_length, np.int32)).to(device)
        self.offset = torch.as_tensor(np.ascontiguousarray(offset, np.int32)).to(device)
        self.device = torch.device(device)
        self._offs = {}
        nt = self.cdf.shape[0]
        self.ntables = nt
        nb = _lib.load().fvc_rans_lut_bytes(nt, self.cdf.shape[1])
        self.lut = torch.empty((nb + 3) // 4, dtype=torch.int32, device=self.device)
        _lib.call("fvc_rans_build_lut", self.cdf.data_ptr(), self.cdf.shape[1], self.cdf_length.data_ptr(), nt,
                  self.lut.data_ptr(), K.stream_handle(self.device))

    def _sym_off(self, S, n):
        key = ("s", S, n)
        if key not in self._offs:
            self._offs[key] = (torch.arange(S + 1, dtype=torch.int64) * n).to(self.device)
        return self._offs[key]

    def _word_off(self, S, n):
        key = ("w", S, n)
        if key not in self._offs:
            cap = 2 * n + 8
            self._offs[key] = (torch.arange(S + 1, dtype=torch.int64) * cap).to(self.device)
        return self._offs[key]

    def encode(self, symbols: torch.Tensor, indexes: torch.Tensor) -> EncodedStreams:
        """symbols/indexes: int32 [S, n] device tensors (S equal-length streams)."""
        S, n = symbols.shape
        K._chk(symbols, name="symbols", dtype=torch.int32)
        K._chk(indexes, (S, n), name="indexes", dtype=torch.int32)
        sym_off = self._sym_off(S, n)
        word_off = self._word_off(S, n)
        words = torch.empty(int(S * (2 * n + 8)), dtype=torch.int32, device=self.device)
        nwords = torch.empty(S, dtype=torch.int32, device=self.device)
        ws = torch.empty(max(1, _lib.load().fvc_rans_encode_ws_bytes(S * n) // 4), dtype=torch.int32,
                         device=self.device)
        st = K.stream_handle()
        _lib.call("fvc_rans_encode", symbols.data_ptr(), indexes.data_ptr(), sym_off.data_ptr(), S, S * n,
                  self.cdf.data_ptr(), self.cdf.shape[1], self.cdf_length.data_ptr(), self.offset.data_ptr(),
                  ws.data_ptr(), words.data_ptr(), word_off.data_ptr(), nwords.data_ptr(), st)
        pack_off = torch.empty(S + 1, dtype=torch.int64, device=self.device)
        packed = torch.empty_like(words)
        _lib.call("fvc_rans_pack", words.data_ptr(), word_off.data_ptr(), nwords.data_ptr(), S,
                  pack_off.data_ptr(), packed.data_ptr(), st)
        return EncodedStreams(packed, pack_off, S)

    def decode(self, enc: EncodedStreams, indexes: torch.Tensor, check=True) -> torch.Tensor:
        S, n = indexes.shape
        K._chk(indexes, name="indexes", dtype=torch.int32)
        if enc.nstreams != S:
            raise ValueError("stream count mismatch")
        sym_off = self._sym_off(S, n)
        out = torch.empty((S, n), dtype=torch.int32, device=self.device)
        status = torch.empty(S, dtype=torch.int32, device=self.device)
        _lib.call("fvc_rans_decode", enc.packed.data_ptr(), enc.pack_off.data_ptr(), indexes.data_ptr(),
                  sym_off.data_ptr(), S, self.ntables, self.cdf.shape[1], self.cdf_length.data_ptr(),
                  self.offset.data_ptr(),
                  self.lut.data_ptr(), out.data_ptr(), status.data_ptr(), K.stream_handle())
        if check and int(status.abs().max()) != 0:
            raise _lib.FvcError("corrupt rANS stream")
        return out


# ------------------------------------------------------------------ compressai pybind11 mirror
def _tables_from_lists(cdfs, cdfs_sizes, offsets):
    L = max(len(c) for c in cdfs)
    cdf = np.zeros((len(cdfs), L), np.int32)
    for i, c in enumerate(cdfs):
        cdf[i, : len(c)] = c
    return cdf, np.asarray(cdfs_sizes, np.int32), np.asarray(offsets, np.int32)


class RansEncoder:
    """compressai.ans.RansEncoder: encode_with_indexes(symbols, indexes, cdfs, cdfs_sizes, offsets) -> bytes."""

    def __init__(self, device="cuda"):
        self.device = device

    def encode_with_indexes(self, symbols, indexes, cdfs, cdfs_sizes, offsets) -> bytes:
        if len(symbols) != len(indexes):
            raise ValueError("symbols and indexes must have the same length")
        cdf, sizes, offs = _tables_from_lists(cdfs, cdfs_sizes, offsets)
        idx = np.asarray(indexes, np.int64)
        if idx.size and (idx.min() < 0 or idx.max() >= len(cdfs)):
            raise ValueError("index out of range")
        coder = RangeCoder(cdf, sizes, offs, self.device)
        n = len(symbols)
        if n == 0:
            return b""
        sym = torch.tensor(np.asarray(symbols, np.int32).reshape(1, n), device=self.device)
        ind = torch.tensor(idx.astype(np.int32).reshape(1, n), device=self.device)
        return coder.encode(sym, ind).to_bytes_list()[0]


class RansDecoder:
    """compressai.ans.RansDecoder: decode_with_indexes(encoded, indexes, cdfs, cdfs_sizes, offsets) -> list[int]."""

    def __init__(self, device="cuda"):
        self.device = device

    def decode_with_indexes(self, encoded, indexes, cdfs, cdfs_sizes, offsets):
        cdf, sizes, offs = _tables_from_lists(cdfs, cdfs_sizes, offsets)
        n = len(indexes)
        if n == 0:
            return []
        coder = RangeCoder(cdf, sizes, offs, self.device)
        ind = torch.tensor(np.asarray(indexes, np.int32).reshape(1, n), device=self.device)
        enc = EncodedStreams.from_bytes_list([bytes(encoded)], self.device)
        return coder.decode(enc, ind).cpu().numpy().reshape(-1).tolist()
