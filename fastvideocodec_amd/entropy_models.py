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
    """Packed rANS output of S streams: words (uint32 little-endian) + offsets (in words).
    ``status`` (device int32[1], from fvc_rans_pack) is FVC_ENOSPC if a stream ran out of space;
    reading the bytes checks it."""

    def __init__(self, packed: torch.Tensor, pack_off: torch.Tensor, nstreams: int, status=None):
        self.packed = packed
        self.pack_off = pack_off
        self.nstreams = nstreams
        self.status = status

    def nbytes_device(self) -> torch.Tensor:
        return self.pack_off[-1] * 4

    def check(self):
        """Raise FvcError if the encoder reported an error (waits for the encode)."""
        if self.status is not None and int(self.status.item()) != 0:
            raise _lib.FvcError(f"rANS encode failed with status {int(self.status.item())}")

    def to_bytes_list(self):
        self.check()
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
        if n == 0:  # every stream is just the flushed initial state; the kernels need real pointers
            symbols = indexes = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.call("fvc_rans_encode", symbols.data_ptr(), indexes.data_ptr(), sym_off.data_ptr(), S, S * n,
                  self.cdf.data_ptr(), self.cdf.shape[1], self.cdf_length.data_ptr(), self.offset.data_ptr(),
                  ws.data_ptr(), words.data_ptr(), word_off.data_ptr(), nwords.data_ptr(), st)
        pack_off = torch.empty(S + 1, dtype=torch.int64, device=self.device)
        packed = torch.empty_like(words)
        status = torch.empty(1, dtype=torch.int32, device=self.device)
        _lib.call("fvc_rans_pack", words.data_ptr(), word_off.data_ptr(), nwords.data_ptr(), S,
                  pack_off.data_ptr(), packed.data_ptr(), status.data_ptr(), st)
        return EncodedStreams(packed, pack_off, S, status)

    def decode(self, enc: EncodedStreams, indexes: torch.Tensor, check=True, defer=None) -> torch.Tensor:
        """defer: a list to append the device status tensors to instead of checking them here
        (the caller checks them all with one host wait, e.g. VideoCompressor.decode_latents)."""
        S, n = indexes.shape
        K._chk(indexes, name="indexes", dtype=torch.int32)
        if enc.nstreams != S:
            raise ValueError("stream count mismatch")
        if check and defer is None:
            enc.check()
        sym_off = self._sym_off(S, n)
        out = torch.empty((S, n), dtype=torch.int32, device=self.device)
        status = torch.empty(S, dtype=torch.int32, device=self.device)
        _lib.call("fvc_rans_decode", enc.packed.data_ptr(), enc.pack_off.data_ptr(), indexes.data_ptr(),
                  sym_off.data_ptr(), S, self.ntables, self.cdf.shape[1], self.cdf_length.data_ptr(),
                  self.offset.data_ptr(),
                  self.lut.data_ptr(), out.data_ptr(), status.data_ptr(), K.rans_streams_per_block(),
                  K.stream_handle())
        if check and defer is not None:
            if enc.status is not None:
                defer.append(enc.status.view(-1))
            defer.append(status)
        elif check and int(status.abs().max()) != 0:
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
        n = len(symbols)  # n == 0 still flushes the initial state (8 bytes), as compressai does
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


# ------------------------------------------------------------------ compressai-framed API
# compressai's EntropyModel.compress emits ONE string per batch item covering the item's whole
# (C, H, W) latent in C order (entropy_models.py:80-94 -> compressai EntropyModel.compress /
# decompress). The classes below reproduce that framing and API on the device coder: the B
# strings of a batch are B independent rANS streams of C*H*W symbols, coded in one launch. (The
# codec's own bitstream, net.PFrameBitstream, cuts each item into one stream per channel so that
# decode runs C-way parallel; both framings code the same symbol sequence per stream the way
# compressai's encode_with_indexes does.)
class _CompressaiEntropyModel:
    """compressai.entropy_models.EntropyModel surface: buffers ``_quantized_cdf``,
    ``_cdf_length``, ``_offset``; ``compress(inputs, indexes, means)`` -> list[bytes];
    ``decompress(strings, indexes, dtype, means)``. Tensors are NCHW on the device."""

    def __init__(self, device=None):
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self._quantized_cdf = self._cdf_length = self._offset = None
        self._coder = None

    def _set_tables(self, cdf, cdf_length, offset):
        self._coder = RangeCoder(cdf, cdf_length, offset, self.device)
        self._quantized_cdf = self._coder.cdf
        self._cdf_length = self._coder.cdf_length
        self._offset = self._coder.offset

    def _check_ready(self):
        if self._coder is None:
            raise ValueError("Uninitialized CDFs. Run update() first")

    def quantize_symbols(self, inputs, means=None) -> torch.Tensor:
        """round(inputs - means).int() (EntropyModel.quantize(..., "symbols", means))."""
        x = inputs.float().contiguous()
        K._chk(x, name="inputs")
        m = None
        if means is not None:
            m = means.float().expand_as(x).contiguous()
            K._chk(m, x.shape, name="means")
        sym = torch.empty(x.shape, dtype=torch.int32, device=x.device)
        _lib.call("fvc_quantize_symbols", x.data_ptr(), K._ptr(m), sym.data_ptr(), x.numel(), K.stream_handle())
        return sym

    def dequantize(self, symbols, means=None, dtype=torch.float):
        out = torch.empty(symbols.shape, dtype=torch.float32, device=symbols.device)
        m = None
        if means is not None:
            m = means.float().expand(symbols.shape).contiguous()
        _lib.call("fvc_dequantize_symbols", symbols.data_ptr(), K._ptr(m), out.data_ptr(), symbols.numel(),
                  K.stream_handle())
        return out.to(dtype)

    def compress(self, inputs, indexes, means=None):
        self._check_ready()
        if inputs.dim() < 2:
            raise ValueError("Invalid `inputs` size. Expected a tensor with at least 2 dimensions.")
        if inputs.shape != indexes.shape:
            raise ValueError("`inputs` and `indexes` should have the same size.")
        sym = self.quantize_symbols(inputs, means)
        B = sym.shape[0]
        idx = indexes.to(self.device, torch.int32).contiguous()
        if int(idx.min()) < 0 or int(idx.max()) >= self._coder.ntables:
            raise ValueError("index out of range")
        enc = self._coder.encode(sym.view(B, -1), idx.view(B, -1))
        return enc.to_bytes_list()

    def decompress(self, strings, indexes, dtype=torch.float, means=None):
        self._check_ready()
        if not isinstance(strings, (tuple, list)):
            raise ValueError("Invalid `strings` parameter type.")
        if len(strings) != indexes.size(0):
            raise ValueError("Invalid strings or indexes parameters")
        if indexes.dim() < 2:
            raise ValueError("Invalid `indexes` size. Expected a tensor with at least 2 dimensions.")
        B = len(strings)
        idx = indexes.to(self.device, torch.int32).contiguous()
        enc = EncodedStreams.from_bytes_list([bytes(x) for x in strings], self.device)
        sym = self._coder.decode(enc, idx.view(B, -1)).view(indexes.shape)
        return self.dequantize(sym, means, dtype)


class EntropyBottleneck(_CompressaiEntropyModel):
    """compressai ``EntropyBottleneck`` surface over DVC's per-channel BitEstimator CDF
    (bitEstimator.py:27-42): tables from ``FactorizedTables`` (medians 0), symbols = round(x),
    table index = channel."""

    def __init__(self, params, device=None):
        super().__init__(device)
        self.params = params  # [11, C] BitEstimator parameters (net.BitEstimator.params())
        self.channels = int(params.shape[1])

    def update(self, force=False):
        if self._coder is not None and not force:
            return False
        t = FactorizedTables(torch.as_tensor(self.params).detach().cpu().numpy())
        self._set_tables(t.cdf, t.cdf_length, t.offset)
        return True

    def _build_indexes(self, size):
        return torch.arange(self.channels, dtype=torch.int32, device=self.device).view(1, -1, *([1] * (len(size) - 2))).expand(size).contiguous()

    def compress(self, x):
        return super().compress(x, self._build_indexes(x.size()))

    def decompress(self, strings, size):
        output_size = (len(strings), self.channels, *size)
        return super().decompress(strings, self._build_indexes(output_size))


class ConditionalEntropyModel(_CompressaiEntropyModel):
    """compressai ``GaussianConditional`` surface: ``update_scale_table``, ``update``,
    ``build_indexes(scales)``; ``dist`` = 'laplace' (DVC's feature likelihood, net.py:138-141;
    LaplaceTables) or 'gaussian' (compressai's own, used by RLVC's RPM; GaussianTables)."""

    def __init__(self, scale_table=None, dist="laplace", device=None):
        super().__init__(device)
        self.dist = dist
        self.scale_table = None if scale_table is None else torch.as_tensor(scale_table, dtype=torch.float32)
        self._table_dev = None

    def update_scale_table(self, scale_table, force=False):
        if self._coder is not None and not force:
            return False
        self.scale_table = torch.as_tensor(scale_table, dtype=torch.float32)
        self.update()
        return True

    def update(self):
        st = self.scale_table if self.scale_table is not None else get_scale_table()
        t = LaplaceTables(st) if self.dist == "laplace" else GaussianTables(st)
        self._set_tables(t.cdf, t.cdf_length, t.offset)
        self._table_dev = torch.from_numpy(np.ascontiguousarray(t.scale_table, np.float32)).to(self.device)

    def build_indexes(self, scales):
        self._check_ready()
        s = scales.float().contiguous()
        K._chk(s, name="scales")
        idx = torch.empty(s.shape, dtype=torch.int32, device=s.device)
        _lib.call("fvc_build_indexes_flat", s.data_ptr(), self._table_dev.data_ptr(), self._table_dev.numel(),
                  idx.data_ptr(), s.numel(), K.stream_handle())
        return idx


class GaussianTables:
    """compressai ``GaussianConditional.update()`` (entropy_models.py:18-23 scale table): float32
    torch arithmetic on the host as compressai computes it (multiplier = -Phi^-1(tail_mass/2),
    pmf = Phi((.5-|k|)/s) - Phi((-.5-|k|)/s), Phi(x) = .5 erfc(-x/sqrt 2))."""

    def __init__(self, scale_table=None, tail_mass: float = TAIL_MASS):
        import scipy.stats
        st = torch.as_tensor(scale_table if scale_table is not None else get_scale_table(), dtype=torch.float32).cpu()
        self.scale_table = st.numpy().astype(np.float32)
        multiplier = -float(scipy.stats.norm.ppf(tail_mass / 2))
        pmf_center = torch.ceil(st * multiplier).int()
        pmf_length = 2 * pmf_center + 1
        max_length = int(pmf_length.max())
        samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
        s = st.unsqueeze(1).float()
        cum = lambda v: 0.5 * torch.erfc(-(2 ** -0.5) * v)
        upper = cum((0.5 - samples) / s)
        lower = cum((-0.5 - samples) / s)
        pmf = (upper - lower).numpy()
        tails = (2 * lower[:, 0]).numpy()
        lengths = pmf_length.numpy().astype(np.int64)
        self.cdf = _pack_tables(pmf, tails, lengths)
        self.cdf_length = (lengths + 2).astype(np.int32)
        self.offset = (-pmf_center.numpy()).astype(np.int32)


class RecProbModel:
    """``entropy_models.py:26-94`` RecProbModel surface (the coder API the reference's RLVC path
    calls): ``update(scale_table=None, force=False)``, ``compress(x) -> list[bytes]`` (one string
    per batch item over (C,H,W)), ``decompress(strings, shape)``, ``get_actual_bits(strings)``,
    ``get_estimate_bits(likelihoods)``. ``RPM_flag`` False: factorized entropy bottleneck;
    True: conditional model on ``self.sigma`` / ``self.mu`` set by the caller (RPM or, for DVC,
    the hyperprior's sigma with mu = None)."""

    def __init__(self, channels, bit_estimator_params=None, dist="gaussian", device=None):
        self.channels = int(channels)
        self.sigma = self.mu = self.prior_latent = None
        self.RPM_flag = False
        self.entropy_bottleneck = (EntropyBottleneck(bit_estimator_params, device)
                                   if bit_estimator_params is not None else None)
        self.gaussian_conditional = ConditionalEntropyModel(None, dist, device)

    def set_RPM(self, RPM_flag):
        self.RPM_flag = RPM_flag

    def update(self, scale_table=None, force=False):
        if scale_table is None:
            scale_table = get_scale_table()
        updated = self.gaussian_conditional.update_scale_table(scale_table, force=force)
        if self.entropy_bottleneck is not None:
            updated |= self.entropy_bottleneck.update(force=force)
        return updated

    def get_actual_bits(self, string):
        return torch.tensor(float(len(b"".join(string)) * 8))

    def get_estimate_bits(self, likelihoods):
        return torch.sum(torch.clamp(-1.0 * torch.log(likelihoods + 1e-5) / math.log(2.0), 0, 50))

    def compress(self, x):
        if self.RPM_flag:
            indexes = self.gaussian_conditional.build_indexes(self.sigma)
            return self.gaussian_conditional.compress(x, indexes, means=self.mu)
        return self.entropy_bottleneck.compress(x)

    def decompress(self, string, shape):
        if self.RPM_flag:
            indexes = self.gaussian_conditional.build_indexes(self.sigma)
            return self.gaussian_conditional.decompress(string, indexes, means=self.mu)
        return self.entropy_bottleneck.decompress(string, shape)
