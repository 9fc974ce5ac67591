"""ORACLE — test infrastructure only (tests/). Pure-Python / numpy restatement of torchac's
float-CDF arithmetic coder, the coder DVC's ``calrealbits`` mode calls:
``torchac.encode_float_cdf(cdfs, x.to(int16), check_input_bounds=True)`` and
``torchac.decode_float_cdf(cdfs, byte_stream)`` with 2*mxrange = 300 bins per element
(DVC/net.py:123-138 Laplace feature, :155-168 BitEstimator z, :183-195 BitEstimator mv).

torchac (fab-jul/torchac, the 0.9.x series) is absent from this image and from every manifest of
the reference: there are no golden vectors, so this module restates its
published algorithm and the device/host coder (fastvideocodec_amd/torchac.py,
csrc/fvc_torchac.hip) is held to it byte for byte — **parity unpinned** against torchac itself.

* normalisation (``_convert_to_int_and_normalize``): with Lp bins, cdf_int[k] = int16(round(
  cdf_float[k] * float32(2^16 - (Lp - 1)))) + k (float32 product, round half to even, int16
  wrap-around; the coder reads the values as uint16);
* coder: 32-bit low/high binary arithmetic coder with E1/E2/E3 renormalisation and pending bits,
  bits packed MSB first; symbol s spans [cdf[s], cdf[s+1]) of 2^16, except the last symbol
  (Lp - 2), whose upper bound is 2^16; the stream ends with one disambiguating bit (+ pending)
  and zero padding to a byte. The decoder reads 32 bits (zeros past the end), finds the symbol
  by binary search over cdf[0 .. Lp-2] and skips the renormalisation after the last symbol.
"""
from __future__ import annotations

import numpy as np

PRECISION = 16
_TOP = 1 << 32


def normalize(cdf_float: np.ndarray, needs_normalization: bool = True) -> np.ndarray:
    """float CDF [..., Lp] in [0, 1] -> uint16 [..., Lp] (torchac's int16 bit pattern)."""
    cdf_float = np.asarray(cdf_float, np.float32)
    Lp = cdf_float.shape[-1]
    m = np.float32(2 ** PRECISION - ((Lp - 1) if needs_normalization else 0))
    r = np.rint(cdf_float * m).astype(np.int64)
    if needs_normalization:
        r = r + np.arange(Lp, dtype=np.int64)
    return (r & 0xFFFF).astype(np.uint16)


def check_bounds(cdf_float, sym):
    cdf_float = np.asarray(cdf_float)
    Lp = cdf_float.shape[-1]
    if cdf_float.min() < 0:
        raise ValueError("cdf_float.min() < 0")
    if cdf_float.max() > 1:
        raise ValueError("cdf_float.max() > 1")
    sym = np.asarray(sym)
    if sym.size and (sym.max() >= Lp - 1 or sym.min() < 0):
        raise ValueError("symbol out of [0, Lp - 2]")


class _BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.cache = 0
        self.count = 0

    def put(self, bit):
        self.cache = ((self.cache << 1) | bit) & 0xFF
        self.count += 1
        if self.count == 8:
            self.out.append(self.cache)
            self.cache = 0
            self.count = 0

    def put_with_pending(self, bit, pending):
        self.put(bit)
        for _ in range(pending):
            self.put(1 - bit)

    def flush(self):
        while self.count:
            self.put(0)


def _bounds(cdf_row, s):
    """[c_low, c_high) of symbol s in a uint16 CDF row of Lp entries."""
    max_symbol = len(cdf_row) - 2
    c_low = int(cdf_row[s])
    c_high = (1 << PRECISION) if s == max_symbol else int(cdf_row[s + 1])
    return c_low, c_high


def encode_bounds(lows, highs) -> bytes:
    """Arithmetic-code the symbol intervals [lows[i], highs[i]) (of 2^16), in order."""
    w = _BitWriter()
    low, high, pending = 0, 0xFFFFFFFF, 0
    for c_low, c_high in zip(lows, highs):
        span = high - low + 1
        high = ((low - 1) + ((span * int(c_high)) >> PRECISION)) % _TOP
        low = (low + ((span * int(c_low)) >> PRECISION)) % _TOP
        while True:
            if high < 0x80000000:
                w.put_with_pending(0, pending)
                pending = 0
                low = (low << 1) % _TOP
                high = ((high << 1) | 1) % _TOP
            elif low >= 0x80000000:
                w.put_with_pending(1, pending)
                pending = 0
                low = (low << 1) % _TOP
                high = ((high << 1) | 1) % _TOP
            elif low >= 0x40000000 and high < 0xC0000000:
                pending += 1
                low = ((low << 1) % _TOP) & 0x7FFFFFFF
                high = ((high << 1) % _TOP) | 0x80000001
            else:
                break
    pending += 1
    w.put_with_pending(0 if low < 0x40000000 else 1, pending)
    w.flush()
    return bytes(w.out)


def encode_int16_normalized_cdf(cdf_u16: np.ndarray, sym: np.ndarray) -> bytes:
    """cdf [N, Lp] uint16 (rows in symbol order), sym [N] -> bytes."""
    cdf_u16 = np.asarray(cdf_u16).reshape(-1, np.asarray(cdf_u16).shape[-1])
    sym = np.asarray(sym).reshape(-1)
    b = [_bounds(cdf_u16[i], int(sym[i])) for i in range(len(sym))]
    return encode_bounds([x[0] for x in b], [x[1] for x in b])


class _BitReader:
    def __init__(self, data: bytes):
        self.data = data
        self.pos = 0
        self.cache = 0
        self.bits = 0

    def get(self, value):
        if self.bits == 0:
            if self.pos == len(self.data):
                return (value << 1) % _TOP
            self.cache = self.data[self.pos]
            self.pos += 1
            self.bits = 8
        value = ((value << 1) | ((self.cache >> (self.bits - 1)) & 1)) % _TOP
        self.bits -= 1
        return value


def _binsearch(row, target, max_sym):
    left, right = 0, max_sym + 1
    while left + 1 < right:
        m = (left + right) // 2
        v = int(row[m])
        if v < target:
            left = m
        elif v > target:
            right = m
        else:
            return m
    return left


def decode_int16_normalized_cdf(cdf_u16: np.ndarray, data: bytes, rows=None, n=None) -> np.ndarray:
    """Decode N symbols; element i uses CDF row rows[i] (default: row i)."""
    cdf_u16 = np.asarray(cdf_u16)
    cdf_u16 = cdf_u16.reshape(-1, cdf_u16.shape[-1])
    Lp = cdf_u16.shape[-1]
    max_symbol = Lp - 2
    N = len(rows) if rows is not None else (cdf_u16.shape[0] if n is None else n)
    r = _BitReader(data)
    low, high, value = 0, 0xFFFFFFFF, 0
    for _ in range(32):
        value = r.get(value)
    out = np.zeros(N, np.int16)
    for i in range(N):
        row = cdf_u16[rows[i] if rows is not None else i]
        span = high - low + 1
        count = (((value - low + 1) * (1 << PRECISION) - 1) // span) & 0xFFFF
        s = _binsearch(row, count, max_symbol)
        out[i] = s
        if i == N - 1:
            break
        c_low, c_high = _bounds(row, s)
        high = ((low - 1) + ((span * c_high) >> PRECISION)) % _TOP
        low = (low + ((span * c_low) >> PRECISION)) % _TOP
        while True:
            if low >= 0x80000000 or high < 0x80000000:
                low = (low << 1) % _TOP
                high = ((high << 1) | 1) % _TOP
                value = r.get(value)
            elif low >= 0x40000000 and high < 0xC0000000:
                low = ((low << 1) % _TOP) & 0x7FFFFFFF
                high = ((high << 1) % _TOP) | 0x80000001
                value = (value - 0x40000000) % _TOP
                value = r.get(value)
            else:
                break
    return out


def encode_float_cdf(cdf_float, sym, needs_normalization=True, check_input_bounds=False) -> bytes:
    if check_input_bounds:
        check_bounds(cdf_float, sym)
    return encode_int16_normalized_cdf(normalize(cdf_float, needs_normalization), sym)


def decode_float_cdf(cdf_float, data, needs_normalization=True) -> np.ndarray:
    return decode_int16_normalized_cdf(normalize(cdf_float, needs_normalization), data)


# ---- DVC's CDF rows (net.py:123-195), float32 as torch computes them
def laplace_cdf_rows(sigma: np.ndarray, mxrange: int = 150) -> np.ndarray:
    """Laplace(0, clamp(sigma, 1e-5, 1e10)).cdf(i - 0.5), i in [-mxrange, mxrange): [N, 2*mxrange]
    (torch.distributions.Laplace.cdf: 0.5 - 0.5 * sign(v) * expm1(-|v| / scale))."""
    s = np.clip(np.asarray(sigma, np.float32).reshape(-1, 1), np.float32(1e-5), np.float32(1e10))
    v = (np.arange(-mxrange, mxrange, dtype=np.float32) - np.float32(0.5))[None, :]
    return (np.float32(0.5) - np.float32(0.5) * np.sign(v) * np.expm1(-np.abs(v) / s)).astype(np.float32)
