"""torchac-compatible float-CDF arithmetic coder, the coder behind DVC's
``calrealbits`` mode (``DVC/net.py:123-138`` feature under Laplace(0, sigma), ``:155-168`` z and
``:183-195`` mv under the BitEstimator CDFs; 2*mxrange = 300 bins per element, one byte string per
latent tensor, elements in NCHW order, symbol = round(x) + mxrange).

API mirror of torchac (third-party, absent here; restated in oracle/torchac_ref.py, which these
functions match byte for byte -- parity unpinned against torchac itself, see that module):
``encode_float_cdf(cdf_float, sym, needs_normalization=True, check_input_bounds=False) -> bytes``,
``decode_float_cdf(cdf_float, byte_stream, needs_normalization=True) -> int16 tensor`` and the
``*_int16_normalized_cdf`` pair. The CDF work runs on the GPU (csrc/fvc_torchac.hip); the
sequential coder runs in native host code on the device-computed bounds / rows (the format is one
chain per tensor: a CPU core is ~50x faster at it than any single GPU lane).

DVC helpers take the codec's NHWC latents directly: ``laplace_encode`` / ``laplace_decode``
(feature, sigma) and ``bitest_encode`` / ``bitest_decode`` (z, mv with BitEstimator params
[11, C]); the decoders return the symbol values (round(x)) as float NHWC tensors.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from . import kernels as K

PRECISION = 16


def _dev(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_cuda else t.to(torch.device("cuda", torch.cuda.current_device()))


def _host_encode(lo: torch.Tensor, hi: torch.Tensor, status: torch.Tensor | None = None) -> bytes:
    if status is not None and int(status.item()) != 0:
        raise ValueError("symbol outside [0, Lp - 2] (torchac check_input_bounds)")
    n = lo.numel()
    lo_h = lo.cpu().numpy()
    hi_h = hi.cpu().numpy()
    cap = _lib.load().fvc_torchac_max_bytes(n)
    out = np.empty(max(cap, 1), np.uint8)
    out_len = ctypes.c_size_t(0)
    _lib.call("fvc_torchac_encode", lo_h.ctypes.data, hi_h.ctypes.data, n, out.ctypes.data, cap,
              ctypes.addressof(out_len))
    return out[:out_len.value].tobytes()


def _host_decode(rows_u16: np.ndarray, Lp: int, row_index: np.ndarray | None, n: int, data: bytes) -> np.ndarray:
    rows_u16 = np.ascontiguousarray(rows_u16, np.uint16)
    nrows = rows_u16.size // Lp
    sym = np.empty(max(n, 1), np.int16)
    buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
    ri = None if row_index is None else np.ascontiguousarray(row_index, np.int32)
    _lib.call("fvc_torchac_decode", rows_u16.ctypes.data, Lp, None if ri is None else ri.ctypes.data, nrows, n,
              buf.ctypes.data, len(data), sym.ctypes.data)
    return sym[:n]


# ---------------------------------------------------------------- torchac API mirror
def _normalize(cdf_float: torch.Tensor, needs_normalization: bool) -> torch.Tensor:
    cdf = _dev(cdf_float).contiguous().float()
    Lp = cdf.shape[-1]
    out = torch.empty(cdf.shape, dtype=torch.int16, device=cdf.device)
    _lib.call("fvc_torchac_normalize", cdf.data_ptr(), cdf.numel() // Lp, Lp, int(needs_normalization),
              out.data_ptr(), K.stream_handle(cdf.device))
    return out


def _check_bounds(cdf_float: torch.Tensor, sym: torch.Tensor):
    Lp = cdf_float.shape[-1]
    if float(cdf_float.min()) < 0:
        raise ValueError("cdf_float.min() < 0")
    if float(cdf_float.max()) > 1:
        raise ValueError("cdf_float.max() > 1")
    if sym.numel() and (int(sym.max()) >= Lp - 1 or int(sym.min()) < 0):
        raise ValueError("symbol out of [0, Lp - 2]")


def encode_int16_normalized_cdf(cdf_int16: torch.Tensor, sym: torch.Tensor) -> bytes:
    """cdf [..., Lp] int16 (torchac's normalised CDF), sym [...] int16 -> bytes."""
    rows = _dev(cdf_int16).contiguous()
    Lp = rows.shape[-1]
    s = sym.to(rows.device, torch.int16).contiguous()
    if s.numel() != rows.numel() // Lp:
        raise ValueError("sym must have cdf.shape[:-1] elements")
    n = s.numel()
    lo = torch.empty(n, dtype=torch.int32, device=rows.device)
    hi = torch.empty_like(lo)
    status = torch.zeros(1, dtype=torch.int32, device=rows.device)
    if n:
        _lib.call("fvc_torchac_rows_bounds", rows.data_ptr(), s.data_ptr(), n, Lp, lo.data_ptr(), hi.data_ptr(),
                  status.data_ptr(), K.stream_handle(rows.device))
    return _host_encode(lo, hi, status)


def decode_int16_normalized_cdf(cdf_int16: torch.Tensor, byte_stream: bytes) -> torch.Tensor:
    Lp = cdf_int16.shape[-1]
    rows = cdf_int16.contiguous().cpu().numpy().view(np.uint16)
    sym = _host_decode(rows, Lp, None, rows.size // Lp, byte_stream)
    return torch.from_numpy(sym.copy()).reshape(cdf_int16.shape[:-1]).to(cdf_int16.device)


def encode_float_cdf(cdf_float: torch.Tensor, sym: torch.Tensor, needs_normalization=True,
                     check_input_bounds=False) -> bytes:
    if check_input_bounds:
        _check_bounds(cdf_float, sym)
    return encode_int16_normalized_cdf(_normalize(cdf_float, needs_normalization), sym)


def decode_float_cdf(cdf_float: torch.Tensor, byte_stream: bytes, needs_normalization=True) -> torch.Tensor:
    out = decode_int16_normalized_cdf(_normalize(cdf_float, needs_normalization), byte_stream)
    return out.to(cdf_float.device)


# ---------------------------------------------------------------- DVC calrealbits helpers
def _latent_dims(x: torch.Tensor, c: int):
    K._chk(x, name="latent")
    B, H, W, cp = x.shape
    if c > cp:
        raise ValueError("channel count exceeds the padded latent")
    return B, H, W, cp


def laplace_encode(x: torch.Tensor, sigma: torch.Tensor, c: int, mxrange: int = 150) -> bytes:
    """torchac.encode_float_cdf(Laplace(0, sigma).cdf rows, round(x) + mxrange) of an NHWC latent
    (net.py:123-132); raises ValueError as check_input_bounds does when |round(x)| > mxrange - 2."""
    B, H, W, cp = _latent_dims(x, c)
    K._chk(sigma, x.shape, name="sigma")
    n = B * c * H * W
    lo = torch.empty(n, dtype=torch.int32, device=x.device)
    hi = torch.empty_like(lo)
    status = torch.zeros(1, dtype=torch.int32, device=x.device)
    _lib.call("fvc_torchac_laplace_bounds", x.data_ptr(), sigma.data_ptr(), B, H, W, c, cp, mxrange, lo.data_ptr(),
              hi.data_ptr(), status.data_ptr(), K.stream_handle(x.device))
    return _host_encode(lo, hi, status)


def laplace_decode(sigma: torch.Tensor, c: int, data: bytes, mxrange: int = 150) -> torch.Tensor:
    """Inverse of laplace_encode: the symbol values (round(x)) as an NHWC float tensor like sigma."""
    B, H, W, cp = _latent_dims(sigma, c)
    Lp = 2 * mxrange
    n = B * c * H * W
    rows = torch.empty((n, Lp), dtype=torch.int16, device=sigma.device)
    _lib.call("fvc_torchac_laplace_rows", sigma.data_ptr(), B, H, W, c, cp, mxrange, rows.data_ptr(),
              K.stream_handle(sigma.device))
    sym = _host_decode(rows.cpu().numpy().view(np.uint16), Lp, None, n, data)
    return _to_nhwc(sym, B, c, H, W, cp, mxrange, sigma.device)


def _bitest_table(params: torch.Tensor, c: int, mxrange: int) -> torch.Tensor:
    Lp = 2 * mxrange
    table = torch.empty((c, Lp), dtype=torch.int16, device=params.device)
    _lib.call("fvc_torchac_bitest_table", params.contiguous().data_ptr(), c, mxrange, table.data_ptr(),
              K.stream_handle(params.device))
    return table


def bitest_encode(x: torch.Tensor, params: torch.Tensor, c: int, mxrange: int = 150) -> bytes:
    """torchac.encode_float_cdf of an NHWC latent under the per-channel BitEstimator CDF rows
    (net.py:155-162, 183-190)."""
    B, H, W, cp = _latent_dims(x, c)
    table = _bitest_table(params, c, mxrange)
    n = B * c * H * W
    lo = torch.empty(n, dtype=torch.int32, device=x.device)
    hi = torch.empty_like(lo)
    status = torch.zeros(1, dtype=torch.int32, device=x.device)
    _lib.call("fvc_torchac_table_bounds", x.data_ptr(), table.data_ptr(), B, H, W, c, cp, mxrange, lo.data_ptr(),
              hi.data_ptr(), status.data_ptr(), K.stream_handle(x.device))
    return _host_encode(lo, hi, status)


def bitest_decode(params: torch.Tensor, shape, c: int, data: bytes, mxrange: int = 150, cp: int | None = None):
    """Inverse of bitest_encode for a latent of NHWC shape (B, H, W, cp)."""
    B, H, W = shape[0], shape[1], shape[2]
    cp = shape[3] if cp is None and len(shape) > 3 else (cp or c)
    Lp = 2 * mxrange
    table = _bitest_table(params, c, mxrange).cpu().numpy().view(np.uint16)
    n = B * c * H * W
    row_index = ((np.arange(n, dtype=np.int64) // (H * W)) % c).astype(np.int32)
    sym = _host_decode(table, Lp, row_index, n, data)
    return _to_nhwc(sym, B, c, H, W, cp, mxrange, params.device)


def _to_nhwc(sym: np.ndarray, B, c, H, W, cp, mxrange, device) -> torch.Tensor:
    v = torch.from_numpy(sym.astype(np.float32) - mxrange).reshape(B, c, H, W).permute(0, 2, 3, 1)
    out = torch.zeros((B, H, W, cp), dtype=torch.float32)
    out[..., :c] = v
    return out.to(device)
