"""Typed wrappers over the libfvc C-ABI for torch device tensors.

Tensors are passed by raw device pointer (``data_ptr``) together with their sizes and the
current HIP stream; every wrapper checks shapes/dtypes/contiguity before launching, since the
kernels trust their arguments (an out-of-bounds launch can fault the whole GPU).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

from . import _lib, profiling

IN_NONE, IN_RELU, IN_ABS, IN_ROUND = 0, 1, 2, 3
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2
POST_NONE, POST_EXP = 0, 1


def cp4(c: int) -> int:
    return (c + 3) // 4 * 4


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def _chk(t, shape=None, dtype=torch.float32, name="tensor"):
    if t is None:
        return
    if not t.is_cuda:
        raise ValueError(f"{name}: libfvc kernels need a device tensor (got {t.device})")
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")


def empty_nhwc(b, h, w, c, like):
    return torch.empty((b, h, w, cp4(c)), dtype=torch.float32, device=like.device)


# ------------------------------------------------------------------ layout
def nchw_to_nhwc(x: torch.Tensor, cp: int | None = None) -> torch.Tensor:
    B, C, H, W = x.shape
    cp = cp or cp4(C)
    _chk(x, name="x")
    y = torch.empty((B, H, W, cp), dtype=torch.float32, device=x.device)
    _lib.call("fvc_nchw_to_nhwc", x.data_ptr(), y.data_ptr(), B, C, H, W, cp, stream_handle())
    return y


def nhwc_to_nchw(x: torch.Tensor, c: int, clamp01: bool = False) -> torch.Tensor:
    B, H, W, cp = x.shape
    _chk(x, name="x")
    y = torch.empty((B, c, H, W), dtype=torch.float32, device=x.device)
    _lib.call("fvc_nhwc_to_nchw", x.data_ptr(), y.data_ptr(), B, c, H, W, cp, int(clamp01), stream_handle())
    return y


def avgpool2(x: torch.Tensor) -> torch.Tensor:
    B, H, W, cp = x.shape
    _chk(x, name="x")
    y = torch.empty((B, H // 2, W // 2, cp), dtype=torch.float32, device=x.device)
    profiling.timed_hbm("avgpool2", 4 * (x.numel() + y.numel()), lambda: _lib.call(
        "fvc_avgpool2_nhwc", x.data_ptr(), y.data_ptr(), B, H, W, cp, stream_handle()))
    return y


def warp(im: torch.Tensor, flow: torch.Tensor) -> torch.Tensor:
    B, H, W, cp = im.shape
    _chk(im, name="im")
    _chk(flow, (B, H, W, 4), name="flow")
    y = torch.empty_like(im)
    _lib.call("fvc_warp_nhwc", im.data_ptr(), flow.data_ptr(), y.data_ptr(), B, H, W, cp, stream_handle())
    return y


def upsample2x_add(src, skip=None, align_corners=True, scale=1.0):
    B, h, w, cp = src.shape
    _chk(src, name="src")
    _chk(skip, (B, 2 * h, 2 * w, cp), name="skip")
    y = torch.empty((B, 2 * h, 2 * w, cp), dtype=torch.float32, device=src.device)
    nb = 4 * (src.numel() + y.numel() + (skip.numel() if skip is not None else 0))
    profiling.timed_hbm("upsample2x_add", nb, lambda: _lib.call(
        "fvc_upsample2x_add_nhwc", src.data_ptr(), _ptr(skip), y.data_ptr(), B, h, w, cp, int(align_corners),
        float(scale), stream_handle()))
    return y


def spynet_assemble(im1, im2, flow_prev):
    B, H, W, _ = im1.shape
    _chk(im1, (B, H, W, 4), name="im1")
    _chk(im2, (B, H, W, 4), name="im2")
    _chk(flow_prev, (B, H // 2, W // 2, 4), name="flow_prev")
    flow_up = torch.empty((B, H, W, 4), dtype=torch.float32, device=im1.device)
    x8 = torch.empty((B, H, W, 8), dtype=torch.float32, device=im1.device)
    nb = 4 * (im1.numel() + im2.numel() + (flow_prev.numel() if flow_prev is not None else 0) + flow_up.numel()
              + x8.numel())
    profiling.timed_hbm("spynet_assemble (warp)", nb, lambda: _lib.call(
        "fvc_spynet_assemble", im1.data_ptr(), im2.data_ptr(), _ptr(flow_prev), flow_up.data_ptr(), x8.data_ptr(), B,
        H, W, stream_handle()))
    return flow_up, x8


def mc_assemble(ref, mv):
    B, H, W, _ = ref.shape
    _chk(ref, (B, H, W, 4), name="ref")
    _chk(mv, (B, H, W, 4), name="mv")
    warpframe = torch.empty((B, H, W, 4), dtype=torch.float32, device=ref.device)
    x8 = torch.empty((B, H, W, 8), dtype=torch.float32, device=ref.device)
    nb = 4 * (ref.numel() + mv.numel() + warpframe.numel() + x8.numel())
    profiling.timed_hbm("mc_assemble (warp)", nb, lambda: _lib.call(
        "fvc_mc_assemble", ref.data_ptr(), mv.data_ptr(), warpframe.data_ptr(), x8.data_ptr(), B, H, W,
        stream_handle()))
    return warpframe, x8


def sub(a, b):
    _chk(a, name="a")
    _chk(b, a.shape, name="b")
    y = torch.empty_like(a)
    _lib.call("fvc_sub_f32", a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), stream_handle())
    return y


def gdn(x, beta, gamma, inverse):
    B, H, W, C = x.shape
    _chk(x, name="x")
    _chk(beta, (C,), name="beta")
    _chk(gamma, (C, C), name="gamma")
    y = torch.empty_like(x)
    profiling.timed_hbm("gdn", 4 * (x.numel() + y.numel()), lambda: _lib.call(
        "fvc_gdn_nhwc", x.data_ptr(), y.data_ptr(), beta.data_ptr(), gamma.data_ptr(), B, H, W, C, int(inverse),
        stream_handle()))
    return y


# ------------------------------------------------------------------ conv
PRECISIONS = ("x3", "f32")
_STATE = {"precision": None, "cu_reserve": 0, "rans_spb": 16}


def conv_precision() -> str:
    """'x3' (default): split-precision fp16 matrix-core kernel (fvc_conv_x3.hip) wherever the
    layer supports it; 'f32': the fp32-MFMA kernel everywhere (FVC_CONV_PRECISION=f32, or inside
    ``with precision('f32')``, which the codec uses to recompute a frame whose activations left
    the split-precision range)."""
    p = _STATE["precision"] or os.environ.get("FVC_CONV_PRECISION", "x3")
    if p not in PRECISIONS:
        raise ValueError(f"FVC_CONV_PRECISION must be x3 or f32, got {p!r}")
    return p


@contextlib.contextmanager
def precision(p: str | None):
    """Override the conv precision for convs packed / run inside the block (None: no override)."""
    if p is not None and p not in PRECISIONS:
        raise ValueError(p)
    old = _STATE["precision"]
    _STATE["precision"] = p if p is not None else old
    try:
        yield
    finally:
        _STATE["precision"] = old


@contextlib.contextmanager
def cu_reserve(n: int):
    """CUs the split-precision conv's persistent grid leaves to other streams' kernels, for the
    convs launched inside the block (gop.py's pipeline)."""
    old = _STATE["cu_reserve"]
    _STATE["cu_reserve"] = int(n)
    try:
        yield
    finally:
        _STATE["cu_reserve"] = old


def rans_streams_per_block() -> int:
    """Streams per rANS decode block for decodes launched now: 16 by default (each block's LDS
    table cache then holds all its streams' tables: lowest latency), 64 inside
    ``rans_throughput()`` (the GOP pipeline: fewer, fuller blocks leave CUs to the concurrent
    convs; MI355X r2: serial decode 2.47 -> 1.81 ms per P-frame at 16, pipelined bench 58.0 at 64
    vs 55.8 at 16)."""
    return _STATE["rans_spb"]


@contextlib.contextmanager
def rans_throughput(on: bool = True):
    old = _STATE["rans_spb"]
    _STATE["rans_spb"] = int(os.environ.get("FVC_RANS_SPB_PIPE", "64")) if on else old
    try:
        yield
    finally:
        _STATE["rans_spb"] = old


_OVF = {}
_SCHED = {}
SCHED_LEN = 4096


def sched_scratch(device=None) -> torch.Tensor:
    """The x3 conv's dynamic-schedule counters (device int32[SCHED_LEN], zero between launches) of
    the current stream of device: launches on one stream are ordered, so they can share it."""
    st = torch.cuda.current_stream(device)
    key = (str(st.device), st.cuda_stream)
    if key not in _SCHED:
        _SCHED[key] = torch.zeros(SCHED_LEN, dtype=torch.int32, device=st.device)
    return _SCHED[key]


def overflow_flag(device=None) -> torch.Tensor:
    """The split-precision overflow flag (device int32[1]) of the current stream of device: every
    x3 conv launched on that stream ORs 1 into it if it staged |v| >= 65000 (or a non-finite v)."""
    st = torch.cuda.current_stream(device)
    key = (str(st.device), st.cuda_stream)
    if key not in _OVF:
        _OVF[key] = torch.zeros(1, dtype=torch.int32, device=st.device)
    return _OVF[key]


class OverflowProbe:
    """Non-blocking read of a stream's overflow flag: copies it to pinned host memory behind the
    work already queued; ``result()`` waits for that copy only (not the device)."""

    def __init__(self, device=None, reset=True):
        flag = overflow_flag(device)
        self.host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        self.host.copy_(flag, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record()
        if reset:
            flag.zero_()

    def ready(self) -> bool:
        return self.event.query()

    def result(self) -> bool:
        self.event.synchronize()
        return bool(self.host.item())


def x3_dispatches(batch, y_image_bytes, res_image_bytes=0):
    """Kernel dispatches of one split-precision direct / all-classes conv call: the C-ABI halves the
    batch recursively while the output (or residual) reaches 4 GB (32-bit buffer offsets,
    fvc_conv_x3.hip run_x3), so the timer counts dispatches as rocprofv3 does. The Winograd kernel
    never splits."""
    split_at = int(os.environ.get("FVC_X3_SPLIT_BYTES", "0") or 0) or (1 << 32) - 4096

    def n(b):
        if b > 1 and (b * y_image_bytes >= split_at or b * res_image_bytes >= split_at):
            return n(b // 2) + n(b - b // 2)
        return 1
    return n(batch)


# every environment switch the split-precision conv sources read (fvc_conv_x3.hip, fvc_deconv_x3.hip,
# fvc_conv_wino.hip): a pack's layout id is re-queried only when one of them changes
_LAYOUT_ENV = ("FVC_DX", "FVC_DX_PAIR", "FVC_X3_BPC", "FVC_X3_CC", "FVC_X3_CIN4", "FVC_X3_DYN", "FVC_X3_PRIO",
               "FVC_X3_PT", "FVC_X3_RESERVE", "FVC_X3_SMALLN", "FVC_X3_SPLIT_BYTES", "FVC_X3_WG", "FVC_X3_WL",
               "FVC_X3_WM", "FVC_X3_WN", "FVC_X3_XCD")


def _layout_env():
    get = os.environ.get
    return tuple(get(k) for k in _LAYOUT_ENV)


class PackedConv:
    """A conv / transposed conv with weights packed once for its HIP kernel: the split-precision
    fp16 x3 kernel where supported (cin padded to a multiple of 8, cout > 4), else fp32 MFMA /
    the small-N VALU kernel."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor, ksize: int, stride: int, transposed: bool,
                 device, precision: str | None = None):
        lib = _lib.load()
        w = weight.detach().to("cpu", torch.float32).contiguous()
        if transposed:
            cin, cout = w.shape[0], w.shape[1]
        else:
            cout, cin = w.shape[0], w.shape[1]
        precision = precision or conv_precision()
        self.cin, self.cout, self.ksize, self.stride, self.transposed = cin, cout, ksize, stride, transposed
        # cout <= 4 with a wide input (mvDecoder deconv8, 128->2 3x3): N padded to a 32-wide MFMA
        # tile wastes 16x, so the layer can run as a 1x1 x3 GEMM to N' = k*k*cout tap partials per
        # input pixel + the LDS-tiled fvc_tap_gather_nhwc (net.py normally fuses the partial GEMM
        # into the producer instead: conv_then_tap, for deconv8 and Warp_net conv6). resDecoder
        # deconv4 (64->3 5x5 s2) stays direct: 1x1 GEMM 0.57 + gather 0.45 ms vs 0.86 ms direct
        # per 4-frame launch (MI355X, r2). FVC_TAPSUM=0 / 2 disables / forces the tap path for
        # every eligible layer.
        self.tap = None
        self.wino = self.dx = self.wino128 = False
        tapsum = os.environ.get("FVC_TAPSUM", "1")
        if (precision == "x3" and cout <= 4 and ksize in (3, 5) and stride == (2 if transposed else 1)
                and cp4(cin) % 8 == 0 and tapsum != "0" and (tapsum == "2" or (cin >= 128 and not transposed))):
            nt = ksize * ksize
            wt = w.permute(2, 3, 1, 0) if transposed else w.permute(2, 3, 0, 1)  # [ky][kx][co][ci]
            self.tap = PackedConv(wt.reshape(nt * cout, cin, 1, 1).contiguous(), torch.zeros(nt * cout), 1, 1,
                                  False, device, precision="x3")
            self.x3 = self.tap.x3
            self.bias = bias.detach().to(device, torch.float32).contiguous()
            return
        self.x3 = precision == "x3" and bool(lib.fvc_conv_x3_supported(cin, cout, ksize, stride, int(transposed)))
        # 64 -> 64 3x3 stride-1 layers (Warp_net's ResBlocks): the Winograd F(2x2,3x3) split-precision
        # kernel (fvc_conv_wino.hip; 2.25x fewer MFMAs); the direct x3 pack stays for the fused tap
        # epilogue. FVC_WINO=0 disables it (A/B, tests).
        self.wino = (self.x3 and os.environ.get("FVC_WINO", "1") != "0" and
                     bool(lib.fvc_conv_wino_supported(cin, cout, ksize, stride, int(transposed))))
        if self.wino:
            upack = torch.empty(lib.fvc_conv_wino_wpack_bytes() // 2, dtype=torch.float16)
            uosc = ctypes.c_float(0.0)
            _lib.call("fvc_conv_wino_pack_weight", w.data_ptr(), upack.data_ptr(), ctypes.addressof(uosc))
            self.upack, self.uosc = upack.to(device), float(uosc.value)
        # 128 -> 128 3x3 stride-1 layers (MV stacks): four 64 -> 64 Winograd quarters of the same
        # kernel on 128-channel pixels (fvc_conv2d_nhwc_wino128); FVC_WINO128=0 keeps them direct
        self.wino128 = (self.x3 and os.environ.get("FVC_WINO128", "1") != "0" and
                        bool(lib.fvc_conv_wino128_supported(cin, cout, ksize, stride, int(transposed))))
        if self.wino128:
            q = torch.empty(lib.fvc_conv_wino128_wpack_bytes() // 2, dtype=torch.float16)
            self.osc4 = (ctypes.c_float * 4)()
            _lib.call("fvc_conv_wino128_pack_weight", w.data_ptr(), q.data_ptr(), ctypes.addressof(self.osc4))
            self.upack128 = q.to(device)
        # SpyNet's 7x7 stride-1 32->64 / 64->32 / 32->16 layers: Winograd-rows F(2,7) split-precision
        # kernel (fvc_conv_wr7.hip; 1.75x fewer MFMAs), as launches of 32 input x 16 * nt output
        # channels: (ci0, co0, nt, mode, upack, osc); a 64-channel input's second half adds the first
        # half's partial sum (mode 1 then 2). FVC_WR7=0 keeps the direct x3 kernel (A/B, tests).
        self.wr7 = []
        if (self.x3 and os.environ.get("FVC_WR7", "1") != "0" and
                bool(lib.fvc_conv_wr7_supported(cin, cout, ksize, stride, int(transposed)))):
            nt = 1 if cout == 16 else 2
            for co0 in range(0, cout, 16 * nt):
                for ci0 in range(0, cin, 32):
                    mode = 0 if cin == 32 else (1 if ci0 == 0 else 2)
                    up = torch.empty(lib.fvc_conv_wr7_wpack_bytes(nt) // 2, dtype=torch.float16)
                    uo = ctypes.c_float(0.0)
                    _lib.call("fvc_conv_wr7_pack_weight", w.data_ptr(), cin, cout, ci0, co0, nt, up.data_ptr(),
                              ctypes.addressof(uo))
                    self.wr7.append((ci0, co0, nt, mode, up.to(device), float(uo.value)))
        # small-input stems (cin <= 8 on a 4- or 8-float pixel, cout 64 / 128, 3x3 s1 / s2, 5x5 s2:
        # Warp_net feature_ext, mvEncoder conv1, resEncoder conv1): the streaming split-precision
        # kernel (fvc_conv_stem.hip); FVC_STEM=0 keeps the direct x3 kernel (A/B, tests)
        self.stem = None
        if (self.x3 and os.environ.get("FVC_STEM", "1") != "0" and
                bool(lib.fvc_conv_stem_supported(cin, cout, ksize, stride, int(transposed)))):
            sp = torch.empty(lib.fvc_conv_stem_wpack_bytes(cin, cout, ksize) // 2, dtype=torch.float16)
            so = ctypes.c_float(0.0)
            _lib.call("fvc_conv_stem_pack_weight", w.data_ptr(), cin, cout, ksize, sp.data_ptr(), ctypes.addressof(so))
            self.stem = (sp.to(device), float(so.value))
        # stride-2 transposed layers on the all-classes kernel (fvc_deconv_x3.hip, conv_dx_kernel)
        self.dx = self.x3 and transposed and bool(lib.fvc_deconv_x3_all_classes(cin, cout, ksize, stride))
        if self.x3:
            nbytes = lib.fvc_conv_x3_wpack_bytes(cin, cout, ksize, stride, int(transposed))
            packed = torch.empty(nbytes // 2, dtype=torch.float16)
            osc = ctypes.c_float(0.0)
            _lib.call("fvc_conv_x3_pack_weight", w.data_ptr(), packed.data_ptr(), ctypes.addressof(osc), cin, cout,
                      ksize, stride, int(transposed))
            self.osc = float(osc.value)
            self.layout = int(lib.fvc_conv_x3_layout_id(cin, cout, ksize, stride, int(transposed)))
        else:
            n = lib.fvc_conv_wpack_floats(cin, cout, ksize, stride, int(transposed))
            if n == 0:
                raise ValueError(f"unsupported conv geometry cin={cin} cout={cout} k={ksize} s={stride}")
            packed = torch.empty(n, dtype=torch.float32)
            _lib.call("fvc_conv_pack_weight", w.data_ptr(), packed.data_ptr(), cin, cout, ksize, stride,
                      int(transposed))
        self.wpack = packed.to(device)
        self.bias = bias.detach().to(device, torch.float32).contiguous()

    def _check_layout(self):
        """The pack's layout must be the one the launch will assume: FVC_DX / FVC_X3_PT / FVC_X3_CIN4 /
        FVC_X3_CC / FVC_X3_SMALLN are read by the C side at pack and at launch. The C
        query rebuilds the tap tables, so it runs again only when one of the switches the conv
        sources read has changed since this pack was last checked."""
        env = _layout_env()
        if env == getattr(self, "_layout_env", None):
            return
        now = int(_lib.load().fvc_conv_x3_layout_id(self.cin, self.cout, self.ksize, self.stride,
                                                      int(self.transposed)))
        if now != self.layout:
            raise _lib.FvcError("x3 weight pack was built under another layout configuration (an FVC_DX / "
                                "FVC_X3_* switch changed since packing); re-create the PackedConv")
        # cached only once the check has passed: a refused env must be refused on every call
        self._layout_env = env

    def out_hw(self, h, w):
        if self.transposed:
            return h * self.stride, w * self.stride
        return h // self.stride, w // self.stride

    def __call__(self, x, in_op=IN_NONE, act=ACT_NONE, post=POST_NONE, res=None, out=None):
        B, H, W, cp = x.shape
        if cp != cp4(self.cin):
            raise ValueError(f"conv input has {cp} channels, expected {cp4(self.cin)}")
        if (not self.transposed) and self.stride == 2 and (H % 2 or W % 2):
            raise ValueError("stride-2 conv needs even input size")
        _chk(x, name="x")
        ho, wo = self.out_hw(H, W)
        oshape = (B, ho, wo, cp4(self.cout))
        _chk(res, oshape, name="res")
        y = out if out is not None else torch.empty(oshape, dtype=torch.float32, device=x.device)
        _chk(y, oshape, name="y")
        if self.tap is not None:
            P = self.tap(x, in_op=in_op)  # timed (if a KernelTimer is active) as an x3 launch
            nb = 4 * (P.numel() + y.numel() * (2 if res is not None else 1))
            profiling.timed_hbm("tap_gather", nb, lambda: _lib.call(
                "fvc_tap_gather_nhwc", P.data_ptr(), P.shape[-1], self.bias.data_ptr(), _ptr(res), y.data_ptr(), B, H, W,
                self.cout, self.ksize, self.stride, int(self.transposed), act, post, stream_handle()))
            return y
        timer = profiling.active()
        if timer is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        wino = self.wino and in_op in (IN_NONE, IN_RELU) and post == POST_NONE
        # the quarters pay 4 launch tails: at 16 GOPs per launch 136x240 0.58 -> 0.62 ms, 272x480
        # 1.97 -> 1.72, 544x960 7.46 -> 6.08 (MI355X, profiles/r3/wino128). r3 measured a 100 K gate
        # bench-neutral against 200 K; r5 +0.8 % (profiles/r5/gate_100k); r6, with the faster
        # pixel-major Winograd rows, 200 K / 100 K / 30 K = 80.3 / 81.0-81.1 / 81.3-81.4 P-frames/s
        # (interleaved, profiles/r6/gate_wino128): images of >= 30 K pixels (544x960, 272x480 and
        # 136x240) take them. Gated per image, not per launch: a frame's result must not depend on
        # how many frames share its batch.
        w128 = (self.wino128 and in_op in (IN_NONE, IN_RELU) and post == POST_NONE and res is None and
                H * W >= int(os.environ.get("FVC_WINO128_MINPIX", "30000")))
        wr7 = bool(self.wr7) and in_op == IN_NONE and post == POST_NONE and res is None
        stem = self.stem is not None and in_op == IN_NONE and post == POST_NONE and res is None
        if stem:
            _lib.call("fvc_conv2d_nhwc_stem", x.data_ptr(), self.stem[0].data_ptr(), self.stem[1], self.bias.data_ptr(),
                      y.data_ptr(), B, H, W, self.cin, self.cout, self.ksize, self.stride, act,
                      overflow_flag(x.device).data_ptr(), stream_handle())
        elif wr7:
            xp, yp = cp4(self.cin), cp4(self.cout)
            for ci0, co0, nt, mode, up, uo in self.wr7:
                _lib.call("fvc_conv2d_nhwc_wr7", x.data_ptr() + 4 * ci0, xp, up.data_ptr(), nt, uo,
                          self.bias.data_ptr() + 4 * co0, y.data_ptr() + 4 * co0, yp, B, H, W, mode,
                          ACT_NONE if mode == 1 else act, _STATE["cu_reserve"], overflow_flag(x.device).data_ptr(),
                          sched_scratch(x.device).data_ptr(), SCHED_LEN, stream_handle())
        elif wino:
            _lib.call("fvc_conv2d_nhwc_wino", x.data_ptr(), self.upack.data_ptr(), self.uosc, self.bias.data_ptr(),
                      _ptr(res), y.data_ptr(), None, B, H, W, in_op, act, _STATE["cu_reserve"],
                      overflow_flag(x.device).data_ptr(), sched_scratch(x.device).data_ptr(), SCHED_LEN,
                      stream_handle())
        elif w128:
            _lib.call("fvc_conv2d_nhwc_wino128", x.data_ptr(), self.upack128.data_ptr(), ctypes.addressof(self.osc4),
                      self.bias.data_ptr(), y.data_ptr(), B, H, W, in_op, act, _STATE["cu_reserve"],
                      overflow_flag(x.device).data_ptr(), sched_scratch(x.device).data_ptr(), SCHED_LEN,
                      stream_handle())
            wino = True
        elif self.x3:
            self._check_layout()
            fn = "fvc_deconv2d_nhwc_x3" if self.transposed else "fvc_conv2d_nhwc_x3"
            _lib.call(fn, x.data_ptr(), self.wpack.data_ptr(), self.osc, self.bias.data_ptr(), _ptr(res),
                      y.data_ptr(), B, H, W, self.cin, self.cout, self.ksize, self.stride, in_op, act, post,
                      _STATE["cu_reserve"], overflow_flag(x.device).data_ptr(), sched_scratch(x.device).data_ptr(),
                      SCHED_LEN, stream_handle())
        else:
            fn = "fvc_deconv2d_nhwc_f32" if self.transposed else "fvc_conv2d_nhwc_f32"
            _lib.call(fn, x.data_ptr(), self.wpack.data_ptr(), self.bias.data_ptr(), _ptr(res), y.data_ptr(), B, H,
                      W, self.cin, self.cout, self.ksize, self.stride, in_op, act, post, stream_handle())
        if timer is not None:
            ev1.record()
            # algorithmic HBM bytes: input + weights + output (+ residual), each touched once
            nbytes = 4 * (x.numel() + y.numel() * (2 if res is not None else 1)) + self.wpack.numel() * \
                self.wpack.element_size()
            timer.records.append((ev0, ev1, profiling.conv_flops(self.cin, self.cout, self.ksize, self.stride,
                                                                 self.transposed, B, H, W),
                                  f"{'deconv' if self.transposed else 'conv'}{self.ksize}s{self.stride} "
                                  f"{self.cin}->{self.cout} @{H}x{W}{' stem' if stem else (' wr7' if wr7 else (' wino' if wino else (' dx' if self.dx else (' x3' if self.x3 else ''))))}"
                                  f"{' x4' if w128 else ''}{f' x{len(self.wr7)}' if wr7 and len(self.wr7) > 1 else ''}",
                                  self.x3, nbytes,
                                  "stem" if stem else ("wr7" if wr7 else ("wino" if wino else ("dx" if self.dx else ("x3" if self.x3 else "f32")))),
                                  len(self.wr7) if wr7 else 4 if w128 else (1 if stem or wino or not self.x3 else
                                                  x3_dispatches(B, 4 * y[0].numel(),
                                                                4 * res[0].numel() if res is not None else 0))))
        return y


    def pool_fusable(self) -> bool:
        return (self.x3 and self.tap is None and not self.transposed and self.stride == 1 and
                (self.wino or bool(_lib.load().fvc_conv_x3_pool_supported(self.cin, self.cout, self.ksize))))

    def call_pool(self, x, act=ACT_NONE, res=None):
        """(y, avg_pool2d(y, 2)) from one launch (fvc_conv2d_nhwc_x3_pool; in_op none, post none)."""
        if not self.pool_fusable():
            raise ValueError("conv not poolable in its epilogue")
        B, H, W, cp = x.shape
        if cp != cp4(self.cin):
            raise ValueError(f"conv input has {cp} channels, expected {cp4(self.cin)}")
        _chk(x, name="x")
        oshape = (B, H, W, cp4(self.cout))
        _chk(res, oshape, name="res")
        y = torch.empty(oshape, dtype=torch.float32, device=x.device)
        pool = torch.empty((B, H // 2, W // 2, cp4(self.cout)), dtype=torch.float32, device=x.device)
        timer = profiling.active()
        if timer is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        if self.wino:
            _lib.call("fvc_conv2d_nhwc_wino", x.data_ptr(), self.upack.data_ptr(), self.uosc, self.bias.data_ptr(),
                      _ptr(res), y.data_ptr(), pool.data_ptr(), B, H, W, IN_NONE, act, _STATE["cu_reserve"],
                      overflow_flag(x.device).data_ptr(), sched_scratch(x.device).data_ptr(), SCHED_LEN,
                      stream_handle())
        else:
            self._check_layout()
            _lib.call("fvc_conv2d_nhwc_x3_pool", x.data_ptr(), self.wpack.data_ptr(), self.osc, self.bias.data_ptr(),
                      _ptr(res), y.data_ptr(), pool.data_ptr(), B, H, W, self.cin, self.cout, self.ksize, act,
                      _STATE["cu_reserve"], overflow_flag(x.device).data_ptr(), sched_scratch(x.device).data_ptr(),
                      SCHED_LEN, stream_handle())
        if timer is not None:
            ev1.record()
            nbytes = 4 * (x.numel() + y.numel() * (2 if res is not None else 1) + pool.numel()) + \
                self.wpack.numel() * self.wpack.element_size()
            timer.records.append((ev0, ev1, profiling.conv_flops(self.cin, self.cout, self.ksize, 1, False, B, H, W),
                                  f"conv{self.ksize}s1 {self.cin}->{self.cout} @{H}x{W} {'wino' if self.wino else 'x3'} +pool",
                                  True, nbytes, "wino" if self.wino else "x3",
                                  1 if self.wino else x3_dispatches(B, 4 * y[0].numel(),
                                                                    4 * res[0].numel() if res is not None else 0)))
        return y, pool

    def up_fusable(self) -> bool:
        """The Winograd kernel can read skip + upsample(low) itself (fvc_conv2d_nhwc_wino_up);
        FVC_UP_FUSE=0 keeps the standalone upsample-add kernel (A/B, tests)."""
        return self.wino and self.tap is None and os.environ.get("FVC_UP_FUSE", "1") != "0"

    def call_up(self, skip, low, in_op=IN_NONE, act=ACT_NONE):
        """(conv(in_op(X)), X) with X = skip + upsample2x(low, bilinear, align_corners=True), X formed
        in the conv's staging and written once (Warp_net c3_u / c4_u, endecoder.py:288-293); X is
        bit-identical to upsample2x_add(low, skip)."""
        if not self.up_fusable():
            raise ValueError("conv cannot take the fused upsample-add input")
        B, H, W, cp = skip.shape
        if cp != cp4(self.cin) or H % 2 or W % 2:
            raise ValueError(f"fused upsample-add input: skip {tuple(skip.shape)}")
        _chk(skip, name="skip")
        _chk(low, (B, H // 2, W // 2, cp), name="low")
        xs = torch.empty_like(skip)
        y = torch.empty((B, H, W, cp4(self.cout)), dtype=torch.float32, device=skip.device)
        timer = profiling.active()
        if timer is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        _lib.call("fvc_conv2d_nhwc_wino_up", skip.data_ptr(), low.data_ptr(), xs.data_ptr(), self.upack.data_ptr(),
                  self.uosc, self.bias.data_ptr(), y.data_ptr(), B, H, W, in_op, act, _STATE["cu_reserve"],
                  overflow_flag(skip.device).data_ptr(), sched_scratch(skip.device).data_ptr(), SCHED_LEN,
                  stream_handle())
        if timer is not None:
            ev1.record()
            # skip + low read, X and y written (the standalone upsample-add's traffic plus the conv's)
            nbytes = 4 * (skip.numel() + low.numel() + xs.numel() + y.numel()) + \
                self.wpack.numel() * self.wpack.element_size()
            timer.records.append((ev0, ev1, profiling.conv_flops(self.cin, self.cout, self.ksize, 1, False, B, H, W),
                                  f"conv{self.ksize}s1 {self.cin}->{self.cout} @{H}x{W} wino +up2add",
                                  True, nbytes, "wino", 1))
        return y, xs

    def _wino_tap(self, tap: "TapConsumer") -> bool:
        """The Winograd kernel's tap epilogue (fvc_conv2d_nhwc_wino_tap) takes this pair;
        FVC_WINO_TAP=0 keeps it on the direct kernel's (A/B, tests)."""
        return (self.wino and tap.wino_wpack is not None and cp4(self.cout) == cp4(tap.cin) and
                os.environ.get("FVC_WINO_TAP", "1") != "0")

    def tap_fusable(self, tap: "TapConsumer") -> bool:
        """True if this conv can run with ``tap``'s 1x1 partial GEMM fused into its epilogue
        (split-precision path, its output feeds tap's layer, every output channel in one wave)."""
        return (self.x3 and self.tap is None and cp4(self.cout) == cp4(tap.cin) and
                (self._wino_tap(tap) or
                 bool(_lib.load().fvc_conv_x3_tap_supported(self.cin, self.cout, self.ksize, self.stride,
                                                             int(self.transposed), tap.pcp))))

    def call_tap(self, x, tap: "TapConsumer", act=ACT_NONE, res=None):
        """This conv (in_op none, act, res) fused with the first half of ``tap``'s layer: returns
        P [B, Ho, Wo, tap.pcp] = tap partials of the output (which itself is never written);
        ``tap.gather(P, ...)`` finishes the next layer (fvc_conv2d_nhwc_x3_tap)."""
        if not self.tap_fusable(tap):
            raise ValueError("conv / tap pair not fusable")
        B, H, W, cp = x.shape
        if cp != cp4(self.cin):
            raise ValueError(f"conv input has {cp} channels, expected {cp4(self.cin)}")
        if (not self.transposed) and self.stride == 2 and (H % 2 or W % 2):
            raise ValueError("stride-2 conv needs even input size")
        _chk(x, name="x")
        ho, wo = self.out_hw(H, W)
        _chk(res, (B, ho, wo, cp4(self.cout)), name="res")
        P = torch.empty((B, ho, wo, tap.pcp), dtype=torch.float32, device=x.device)
        timer = profiling.active()
        if timer is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        wino = self._wino_tap(tap)
        if wino:
            _lib.call("fvc_conv2d_nhwc_wino_tap", x.data_ptr(), self.upack.data_ptr(), self.uosc, self.bias.data_ptr(),
                      _ptr(res), P.data_ptr(), B, H, W, act, tap.wino_wpack.data_ptr(), tap.wino_osc, tap.pcp,
                      _STATE["cu_reserve"], overflow_flag(x.device).data_ptr(), sched_scratch(x.device).data_ptr(),
                      SCHED_LEN, stream_handle())
        else:
            self._check_layout()
            fn = "fvc_deconv2d_nhwc_x3_tap" if self.transposed else "fvc_conv2d_nhwc_x3_tap"
            _lib.call(fn, x.data_ptr(), self.wpack.data_ptr(), self.osc, self.bias.data_ptr(), _ptr(res), P.data_ptr(),
                      B, H, W, self.cin, self.cout, self.ksize, self.stride, act, tap.wpack.data_ptr(), tap.osc,
                      tap.pcp, _STATE["cu_reserve"], overflow_flag(x.device).data_ptr(),
                      sched_scratch(x.device).data_ptr(), SCHED_LEN, stream_handle())
        if timer is not None:
            ev1.record()
            # algorithmic work: this conv + the next layer's MACs (the partial GEMM does all of them)
            fl = (profiling.conv_flops(self.cin, self.cout, self.ksize, self.stride, self.transposed, B, H, W) +
                  2.0 * B * ho * wo * tap.cin * tap.np)
            nbytes = 4 * (x.numel() + P.numel() + (res.numel() if res is not None else 0)) + \
                self.wpack.numel() * self.wpack.element_size() + tap.wpack.numel() * tap.wpack.element_size()
            timer.records.append((ev0, ev1, fl, f"{'deconv' if self.transposed else 'conv'}{self.ksize}s{self.stride} "
                                  f"{self.cin}->{self.cout} @{H}x{W} {'wino' if wino else ('dx' if self.dx else 'x3')} "
                                  f"+tap{tap.ksize}x{tap.ksize}->{tap.cout}", True, nbytes,
                                  "wino" if wino else ("dx" if self.dx else "x3"),
                                  1 if wino else x3_dispatches(B, 4 * P[0].numel(),
                                                               4 * res[0].numel() if res is not None else 0)))
        return P


class TapConsumer:
    """A cout <= 4 conv (stride 1) / transposed conv (stride 2) in tap-partial form for fusion into
    its producer's epilogue: np = k*k*cout partial rows [t*cout + co][cin] (t = ky*k + kx), packed
    for the producer tile's accumulator order (fvc_x3_tap_pack_weight), plus the gather that sums
    them into the layer's output (fvc_tap_gather_nhwc). Used for synthesis_mv.py:41-43
    (deconv7 -> deconv8) and endecoder.py:278-279 (Warp_net conv5 -> conv6)."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor, ksize: int, stride: int, transposed: bool, device):
        lib = _lib.load()
        w = weight.detach().to("cpu", torch.float32).contiguous()
        cin, cout = (w.shape[0], w.shape[1]) if transposed else (w.shape[1], w.shape[0])
        if cout > 4 or ksize not in (3, 5) or stride != (2 if transposed else 1):
            raise ValueError("tap form needs cout <= 4, k 3/5, conv stride 1 or transposed stride 2")
        self.cin, self.cout, self.ksize, self.stride, self.transposed = cin, cout, ksize, stride, transposed
        nt = ksize * ksize
        wt = w.permute(2, 3, 1, 0) if transposed else w.permute(2, 3, 0, 1)  # [ky][kx][co][ci]
        wt = wt.reshape(nt * cout, cin).contiguous()
        self.np, self.pcp = nt * cout, cp4(nt * cout)
        nbytes = lib.fvc_x3_tap_wpack_bytes(self.np, cin)
        if nbytes == 0:
            raise ValueError(f"tap form unsupported: {self.np} partials from {cin} channels")
        packed = torch.empty(nbytes // 2, dtype=torch.float16)
        osc = ctypes.c_float(0.0)
        _lib.call("fvc_x3_tap_pack_weight", wt.data_ptr(), packed.data_ptr(), ctypes.addressof(osc), self.np, cin)
        self.osc = float(osc.value)
        self.wpack = packed.to(device)
        # the same rows for the Winograd producer's tap epilogue (64-channel producers only)
        self.wino_wpack, self.wino_osc = None, 0.0
        if cin == 64 and lib.fvc_wino_tap_wpack_bytes(self.np):
            wp = torch.empty(lib.fvc_wino_tap_wpack_bytes(self.np) // 2, dtype=torch.float16)
            wosc = ctypes.c_float(0.0)
            _lib.call("fvc_wino_tap_pack_weight", wt.data_ptr(), wp.data_ptr(), ctypes.addressof(wosc), self.np)
            self.wino_wpack, self.wino_osc = wp.to(device), float(wosc.value)
        self.bias = bias.detach().to(device, torch.float32).contiguous()

    def gather(self, P, act=ACT_NONE, post=POST_NONE, res=None):
        B, H, W, pcp = P.shape
        if pcp != self.pcp:
            raise ValueError(f"P has {pcp} channels, expected {self.pcp}")
        _chk(P, name="P")
        ho, wo = (H * self.stride, W * self.stride) if self.transposed else (H, W)
        y = torch.empty((B, ho, wo, cp4(self.cout)), dtype=torch.float32, device=P.device)
        _chk(res, y.shape, name="res")
        nb = 4 * (P.numel() + y.numel() * (2 if res is not None else 1))
        profiling.timed_hbm("tap_gather", nb, lambda: _lib.call(
            "fvc_tap_gather_nhwc", P.data_ptr(), pcp, self.bias.data_ptr(), _ptr(res), y.data_ptr(), B, H, W,
            self.cout, self.ksize, self.stride, int(self.transposed), act, post, stream_handle()))
        return y


class GdnTap:
    """GDN / IGDN (64 channels) fused with a cout <= 4 consumer conv / transposed conv in tap form
    (fvc_gdn_tap_nhwc: up to 4 tiles of 32 partials, so k*k*cout <= 128) + the gather: resDecoder
    igdn3 -> deconv4 (synthesis.py:26,57; 64 -> 3, 5x5 s2, 75 partials)."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor, ksize: int, stride: int, transposed: bool, device):
        lib = _lib.load()
        w = weight.detach().to("cpu", torch.float32).contiguous()
        cin, cout = (w.shape[0], w.shape[1]) if transposed else (w.shape[1], w.shape[0])
        nt = ksize * ksize
        if cin != 64 or cout > 4 or ksize not in (3, 5) or stride != (2 if transposed else 1) or nt * cout > 128:
            raise ValueError("GDN + tap form needs 64 input channels, cout <= 4, k 3/5, <= 128 partials")
        self.cin, self.cout, self.ksize, self.stride, self.transposed = cin, cout, ksize, stride, transposed
        wt = (w.permute(2, 3, 1, 0) if transposed else w.permute(2, 3, 0, 1)).reshape(nt * cout, cin).contiguous()
        self.np, self.pcp = nt * cout, cp4(nt * cout)
        self.ntiles = (self.np + 31) // 32
        packs, oscs = [], []
        for t in range(self.ntiles):
            rows = wt[32 * t: 32 * t + 32].contiguous()
            nbytes = lib.fvc_x3_tap_wpack_bytes(rows.shape[0], cin)
            pk = torch.empty(nbytes // 2, dtype=torch.float16)
            osc = ctypes.c_float(0.0)
            _lib.call("fvc_x3_tap_pack_weight", rows.data_ptr(), pk.data_ptr(), ctypes.addressof(osc), rows.shape[0], cin)
            packs.append(pk)
            oscs.append(float(osc.value))
        self.wpack = torch.cat(packs).to(device)
        self.osc = (ctypes.c_float * 4)(*(oscs + [0.0] * (4 - len(oscs))))
        self.bias = bias.detach().to(device, torch.float32).contiguous()

    def __call__(self, x, beta, gamma, inverse, act=ACT_NONE, post=POST_NONE, res=None):
        """consumer(gdn(x)) without writing gdn(x)."""
        B, H, W, C = x.shape
        if C != 64:
            raise ValueError("GDN + tap needs 64 channels")
        _chk(x, name="x")
        P = torch.empty((B, H, W, self.pcp), dtype=torch.float32, device=x.device)
        nb = 4 * (x.numel() + P.numel())
        profiling.timed_hbm("gdn+tap", nb, lambda: _lib.call(
            "fvc_gdn_tap_nhwc", x.data_ptr(), P.data_ptr(), beta.data_ptr(), gamma.data_ptr(), self.wpack.data_ptr(),
            ctypes.addressof(self.osc), self.ntiles, self.pcp, B, H, W, C, int(inverse),
            overflow_flag(x.device).data_ptr(), stream_handle()))
        ho, wo = (H * self.stride, W * self.stride) if self.transposed else (H, W)
        y = torch.empty((B, ho, wo, cp4(self.cout)), dtype=torch.float32, device=x.device)
        _chk(res, y.shape, name="res")
        nb = 4 * (P.numel() + y.numel() * (2 if res is not None else 1))
        profiling.timed_hbm("tap_gather", nb, lambda: _lib.call(
            "fvc_tap_gather_nhwc", P.data_ptr(), self.pcp, self.bias.data_ptr(), _ptr(res), y.data_ptr(), B, H, W,
            self.cout, self.ksize, self.stride, int(self.transposed), act, post, stream_handle()))
        return y


def x3_overflow(reset: bool = True, device=None) -> bool:
    """True if any split-precision conv on the current stream staged an activation with
    |v| >= 65000 since the last reset (waits for the stream's queued work)."""
    return OverflowProbe(device, reset).result()


# ------------------------------------------------------------------ reductions
_WS = {}


def _ws(device):
    key = (str(device), stream_handle())  # one reduction workspace per stream (overlapped pipelines)
    if key not in _WS:
        n = _lib.load().fvc_reduce_ws_doubles()
        _WS[key] = torch.empty(n, dtype=torch.float64, device=device)
    return _WS[key]


def recon_finalize(recon, inp, warpframe, prediction):
    B, H, W, _ = recon.shape
    for t, n in ((recon, "recon"), (inp, "input"), (warpframe, "warpframe"), (prediction, "prediction")):
        _chk(t, (B, H, W, 4), name=n)
    clipped = torch.empty((B, 3, H, W), dtype=torch.float32, device=recon.device)
    out4 = torch.empty(4, dtype=torch.float64, device=recon.device)  # recon, warp, pred, clipped SSEs
    nb = 4 * (recon.numel() + inp.numel() + warpframe.numel() + prediction.numel() + clipped.numel())
    ws = _ws(recon.device)
    profiling.timed_hbm("recon_finalize", nb, lambda: _lib.call(
        "fvc_recon_finalize", recon.data_ptr(), inp.data_ptr(), warpframe.data_ptr(), prediction.data_ptr(),
        clipped.data_ptr(), out4.data_ptr(), ws.data_ptr(), B, H, W, stream_handle()))
    return clipped, out4


def bits_laplace(feature, sigma, c):
    B, H, W, cp = feature.shape
    _chk(feature, name="feature")
    _chk(sigma, feature.shape, name="sigma")
    out = torch.empty(1, dtype=torch.float64, device=feature.device)
    _lib.call("fvc_bits_laplace", feature.data_ptr(), sigma.data_ptr(), out.data_ptr(),
              _ws(feature.device).data_ptr(), B, H, W, c, cp, stream_handle())
    return out


def bits_factorized(v, params, c):
    B, H, W, cp = v.shape
    _chk(v, name="v")
    _chk(params, (11, c), name="params")
    out = torch.empty(1, dtype=torch.float64, device=v.device)
    _lib.call("fvc_bits_factorized", v.data_ptr(), params.data_ptr(), out.data_ptr(), _ws(v.device).data_ptr(),
              B, H, W, c, cp, stream_handle())
    return out


# ------------------------------------------------------------------ entropy coding
def latent_to_symbols(lat, c):
    B, H, W, cp = lat.shape
    _chk(lat, name="latent")
    sym = torch.empty((B, c, H * W), dtype=torch.int32, device=lat.device)
    _lib.call("fvc_latent_to_symbols", lat.data_ptr(), sym.data_ptr(), B, H, W, c, cp, stream_handle())
    return sym


def symbols_to_latent(sym, h, w, c):
    B = sym.shape[0]
    _chk(sym, (B, c, h * w), dtype=torch.int32, name="symbols")
    lat = torch.empty((B, h, w, cp4(c)), dtype=torch.float32, device=sym.device)
    _lib.call("fvc_symbols_to_latent", sym.data_ptr(), lat.data_ptr(), B, h, w, c, cp4(c), stream_handle())
    return lat


def build_indexes(sigma, scale_table, c):
    B, H, W, cp = sigma.shape
    _chk(sigma, name="sigma")
    _chk(scale_table, name="scale_table")
    idx = torch.empty((B, c, H * W), dtype=torch.int32, device=sigma.device)
    _lib.call("fvc_build_indexes", sigma.data_ptr(), scale_table.data_ptr(), scale_table.numel(), idx.data_ptr(),
              B, H, W, c, cp, stream_handle())
    return idx


def channel_indexes(b, hw, c, device):
    idx = torch.empty((b, c, hw), dtype=torch.int32, device=device)
    _lib.call("fvc_channel_indexes", idx.data_ptr(), b, hw, c, stream_handle())
    return idx
