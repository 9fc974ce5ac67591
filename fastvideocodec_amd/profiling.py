"""Live per-kernel timing with HIP events on the launching stream (used by bench.py).

When a ``KernelTimer`` is active, every ``PackedConv`` launch records a start/end
``torch.cuda.Event`` pair on the current stream (the stream the kernel is launched on) and
the algorithmic FLOPs of that launch. Events only; no host synchronisation until ``collect``.
"""
from __future__ import annotations

import torch

_ACTIVE = None


def conv_flops(cin, cout, k, stride, transposed, batch, h, w):
    """Algorithmic FLOPs (2 x MAC, unpadded channels) of one conv / deconv launch."""
    if transposed:
        # every input pixel scatters k*k taps into the output: MAC = B*h*w*cin*cout*k*k
        return 2.0 * batch * h * w * cin * cout * k * k
    ho, wo = h // stride, w // stride
    return 2.0 * batch * ho * wo * cin * cout * k * k


class KernelTimer:
    def __init__(self):
        self.records = []
        self.hbm_records = []  # (ev0, ev1, name, algorithmic bytes) of the HBM-bound kernels

    def __enter__(self):
        global _ACTIVE
        _ACTIVE = self
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = None

    def _select(self, x3, family):
        return [r for r in self.records if (x3 is None or (len(r) > 4 and r[4]) == x3) and
                (family is None or (len(r) > 6 and r[6] == family))]

    def collect(self, x3=None, family=None):
        """Synchronise and return (total_ms, total_flops, n_launches); x3=True/False restricts to
        the split-precision / the fp32+VALU conv launches, family to one kernel ('x3': the direct
        conv_x3_kernel, 'wino': conv_wino_kernel, 'f32'). n_launches counts kernel dispatches (a
        record's 8th field; the 128-channel Winograd quarters are 4 per call), as rocprofv3 does."""
        torch.cuda.synchronize()
        rs = self._select(x3, family)
        ms = sum(r[0].elapsed_time(r[1]) for r in rs)
        fl = sum(r[2] for r in rs)
        return ms, fl, sum(r[7] if len(r) > 7 else 1 for r in rs)

    def collect_bytes(self, x3=None, family=None):
        """Algorithmic HBM bytes (input + packed weights + output + residual) of the launches
        ``collect(x3, family)`` counts."""
        return sum(r[5] for r in self._select(x3, family) if len(r) > 5)

    def collect_hbm(self):
        """{name: [launches, ms, algorithmic bytes]} of the HBM-bound (non-conv) kernels."""
        torch.cuda.synchronize()
        agg = {}
        for ev0, ev1, name, nbytes in self.hbm_records:
            a = agg.setdefault(name, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += ev0.elapsed_time(ev1)
            a[2] += nbytes
        return agg

    def breakdown(self):
        """Per-geometry aggregate: {key: [launches, ms, flops]} (keys recorded by the caller)."""
        torch.cuda.synchronize()
        agg = {}
        for r in self.records:
            key = r[3] if len(r) > 3 else "?"
            a = agg.setdefault(key, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += r[0].elapsed_time(r[1])
            a[2] += r[2]
        return agg


def active():
    return _ACTIVE


def timed_hbm(name, nbytes, fn):
    """Run fn (one HBM-bound kernel launch); with a KernelTimer active, bracket it with HIP events
    on the current stream and record its algorithmic bytes (each input read once, each output
    written once, padded channels included: they are moved)."""
    t = _ACTIVE
    if t is None:
        return fn()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    r = fn()
    ev1.record()
    t.hbm_records.append((ev0, ev1, name, float(nbytes)))
    return r
