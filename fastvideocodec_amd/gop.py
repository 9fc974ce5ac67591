"""GOP driver for real encode+decode (the bitstream counterpart of models.parallel_compression,
models.py:368-383): the I-frame passes through (BPG out of scope), every P-frame is encoded and
then decoded from its bitstream.

Four HIP streams form a pipeline (four, because the GPU exposes GPU_MAX_HW_QUEUES = 4 hardware
queues per process: a fifth stream would share a queue and serialise behind another stream's
work):
  * encoder stream (the caller's current stream): the encoder forward of frame t, using the
    encoder's own reconstruction of frame t-1 as reference (exactly what the reference loop
    does: x_prev = model(...)[0]);
  * two coder streams, round-robin over frames: symbols -> rANS encode of frame t (waits only on
    frame t's latents), then rANS decode of its z -> hyperprior -> feature, and mv (no reference
    frame needed, so consecutive frames code and decode concurrently);
  * reconstruction stream: mvDecoder + motion compensation + resDecoder of frame t against the
    decoder's own previous reconstruction (waits on frame t's latents).
Encoder and decoder reconstructions are bit-identical (same kernels, same operand order;
checked by tests and by bench.py), so the decoder never gates the encoder, and the pipelines
overlap on the GPU (the rANS chains are latency-bound on few CUs, beside compute-bound convs).

G GOPs are batched along dim 0 (frame t of every GOP in one forward).
"""
from __future__ import annotations

import os

import torch

from . import _lib
from . import kernels as K

# CUs the conv kernels' persistent grids leave free while the pipeline's side streams run.
# r1 (static schedule, 4 GOPs per step, scripts/gpu_reserve_sweep.sh): 16 -> 49.2, 24 -> 50.3,
# 32 -> 51.1, 40 -> 50.4, 48 -> 49.4, 64 -> 48.7 P-frames/s. r4 (dynamic work-item schedule,
# segment-framed rANS with short chains, 16 GOPs, two runs each; data in profiles/r4/reserve_sweep/):
# 32 -> 71.13 / 71.00, 16 -> 71.79 / 71.68, 8 -> 72.27 / 72.37, 0 -> 72.49 / 72.56: no reserve.
PIPELINE_CU_RESERVE = int(os.environ.get("FVC_PIPELINE_CU_RESERVE", "0"))

_STREAMS = {}


def _side_streams(device):
    key = str(device)
    if key not in _STREAMS:
        _STREAMS[key] = tuple(torch.cuda.Stream(device=device) for _ in range(3))
    return _STREAMS[key]


def _record(obj, stream, seen=None):
    """record_stream every tensor reachable from obj (dicts, sequences, plain objects) on stream,
    so the caching allocator does not hand its memory out again before that stream's use ends."""
    seen = set() if seen is None else seen
    if id(obj) in seen:
        return
    seen.add(id(obj))
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record(v, stream, seen)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _record(v, stream, seen)
    elif hasattr(obj, "__dict__"):
        for v in vars(obj).values():
            _record(v, stream, seen)


def encode_decode_gop(model, frames: torch.Tensor, check=False, overlap=True, join=True):
    """frames: [G, T, 3, H, W] device tensor. Returns (bitstreams, decoder recons, encoder sse
    list, encoder recons); with join=True every returned tensor is ready on the caller's stream.

    join=False (streaming use, e.g. back-to-back GOPs in bench.py): the caller's stream does not
    wait for this GOP's coder/decoder tail, so the next GOP's encoder starts while the last
    frames are still being range-decoded and reconstructed; every tensor that crosses streams is
    record_stream'ed, and the caller synchronises the device (or waits on the side streams via
    join_side_streams) before reading the returned bitstreams / recons.

    Split-precision overflow: after each frame's encoder pass a non-blocking probe copies the
    encoder stream's overflow flag to pinned memory. join=True resolves the probes at the end:
    on a hit the GOP is re-coded on the fp32 kernels (model.on_overflow == "recompute"; its
    bitstreams then carry precision 'f32') or FvcError is raised. join=False leaves the probes
    on the model; the caller resolves them with check_overflow(model) after synchronising."""
    if join:
        pending = getattr(model, "_overflow_probes", [])
        model._overflow_probes = []
        err = None
        try:
            out = _encode_decode_gop(model, frames, check, overlap, join)
        except _lib.FvcError as e:  # e.g. a corrupt-stream check tripped by an overflowed frame
            err = e
        hit = any(p.result() for p in model._overflow_probes)
        model._overflow_probes = pending
        if err is not None and not hit:
            raise err
        if hit and K.conv_precision() != "f32":
            model.overflow_events = getattr(model, "overflow_events", 0) + 1
            if model.on_overflow == "raise":
                raise _lib.FvcError("split-precision conv operand overflow in a GOP")
            with K.precision("f32"):
                return encode_decode_gop(model, frames, check, overlap, join)
        return out
    return _encode_decode_gop(model, frames, check, overlap, join)


def check_overflow(model) -> bool:
    """Resolve the overflow probes of join=False GOPs (waits for their copies). Raises FvcError
    on a hit: streamed bitstreams cannot be re-coded after the fact."""
    probes = getattr(model, "_overflow_probes", [])
    model._overflow_probes = []
    if any(p.result() for p in probes):
        model.overflow_events = getattr(model, "overflow_events", 0) + 1
        raise _lib.FvcError("split-precision conv operand overflow in a streamed GOP; re-code it "
                            "with kernels.precision('f32')")
    return False


def _encode_decode_gop(model, frames, check, overlap, join):
    G, T = frames.shape[:2]
    main = torch.cuda.current_stream(frames.device)
    if overlap:
        s_cd0, s_cd1, s_rec = _side_streams(frames.device)
    else:
        s_cd0 = s_cd1 = s_rec = main
    if not hasattr(model, "_overflow_probes"):
        model._overflow_probes = []
    if K.conv_precision() != "f32":
        K.overflow_flag(frames.device).zero_()
    x_enc = frames[:, 0].contiguous()
    x_dec = x_enc
    bitstreams, decoded, sses, enc_recons, keep = [], [], [], [], [x_enc]
    model.update()
    # launches outside the pipeline get the whole GPU: the reserve applies inside this block only
    with torch.no_grad(), K.cu_reserve(PIPELINE_CU_RESERVE if overlap else 0), K.rans_throughput(overlap):
        for t in range(1, T):
            cur = frames[:, t].contiguous()
            tens = model._encode_graph(cur, x_enc)
            clipped, sse = K.recon_finalize(tens["recon"], tens["cur4"], tens["warpframe"], tens["prediction"])
            if K.conv_precision() != "f32":
                model._overflow_probes.append(K.OverflowProbe(frames.device))
            lat = {k: tens[k] for k in ("mvfeature", "z", "feature", "sigma")}
            del tens
            s_cd = s_cd0 if t % 2 else s_cd1
            s_cd.wait_stream(main)
            with torch.cuda.stream(s_cd):
                bs = model.compress_tensors(lat)
                dlat = model.decode_latents(bs, check=check)
            s_rec.wait_stream(s_cd)
            with torch.cuda.stream(s_rec):
                rec_dec = model.reconstruct(dlat, x_dec)
            if overlap and not join:
                if t == 1:
                    _record(x_enc, s_rec)  # the I-frame: decoder reference of frame 1
                _record(lat, s_cd)
                _record(dlat, s_rec)
            keep.append((lat, cur, dlat))  # cross-stream tensors stay alive until the pipeline drains
            bitstreams.append(bs)
            decoded.append(rec_dec)
            enc_recons.append(clipped)
            sses.append(sse)
            x_enc, x_dec = clipped, rec_dec
    if join:
        join_side_streams(frames.device)
    return bitstreams, decoded, sses, enc_recons


def join_side_streams(device):
    """Make the current stream wait for all pipeline side streams of device."""
    main = torch.cuda.current_stream(device)
    for st in _side_streams(device):
        main.wait_stream(st)
