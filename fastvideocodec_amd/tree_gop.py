"""LSVC-style tree GOP: P-frames grouped into the layers of a reference tree
and coded one layer per forward, so every frame of a layer (of every batched GOP) shares one
launch sequence.

The graph functions mirror the reference (``models.py:683-728`` generate_graph,
``models.py:923-940`` graph_from_batch, ``models.py:942-949`` refidx_from_graph). The reference
LSVC codec (``models.py:1347-1411``) runs its tree with its own networks; here the tree drives
the DVC P-frame codec: frame t is coded by ``VideoCompressor`` against the reconstruction of its
parent ``parents[t]`` (frame 0 = the I-frame), exactly as if it were the next frame of a linear
GOP whose previous frame is that parent. A layer's frames only depend on earlier layers, so they
form one batch; the result of every frame equals coding it alone against its parent (the kernels
are batch-invariant: tests/test_gpu_tree_gop.py).
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K
from .gop import PIPELINE_CU_RESERVE, _record, _side_streams, join_side_streams


def generate_graph(graph_type="default"):
    """models.py:683-728: (children dict, layers, parents) of a reference tree over P-frames
    1..n (node 0 is the I-frame)."""
    if graph_type == "default":
        g = {k: [k + 1] for k in range(30)}
        layers = [[i + 1] for i in range(30)]
        parents = {i + 1: i for i in range(30)}
    elif graph_type == "onehop":
        g = {0: [i + 1 for i in range(14)]}
        layers = [[i + 1 for i in range(14)]]
        parents = {i + 1: 0 for i in range(14)}
    elif graph_type == "2layers":
        g = {0: [1, 2]}
        layers = [[1, 2]]
        parents = {1: 0, 2: 0}
    elif graph_type == "3layers":
        g = {0: [1, 4], 1: [2, 3], 4: [5, 6]}
        layers = [[1, 4], [2, 3, 5, 6]]
        parents = {1: 0, 4: 0, 2: 1, 3: 1, 5: 4, 6: 4}
    elif graph_type == "4layers":
        g = {0: [1, 8], 1: [2, 5], 8: [9, 12], 2: [3, 4], 5: [6, 7], 9: [10, 11], 12: [13, 14]}
        layers = [[1, 8], [2, 5, 9, 12], [3, 4, 6, 7, 10, 11, 13, 14]]
        parents = {1: 0, 8: 0, 2: 1, 5: 1, 9: 8, 12: 8, 3: 2, 4: 2, 6: 5, 7: 5, 10: 9, 11: 9, 13: 12, 14: 12}
    elif graph_type == "5layers":
        g = {0: [1, 16], 1: [2, 9], 16: [17, 24], 2: [3, 6], 9: [10, 13], 17: [18, 21], 24: [25, 28],
             3: [4, 5], 6: [7, 8], 10: [11, 12], 13: [14, 15], 18: [19, 20], 21: [22, 23], 25: [26, 27],
             28: [29, 30]}
        layers = [[1, 16], [2, 9, 17, 24], [3, 6, 10, 13, 18, 21, 25, 28],
                  [4, 5, 7, 8, 11, 12, 14, 15, 19, 20, 22, 23, 26, 27, 29, 30]]
        parents = {1: 0, 16: 0, 2: 1, 9: 1, 17: 16, 24: 16, 3: 2, 6: 2, 10: 9, 13: 9, 18: 17, 21: 17, 25: 24,
                   28: 24, 4: 3, 5: 3, 7: 6, 8: 6, 11: 10, 12: 10, 14: 13, 15: 13, 19: 18, 20: 18, 22: 21,
                   23: 21, 26: 25, 27: 25, 29: 28, 30: 28}
    else:
        raise ValueError(f"Undefined graph type: {graph_type}")
    return g, layers, parents


def graph_from_batch(bs, isLinear=False, isOnehop=False):
    """models.py:923-940: the smallest tree holding bs P-frames (linear / one-hop on request)."""
    if isLinear:
        return generate_graph("default")
    if isOnehop:
        return generate_graph("onehop")
    if bs <= 2:
        return generate_graph("2layers")
    if bs <= 6:
        return generate_graph("3layers")
    if bs <= 14:
        return generate_graph("4layers")
    if bs <= 30:
        return generate_graph("5layers")
    raise ValueError(f"Batch size not supported yet: {bs}")


def refidx_from_graph(g, bs):
    """models.py:942-949: ref_index[k-1] = parent of P-frame k (0 = the I-frame)."""
    ref_index = [-1 for _ in range(bs)]
    for start in g:
        if start > bs:
            continue
        for k in g[start]:
            if k > bs:
                continue
            ref_index[k - 1] = start
    return ref_index


def binary_tree_graph(depth):
    """The reference's tree shape generalised: P-frames 1..2^depth - 2 as a complete binary tree
    in pre-order under the I-frame, children of node k at k + 1 and k + 1 + (size of k's left
    subtree). depth 2..5 give exactly generate_graph('2layers' .. '5layers') (tests/
    test_tree_gop.py); depth 6 (62 frames) is this build's extension for GOPs past the
    reference's 30-frame limit (graph_from_batch raises there, as the reference fails)."""
    if depth < 2:
        raise ValueError("depth >= 2")
    g, parents, layers = {}, {}, []

    def build(k, level, size):  # node k at tree level `level` (0 = I-frame) heads `size` nodes
        if size <= 1:
            return
        half = (size - 1) // 2  # nodes under each child
        kids = [k + 1, k + 1 + half]
        g[k] = kids
        while len(layers) <= level:
            layers.append([])
        for c in kids:
            parents[c] = k
            layers[level].append(c)
            build(c, level + 1, half)

    build(0, 0, 2 ** depth - 1)
    return g, [sorted(l) for l in layers], parents


def coding_layers(bs, isLinear=False, isOnehop=False, extend=False):
    """The layers of graph_from_batch(bs) restricted to frames 1..bs, with each frame's parent.
    extend=True: past the reference's 30 frames, the 62-frame binary tree (binary_tree_graph)."""
    if extend and bs > 30 and not (isLinear or isOnehop):
        if bs > 62:
            raise ValueError(f"Batch size not supported yet: {bs}")
        _, layers, parents = binary_tree_graph(6)
    else:
        _, layers, parents = graph_from_batch(bs, isLinear, isOnehop)
    out = []
    for layer in layers:
        tl = [t for t in layer if t <= bs]
        if tl:
            out.append([(t, parents[t]) for t in tl])
    return out


def encode_decode_tree_gop(model, frames: torch.Tensor, check=False, overlap=True, isLinear=False,
                           isOnehop=False, join=True, extend=False):
    """frames: [G, T, 3, H, W] device tensor (frame 0 of each GOP is the I-frame, passed through).
    Codes the T-1 P-frames of every GOP layer by layer: one encoder forward per layer over all
    G x len(layer) frames, then range coding, entropy decoding and reconstruction of that layer
    on side streams (as gop.encode_decode_gop). Returns (bitstreams, decoded, sses, enc_recons):
    bitstreams[i] is the PFrameBitstream of layer i with batch order (frame-major: frame j of the
    layer, GOP g at j*G + g); decoded / enc_recons map P-frame index t to its [G,3,H,W] recon;
    sses[i] are layer i's encoder SSE sums (device doubles). With join=True all results are
    joined to the caller's stream and a split-precision overflow in any layer re-codes the GOP on
    the fp32 kernels (model.on_overflow == "recompute") or raises FvcError. join=False
    (streaming, bench.py's timed loop, as gop.encode_decode_gop): no host wait and no join; the
    overflow probes stay on the model for gop.check_overflow after the caller synchronises."""
    if not join:
        if not hasattr(model, "_overflow_probes"):
            model._overflow_probes = []
        return _tree(model, frames, check, overlap, isLinear, isOnehop, model._overflow_probes, join, extend)
    probes = []
    out = _tree(model, frames, check, overlap, isLinear, isOnehop, probes, join, extend)
    if probes and any(p.result() for p in probes):
        model.overflow_events = getattr(model, "overflow_events", 0) + 1
        if model.on_overflow == "raise":
            raise _lib.FvcError("split-precision conv operand overflow in a tree GOP")
        with K.precision("f32"):
            return _tree(model, frames, check, overlap, isLinear, isOnehop, [], join, extend)
    return out


def _tree(model, frames, check, overlap, isLinear, isOnehop, probes, join=True, extend=False):
    G, T = frames.shape[:2]
    lay = coding_layers(T - 1, isLinear, isOnehop, extend)
    main = torch.cuda.current_stream(frames.device)
    if overlap:
        s_cd0, s_cd1, s_rec = _side_streams(frames.device)
    else:
        s_cd0 = s_cd1 = s_rec = main
    enc = {0: frames[:, 0].contiguous()}
    dec = {0: enc[0]}
    bitstreams, sses = [], []
    model.update()
    if K.conv_precision() != "f32":
        K.overflow_flag(frames.device).zero_()
    with torch.no_grad(), K.cu_reserve(PIPELINE_CU_RESERVE if overlap else 0), K.rans_throughput(overlap):
        for i, layer in enumerate(lay):
            cur = torch.cat([frames[:, t] for t, _ in layer], 0).contiguous()
            ref_e = torch.cat([enc[p] for _, p in layer], 0).contiguous()
            tens = model._encode_graph(cur, ref_e)
            clipped, sse = K.recon_finalize(tens["recon"], tens["cur4"], tens["warpframe"], tens["prediction"])
            if K.conv_precision() != "f32":
                probes.append(K.OverflowProbe(frames.device))
            lat = {k: tens[k] for k in ("mvfeature", "z", "feature", "sigma")}
            del tens
            s_cd = s_cd0 if i % 2 == 0 else s_cd1
            s_cd.wait_stream(main)
            with torch.cuda.stream(s_cd):
                bs = model.compress_tensors(lat)
                dlat = model.decode_latents(bs, check=check)
            s_rec.wait_stream(s_cd)
            with torch.cuda.stream(s_rec):
                ref_d = torch.cat([dec[p] for _, p in layer], 0).contiguous()
                rec = model.reconstruct(dlat, ref_d)
            if overlap:
                if i == 0 and not join:
                    _record(enc[0], s_rec)  # the I-frames: decoder references of layer 0
                _record(lat, s_cd)
                _record(dlat, s_rec)
                if not join:
                    _record(ref_d, s_rec)
            for j, (t, _) in enumerate(layer):
                enc[t] = clipped[j * G:(j + 1) * G]
                dec[t] = rec[j * G:(j + 1) * G]
            bitstreams.append(bs)
            sses.append(sse)
    if join:
        join_side_streams(frames.device)
    decoded = {t: v for t, v in dec.items() if t > 0}
    enc_recons = {t: v for t, v in enc.items() if t > 0}
    return bitstreams, decoded, sses, enc_recons
