"""Debug aid (r5): encoder recon vs decoder recon of one GOP through the overlapped pipeline and
the serial one, frame by frame (which frame first differs, by how much, and whether the
split-precision overflow recompute fired). Run with FVC_LIB_PATH / FVC_* switches to compare."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fastvideocodec_amd import kernels as K  # noqa: E402
from fastvideocodec_amd.gop import encode_decode_gop  # noqa: E402

dev = torch.device("cuda")
views = int(os.environ.get("VIEWS", "8"))
base = dict(gpus=1, steps=1, warmup=0, height=1080, width=1920, gop=3, gops_per_gpu=1, views=0, cpu_baseline="none",
            json_out=None, breakdown=False, tree=False, serial=False)
if views > 1:
    base.update(views=views)
    job = bench.GpuGopJob(argparse.Namespace(**base), 0, 1, dev)
else:
    base.update(height=2160, width=3840, gop=32)
    job = bench.GpuGopJob(argparse.Namespace(**base), 2, 4, dev)
for overlap in (True, False):
    K.x3_overflow(reset=True)
    job.model.overflow_events = 0
    bss, dec, _, enc = encode_decode_gop(job.model, job.frames, check=True, overlap=overlap)
    torch.cuda.synchronize()
    bad = [(t + 1, float((a - b).abs().max())) for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print(f"overlap={overlap}: frames {len(dec)}, mismatching {bad[:5]}, overflow_events "
          f"{getattr(job.model, 'overflow_events', 0)}, precisions {sorted(set(b.precision for b in bss))}", flush=True)

# where does the overlapped run diverge? re-decode every bitstream serially and rebuild the
# decoder chain from the pipeline's own previous decoded frame
if os.environ.get("LOCATE", "0") == "1":
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(job.model, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    x_prev = job.frames[:, 0].contiguous()
    with torch.no_grad():
        for t, bs in enumerate(bss, 1):
            dl = job.model.decode_latents(bs, check=True)
            r = job.model.reconstruct(dl, x_prev)
            torch.cuda.synchronize()
            print(f"t={t}: serial(bs, pipeline dec[t-1]) == pipeline dec[t]: {torch.equal(r, dec[t - 1])}, "
                  f"== enc[t]: {torch.equal(r, enc[t - 1])}; pipeline dec == enc: {torch.equal(dec[t - 1], enc[t - 1])}",
                  flush=True)
            x_prev = dec[t - 1]
            if t >= 8:
                break

# which decoder stage goes wrong? keep copies (stream-ordered clones) of every decode_latents
# output and every reconstruct stage in the overlapped run, then replay the first bad frame serially
if os.environ.get("LOCATE", "0") == "2":
    m = job.model
    saved = {"dl": [], "rec": []}
    orig_dl, orig_rec = m.decode_latents, m.reconstruct

    def dl_wrap(bs, check=True):
        d = orig_dl(bs, check)
        saved["dl"].append({k: (v.clone() if torch.is_tensor(v) else v) for k, v in d.items()})
        return d

    def rec_wrap(lat, referframe):
        with torch.no_grad(), K.precision(lat.get("precision")):
            ref4 = K.nchw_to_nhwc(referframe.float().contiguous(), 4)
            mv_up = m.mvDecoder.run(lat["mv"])
            prediction, _ = m.motioncompensation(ref4, mv_up)
            recon = m.resDecoder.run(lat["feature"], prediction)
            out = K.nhwc_to_nchw(recon, 3, clamp01=True)
            saved["rec"].append({"ref": referframe.clone(), "mv_up": mv_up.clone(), "prediction": prediction.clone(),
                                 "recon": recon.clone(), "out": out.clone()})
            return out

    m.decode_latents, m.reconstruct = dl_wrap, rec_wrap
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(m, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    m.decode_latents, m.reconstruct = orig_dl, orig_rec
    bad = [t for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print("mismatching frames (0-based):", bad[:6], flush=True)
    if bad:
        t = bad[0]
        with torch.no_grad():
            dl = orig_dl(bss[t], True)
            for k in ("mv", "feature", "z"):
                print(f"frame {t}: decoded {k} equal: {torch.equal(dl[k], saved['dl'][t][k])}", flush=True)
            s = saved["rec"][t]
            print(f"frame {t}: reference equal to the pipeline's previous output: "
                  f"{torch.equal(s['ref'], dec[t - 1] if t else job.frames[:, 0])}", flush=True)
            ref4 = K.nchw_to_nhwc(s["ref"].float().contiguous(), 4)
            mv_up = m.mvDecoder.run(saved["dl"][t]["mv"])
            print(f"frame {t}: mv_up equal: {torch.equal(mv_up, s['mv_up'])}", flush=True)
            prediction, _ = m.motioncompensation(ref4, s["mv_up"])
            print(f"frame {t}: prediction equal: {torch.equal(prediction, s['prediction'])}", flush=True)
            recon = m.resDecoder.run(saved["dl"][t]["feature"], s["prediction"])
            print(f"frame {t}: recon equal: {torch.equal(recon, s['recon'])}", flush=True)
            torch.cuda.synchronize()

# is the encoder-stream kernel itself also wrong in the overlapped run? (both sides wrong would
# point below the kernels: co-resident workgroups disturbing each other)
if os.environ.get("LOCATE", "0") == "3":
    m = job.model
    of = m.opticFlow
    saved = []
    orig_run = of.run

    def of_wrap(cur4, ref4):
        out = orig_run(cur4, ref4)
        saved.append((cur4.clone(), ref4.clone(), out.clone()))
        return out

    of.run = of_wrap
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(m, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    of.run = orig_run
    bad = [t for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print("decoder mismatching frames (0-based):", bad[:6], flush=True)
    with torch.no_grad():
        for t, (c4, r4, o) in enumerate(saved[:12]):
            o2 = orig_run(c4, r4)
            torch.cuda.synchronize()
            print(f"frame {t}: SpyNet output in the pipeline equal to its serial replay: {torch.equal(o, o2)}"
                  f" (max diff {float((o - o2).abs().max()):.3e})", flush=True)

# which kernel is it? every libfvc op of the GOP (both streams) runs twice back to back on its own
# stream with the same inputs; the two outputs must be equal (the kernels are deterministic), so a
# pair that differs names the op that computed a wrong result while the other stream was busy
if os.environ.get("LOCATE", "0") == "4":
    from fastvideocodec_amd import gop as G
    m = job.model
    s_rec = G._side_streams(dev)[2]
    flags = []

    def _tensors(o):
        if torch.is_tensor(o):
            return [o]
        if isinstance(o, (tuple, list)):
            return [t for v in o for t in _tensors(v)]
        return []

    def dup(name, fn):
        def w(*a, **kw):
            out = fn(*a, **kw)
            if kw.get("out") is None:
                out2 = fn(*a, **kw)
                d = [(x != y).any() for x, y in zip(_tensors(out), _tensors(out2)) if x.shape == y.shape]
                if d:
                    cs = torch.cuda.current_stream(dev).cuda_stream
                    flags.append((name, "rec" if cs == s_rec.cuda_stream else str(cs), torch.stack(d).any()))
            return out
        return w

    patches = [(K.PackedConv, "__call__"), (K.PackedConv, "call_pool"), (K.PackedConv, "call_tap"),
               (K.TapConsumer, "gather"), (K, "upsample2x_add"), (K, "mc_assemble")]
    saved_fns = [(o, n, getattr(o, n)) for o, n in patches]
    for o, n, f in saved_fns:
        setattr(o, n, dup(n, f))
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(m, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    for o, n, f in saved_fns:
        setattr(o, n, f)
    bad = [t for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print("decoder mismatching frames (0-based):", bad[:6], flush=True)
    diffs = [(i, n, s) for i, (n, s, f) in enumerate(flags) if bool(f)]
    print(f"ops run twice: {len(flags)}; pairs that differ: {len(diffs)}", flush=True)
    for i, n, s in diffs[:40]:
        print(f"  call {i}: {n} on stream {s}", flush=True)

# running ops twice hides it (LOCATE=4 saw no mismatch at all), so: one run, an exact integer
# checksum of every reconstruction-stream op's output taken stream-ordered right after the op,
# then a serial replay of the first bad frame from its saved inputs with the same checksums: the
# first op whose checksum differs is the one that went wrong
if os.environ.get("LOCATE", "0") == "5":
    m = job.model
    state = {"frame": -1, "in_rec": False}
    sums = {}
    saved = {"dl": [], "ref": []}

    def _tensors(o):
        if torch.is_tensor(o):
            return [o]
        if isinstance(o, (tuple, list)):
            return [t for v in o for t in _tensors(v)]
        return []

    def ck(name, fn):
        def w(*a, **kw):
            out = fn(*a, **kw)
            if state["in_rec"]:
                for t in _tensors(out):
                    if t.dtype == torch.float32 and t.is_contiguous():
                        sums.setdefault(state["frame"], []).append((name, tuple(t.shape),
                                                                   t.view(torch.int32).sum(dtype=torch.int64)))
            return out
        return w

    orig_dl, orig_rec = m.decode_latents, m.reconstruct

    def dl_wrap(bs, check=True):
        d = orig_dl(bs, check)
        saved["dl"].append({k: (v.clone() if torch.is_tensor(v) else v) for k, v in d.items()})
        return d

    def rec_wrap(lat, referframe):
        state["frame"] += 1
        saved["ref"].append(referframe.clone())
        state["in_rec"] = True
        try:
            return orig_rec(lat, referframe)
        finally:
            state["in_rec"] = False

    patches = [(K.PackedConv, "__call__"), (K.PackedConv, "call_pool"), (K.PackedConv, "call_tap"),
               (K.TapConsumer, "gather"), (K, "upsample2x_add"), (K, "mc_assemble"), (K, "nchw_to_nhwc")]
    saved_fns = [(o, n, getattr(o, n)) for o, n in patches]
    for o, n, f in saved_fns:
        setattr(o, n, ck(n, f))
    m.decode_latents, m.reconstruct = dl_wrap, rec_wrap
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(m, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    m.decode_latents, m.reconstruct = orig_dl, orig_rec
    bad = [t for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print("decoder mismatching frames (0-based):", bad[:6], flush=True)
    pipe = {f: [(n, s, int(v)) for n, s, v in lst] for f, lst in sums.items()}
    for t in (bad[:1] or [len(dec) - 1]):
        state["frame"] = -10 - t  # record on the current (main) stream for the replay
        sums.clear()
        state["in_rec"] = True
        with torch.no_grad():
            r = m.reconstruct(saved["dl"][t], saved["ref"][t])
        state["in_rec"] = False
        torch.cuda.synchronize()
        rep = [(n, s, int(v)) for n, s, v in sums[-10 - t]]
        print(f"frame {t}: replay output == pipeline dec: {torch.equal(r, dec[t])}, == enc: {torch.equal(r, enc[t])}; "
              f"ops pipeline {len(pipe.get(t, []))}, replay {len(rep)}", flush=True)
        for j, (a, b) in enumerate(zip(pipe.get(t, []), rep)):
            print(f"  op {j:3d} {a[0]:16s} {str(a[1]):24s} {'==' if a == b else '!= <<<'}", flush=True)
    for o, n, f in saved_fns:
        setattr(o, n, f)

# LOCATE=5 named the MC warp/assemble kernel (its inputs' checksums equal, its output not). Did
# its inputs change under it, or did it compute wrongly from the right inputs? Checksums of both
# inputs immediately before and after it (stream-ordered), copies of everything, then replays.
if os.environ.get("LOCATE", "0") == "6":
    m = job.model
    state = {"in_rec": False}
    rec = []
    orig_mc, orig_rec = K.mc_assemble, m.reconstruct

    def isum(t):
        return t.view(torch.int32).sum(dtype=torch.int64)

    def mc_wrap(ref, mv):
        if not state["in_rec"]:
            return orig_mc(ref, mv)
        before = (isum(ref), isum(mv))
        wf, x8 = orig_mc(ref, mv)
        after = (isum(ref), isum(mv))
        rec.append(dict(before=before, after=after, ref=ref.clone(), mv=mv.clone(), wf=wf.clone(), x8=x8.clone(),
                        ptr=(ref.data_ptr(), mv.data_ptr(), wf.data_ptr(), x8.data_ptr())))
        return wf, x8

    def rec_wrap(lat, referframe):
        state["in_rec"] = True
        try:
            return orig_rec(lat, referframe)
        finally:
            state["in_rec"] = False

    K.mc_assemble, m.reconstruct = mc_wrap, rec_wrap
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(m, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    K.mc_assemble, m.reconstruct = orig_mc, orig_rec
    bad = [t for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print("decoder mismatching frames (0-based):", bad[:6], flush=True)
    for t, r in enumerate(rec):
        ch = [int(a) != int(b) for a, b in zip(r["before"], r["after"])]
        wf2, x82 = orig_mc(r["ref"], r["mv"])
        torch.cuda.synchronize()
        same = torch.equal(wf2, r["wf"]) and torch.equal(x82, r["x8"])
        line = f"frame {t}: inputs changed during the kernel (ref, mv): {ch}; replay from the inputs as left == output: {same}"
        if not same:
            d = (wf2 != r["wf"]).any(-1)[0]
            ys, xs = torch.nonzero(d, as_tuple=True)
            npx = int(d.sum())
            H, W = d.shape
            flat = (ys * W + xs)
            line += (f"; {npx} pixels differ, rows {int(ys.min())}..{int(ys.max())}, cols {int(xs.min())}..{int(xs.max())}, "
                     f"flat {int(flat.min())}..{int(flat.max())}")
            dx8 = (x82 != r["x8"]).any(-1)[0]
            line += f"; x8 pixels differ {int(dx8.sum())}"
            # do the wrong values look like another frame's warp (stale data) or garbage?
            wrong = r["wf"][0][d][:4].tolist()
            right = wf2[0][d][:4].tolist()
            line += f"; wrong {wrong} right {right}"
        print(line + f"; ptrs {[hex(p) for p in r['ptr']]}", flush=True)

# LOCATE=6's reads before the kernel hid it. LOCATE=7 keeps LOCATE=5's timing (checksums only
# AFTER each reconstruction op) and, after the warp/assemble kernel, also copies its inputs and
# output: a wrong output next to unchanged inputs means the kernel read wrong data
if os.environ.get("LOCATE", "0") in ("7", "8", "9"):
    m = job.model
    state = {"in_rec": False}
    sums, mcrec = [], []

    def isum(t):
        return t.view(torch.int32).sum(dtype=torch.int64)

    def _tensors(o):
        if torch.is_tensor(o):
            return [o]
        if isinstance(o, (tuple, list)):
            return [t for v in o for t in _tensors(v)]
        return []

    def ck(name, fn):
        def w(*a, **kw):
            out = fn(*a, **kw)
            if state["in_rec"]:
                for t in _tensors(out):
                    if t.dtype == torch.float32 and t.is_contiguous():
                        sums[-1].append((name, isum(t)))
                if name == "mc_assemble":
                    ref, mv = a
                    mcrec.append(dict(sref=isum(ref), smv=isum(mv), ref=ref.clone(), mv=mv.clone(),
                                      wf=out[0].clone(), x8=out[1].clone(),
                                      ptr=dict(ref=ref.data_ptr(), mv=mv.data_ptr(), wf=out[0].data_ptr(),
                                               x8=out[1].data_ptr())))
            return out
        return w

    orig_rec = m.reconstruct

    def rec_wrap(lat, referframe):
        sums.append([])
        state["in_rec"] = True
        try:
            return orig_rec(lat, referframe)
        finally:
            state["in_rec"] = False

    patches = [(K.PackedConv, "__call__"), (K.PackedConv, "call_pool"), (K.PackedConv, "call_tap"),
               (K.TapConsumer, "gather"), (K, "upsample2x_add"), (K, "mc_assemble"), (K, "nchw_to_nhwc")]
    saved_fns = [(o, n, getattr(o, n)) for o, n in patches]
    for o, n, f in saved_fns:
        setattr(o, n, ck(n, f))
    m.reconstruct = rec_wrap
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(m, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    m.reconstruct = orig_rec
    for o, n, f in saved_fns:
        setattr(o, n, f)
    bad = [t for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print("decoder mismatching frames (0-based):", bad[:6], flush=True)
    mc = K.mc_assemble
    for t, r in enumerate(mcrec[:12 if os.environ["LOCATE"] == "7" else 6]):
        s = sums[t]
        # checksums of ref4 (op 0) and of the flow (the gather just before the assemble) when made
        i_mc = [n for n, _ in s].index("mc_assemble")
        ref_ok = int(s[0][1]) == int(r["sref"])
        mv_ok = int(s[i_mc - 1][1]) == int(r["smv"])
        wf2, x82 = mc(r["ref"], r["mv"])
        torch.cuda.synchronize()
        same = torch.equal(wf2, r["wf"]) and torch.equal(x82, r["x8"])
        line = f"frame {t}: ref unchanged {ref_ok}, flow unchanged {mv_ok}; output == replay from them: {same}"
        if not same:
            d = (wf2 != r["wf"]).any(-1)[0]
            ys, xs = torch.nonzero(d, as_tuple=True)
            W = d.shape[1]
            flat = ys * W + xs
            line += (f"; {int(d.sum())} px differ, rows {int(ys.min())}..{int(ys.max())}, cols {int(xs.min())}.."
                     f"{int(xs.max())}, flat {int(flat.min())}..{int(flat.max())}; x8 px differ "
                     f"{int((x82 != r['x8']).any(-1)[0].sum())}")
            line += f"; wrong {r['wf'][0][d][:3].tolist()} right {wf2[0][d][:3].tolist()}"
            # the ref half of x8 (a plain copy of ref, no gather) -- wrong too?
            line += f"; x8 ref-half differs {int((x82[..., 3:6] != r['x8'][..., 3:6]).any(-1).sum())}"
            # clusters: distinct 4096-pixel (64 KB of warpframe) pages touched
            line += f"; 64KB pages {len(set((flat // 4096).tolist()))}"
        print(line, flush=True)

    # LOCATE=8: are the wrong values the bilinear warp with some taps read from the memory's
    # PREVIOUS content (stale cached lines), i.e. what an earlier frame's tensor held at that address?
    if os.environ["LOCATE"] == "8":
        import itertools
        import numpy as np
        for t, r in enumerate(mcrec[:6]):
            wf2, _ = mc(r["ref"], r["mv"])
            torch.cuda.synchronize()
            d = (wf2 != r["wf"]).any(-1)[0]
            if not bool(d.any()):
                continue
            nbytes = r["ref"].numel() * 4
            a0 = r["ptr"]["ref"]
            prev = None  # the most recent earlier tensor whose memory covered ref's first byte
            for u in range(t - 1, -1, -1):
                for k in ("wf", "x8", "ref", "mv"):
                    pa, tt = mcrec[u]["ptr"][k], mcrec[u][k]
                    if pa <= a0 < pa + tt.numel() * 4:
                        prev = (u, k, pa, tt)
                        break
                if prev:
                    break
            if prev is None:
                print(f"frame {t}: no earlier recorded tensor at the ref's address", flush=True)
                continue
            u, k, pa, tt = prev
            flat = tt.reshape(-1).view(torch.int32)
            off = (a0 - pa) // 4
            n = min(r["ref"].numel(), flat.numel() - off)
            stale = r["ref"].clone().reshape(-1).view(torch.int32)
            stale[:n] = flat[off:off + n]
            stale = stale.view(torch.float32).reshape(r["ref"].shape)[0].double().cpu().numpy()
            fresh = r["ref"][0].double().cpu().numpy()
            mv = r["mv"][0].double().cpu().numpy()
            wrong = r["wf"][0].double().cpu().numpy()
            H, W = d.shape
            ys, xs = [v.cpu().numpy() for v in torch.nonzero(d, as_tuple=True)]
            hits, total, zhits, zt = 0, len(ys), 0, []
            for y, x in zip(ys, xs):
                gx = (-1.0 + 2.0 * x / (W - 1)) + mv[y, x, 0] / ((W - 1) / 2.0)
                gy = (-1.0 + 2.0 * y / (H - 1)) + mv[y, x, 1] / ((H - 1) / 2.0)
                ix = min(max((gx + 1) * W / 2 - 0.5, 0.0), W - 1.0)
                iy = min(max((gy + 1) * H / 2 - 0.5, 0.0), H - 1.0)
                x0, y0 = int(np.floor(ix)), int(np.floor(iy))
                fx, fy = ix - x0, iy - y0
                taps = [(y0, x0, (1 - fx) * (1 - fy)), (y0, x0 + 1, fx * (1 - fy)), (y0 + 1, x0, (1 - fx) * fy),
                        (y0 + 1, x0 + 1, fx * fy)]
                taps = [(a, b, w) for a, b, w in taps if a < H and b < W]
                ok = False
                for mask in itertools.product((0, 1), repeat=len(taps)):
                    v = sum(w * (stale if mk else fresh)[a, b, :3] for (a, b, w), mk in zip(taps, mask))
                    if np.abs(v - wrong[y, x, :3]).max() < 1e-5:
                        ok = True
                        break
                hits += ok
                for mask in itertools.product((0, 1), repeat=len(taps)):
                    if not any(mask):
                        continue
                    v = sum(w * (0.0 if mk else fresh[a, b, :3]) for (a, b, w), mk in zip(taps, mask))
                    if np.abs(v - wrong[y, x, :3]).max() < 1e-5:
                        zhits += 1
                        zt.extend((a * W + b) for (a, b, w), mk in zip(taps, mask) if mk)
                        break
            print(f"frame {t}: ref memory held frame {u}'s {k} before (offset {off} floats); wrong pixels explained "
                  f"by stale taps: {hits} / {total}; by taps that read zeros: {zhits} / {total}", flush=True)
            if zt:
                zt = sorted(set(zt))
                print(f"  zero-read tap pixels (flat, first 24): {zt[:24]}; 16-B pixel -> 128-B line: "
                      f"{sorted(set(v // 8 for v in zt))[:24]}", flush=True)

    # LOCATE=9: is a wrong pixel exactly the warp of this frame's reference by an EARLIER frame's
    # flow (a stale flow read), or of an earlier frame's reference by this frame's flow?
    if os.environ["LOCATE"] == "9":
        shown = 0
        for t, r in enumerate(mcrec):
            if shown >= 6:
                break
            wf2, _ = mc(r["ref"], r["mv"])
            torch.cuda.synchronize()
            d = (wf2 != r["wf"]).any(-1)
            if not bool(d.any()):
                continue
            n = int(d.sum())
            got_f, got_r = torch.zeros_like(d), torch.zeros_like(d)
            shown += 1
            for u in range(max(0, t - 6), t):
                wu, _ = mc(r["ref"], mcrec[u]["mv"])
                got_f |= d & (wu == r["wf"]).all(-1)
                wu, _ = mc(mcrec[u]["ref"], r["mv"])
                got_r |= d & (wu == r["wf"]).all(-1)
            print(f"frame {t}: {n} wrong px; = this ref warped by an earlier frame's flow: {int(got_f.sum())}; "
                  f"= an earlier ref warped by this flow: {int(got_r.sum())}", flush=True)

# LOCATE=10 (r6): LOCATE=7's timing, plus (a) the pointer range and stream of every conv / HBM op
# of every stream while the GOP runs, and (b) per wrong pixel of the first bad frames: the flow,
# the four taps (pixel index, byte address, bilinear weight, the value memory holds), the wrong and
# the right output, and which single-cause models reproduce the wrong value: a tap read as zeros
# (any subset, whole 16 B), a dword read as zero (per channel), a zero flow component. Written to
# gpurun_out/race10_<tag>.json for offline analysis.
if os.environ.get("LOCATE", "0") == "10":
    import itertools
    import json
    import numpy as np
    m = job.model
    state = {"in_rec": False, "frame": -1}
    mcrec, opsrec = [], []

    def _tensors(o):
        if torch.is_tensor(o):
            return [o]
        if isinstance(o, (tuple, list)):
            return [t for v in o for t in _tensors(v)]
        return []

    def rng(t):
        return [t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()]

    def ck(name, fn):
        def w(*a, **kw):
            out = fn(*a, **kw)
            sid = torch.cuda.current_stream().cuda_stream
            ins = [rng(t) for t in _tensors(list(a)) if t.is_cuda]
            outs = [rng(t) for t in _tensors(out) if t.is_cuda]
            opsrec.append(dict(name=name, stream=sid, rec=state["in_rec"], frame=state["frame"], ins=ins, outs=outs))
            if state["in_rec"] and name == "mc_assemble":
                ref, mv = a
                mcrec.append(dict(ref=ref.clone(), mv=mv.clone(), wf=out[0].clone(), frame=state["frame"],
                                  op_index=len(opsrec) - 1, ptr=ref.data_ptr()))
            return out
        return w

    orig_rec = m.reconstruct

    def rec_wrap(lat, referframe):
        state["frame"] += 1
        state["in_rec"] = True
        try:
            return orig_rec(lat, referframe)
        finally:
            state["in_rec"] = False

    patches = [(K.PackedConv, "__call__"), (K.PackedConv, "call_pool"), (K.PackedConv, "call_tap"),
               (K.TapConsumer, "gather"), (K, "upsample2x_add"), (K, "mc_assemble"), (K, "nchw_to_nhwc"),
               (K, "spynet_assemble"), (K, "avgpool2")]
    saved_fns = [(o, n, getattr(o, n)) for o, n in patches]
    for o, n, f in saved_fns:
        setattr(o, n, ck(n, f))
    m.reconstruct = rec_wrap
    K.x3_overflow(reset=True)
    bss, dec, _, enc = encode_decode_gop(m, job.frames, check=True, overlap=True)
    torch.cuda.synchronize()
    m.reconstruct = orig_rec
    for o, n, f in saved_fns:
        setattr(o, n, f)
    bad = [t for t, (a, b) in enumerate(zip(dec, enc)) if not torch.equal(a, b)]
    print("decoder mismatching frames (0-based):", bad[:8], flush=True)
    mc = K.mc_assemble
    report = dict(lib=os.environ.get("FVC_LIB_PATH", "product"), bad=bad[:16], frames=[])
    summary = {"px": 0, "zero_tap": 0, "zero_dword": 0, "flow0": 0, "unexplained": 0}
    for r in mcrec[:8]:
        wf2, _ = mc(r["ref"], r["mv"])
        torch.cuda.synchronize()
        d = (wf2 != r["wf"]).any(-1)[0]
        if not bool(d.any()):
            continue
        ref = r["ref"][0].double().cpu().numpy()
        mvv = r["mv"][0].double().cpu().numpy()
        wrong = r["wf"][0].double().cpu().numpy()
        right = wf2[0].double().cpu().numpy()
        H, W = d.shape
        ys, xs = [v.cpu().numpy() for v in torch.nonzero(d, as_tuple=True)]
        base = r["ptr"]
        # ops of any stream launched between the previous reconstruct's mc and this one (program order)
        lo = max([q["op_index"] for q in mcrec if q["op_index"] < r["op_index"]] + [0])
        window = [dict(name=o["name"], stream=o["stream"], rec=o["rec"], ins=o["ins"], outs=o["outs"])
                  for o in opsrec[lo:r["op_index"] + 1]]
        pxs = []
        for y, x in zip(ys, xs):
            fx, fy = mvv[y, x, 0], mvv[y, x, 1]

            def taps_of(fx, fy):
                gx = (-1.0 + 2.0 * x / (W - 1)) + fx / ((W - 1) / 2.0)
                gy = (-1.0 + 2.0 * y / (H - 1)) + fy / ((H - 1) / 2.0)
                ix = min(max((gx + 1) * W / 2 - 0.5, 0.0), W - 1.0)
                iy = min(max((gy + 1) * H / 2 - 0.5, 0.0), H - 1.0)
                x0, y0 = int(np.floor(ix)), int(np.floor(iy))
                ax, ay = ix - x0, iy - y0
                tt = [(y0, x0, (1 - ax) * (1 - ay)), (y0, x0 + 1, ax * (1 - ay)), (y0 + 1, x0, (1 - ax) * ay),
                      (y0 + 1, x0 + 1, ax * ay)]
                return [(a, b, w) for a, b, w in tt if a < H and b < W]

            taps = taps_of(fx, fy)
            tol = 2e-5
            z_tap = any(np.abs(sum(w * (0.0 if mk else ref[a, b, :3]) for (a, b, w), mk in zip(taps, mask))
                               - wrong[y, x, :3]).max() < tol
                        for mask in itertools.product((0, 1), repeat=len(taps)) if any(mask))
            z_dw = all(any(abs(sum(w * (0.0 if mk else ref[a, b, c]) for (a, b, w), mk in zip(taps, mask))
                               - wrong[y, x, c]) < tol for mask in itertools.product((0, 1), repeat=len(taps)))
                       for c in range(3))
            f0 = False
            for gfx, gfy in ((0.0, 0.0), (0.0, fy), (fx, 0.0)):
                tq = taps_of(gfx, gfy)
                if np.abs(sum(w * ref[a, b, :3] for a, b, w in tq) - wrong[y, x, :3]).max() < tol:
                    f0 = True
            summary["px"] += 1
            summary["zero_tap"] += z_tap
            summary["zero_dword"] += z_dw
            summary["flow0"] += f0
            summary["unexplained"] += not (z_tap or z_dw or f0)
            if len(pxs) < 24:
                pxs.append(dict(y=int(y), x=int(x), flow=[fx, fy],
                                taps=[dict(y=a, x=b, w=w, addr=base + 16 * (a * W + b),
                                           val=ref[a, b, :3].tolist()) for a, b, w in taps],
                                wrong=wrong[y, x, :3].tolist(), right=right[y, x, :3].tolist(),
                                zero_tap=bool(z_tap), zero_dword=bool(z_dw), flow0=bool(f0)))
        # which ranges of other-stream ops hold any wrong tap's address?
        hits = {}
        for pxd in pxs:
            for tp in pxd["taps"]:
                for o in window:
                    for kind in ("ins", "outs"):
                        for lo_, hi_ in o[kind]:
                            if lo_ <= tp["addr"] < hi_ and not (o["rec"] and o["name"] in ("mc_assemble", "nchw_to_nhwc")):
                                key = f"{o['name']}:{kind}:stream{o['stream']}:rec{int(o['rec'])}"
                                hits[key] = hits.get(key, 0) + 1
        fr = dict(frame=r["frame"], wrong_px=int(d.sum()), ref_range=[base, base + r["ref"].numel() * 4],
                  pixels=pxs, alias_hits=hits, window=window)
        report["frames"].append(fr)
        print(f"frame {r['frame']}: {int(d.sum())} wrong px; alias hits {hits}", flush=True)
    print("summary (per wrong pixel, single-cause models):", summary, flush=True)
    report["summary"] = summary
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/race10_{os.environ.get('TAG', 'x')}.json", "w") as f:
        json.dump(report, f)
