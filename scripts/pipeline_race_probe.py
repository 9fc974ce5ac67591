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
