"""Measure the REFERENCE's own cross-backend behaviour at full size (build container only).

Run from the repo root:  python tests/golden/gen_fullsize_parity.py [4k|1080|all]

It imports the reference DVC forward exactly as ``gen_golden.py`` does (same stubs, same CPU
``torch_warp``) with the build's seeded weights and synthetic frames, and runs it
under several CPU backends:

* ``onednn8`` -- the default: oneDNN convolutions, 8 threads (the anchor every other run is
  compared with);
* ``onednn1`` / ``onednn4`` -- the same on 1 / 4 threads;
* ``chlast``  -- oneDNN on channels_last tensors (a different oneDNN kernel family);
* ``native``  -- oneDNN off: ATen's im2col + MKL GEMM convolution (``slow_conv2d``). Its im2col
  buffer for SpyNet's 7x7 64->32 layer at 4K is 105 GB, so every Conv2d runs on output-row bands
  of <= 2 GB of im2col (explicit zero padding, then padding 0 per band). The GEMM's blocking
  follows the band width, so banding moves outputs by ulps (128x192: 0 flips, max |d clipped|
  3e-6); ``native_unbanded`` at 1080p frame 1 records the unbanded run beside it;
* ``fp64``    -- the reference modules in float64 (same banded native convs): the exact-math
  anchor; its distance from ``onednn8`` is the fp32 rounding floor of any implementation.

Outputs ``tests/golden/ref_fullsize_parity.json``:

* ``k4_frame1``: BASELINE configs[3]'s first P-frame (3840x2160 -> 2176, GOP-32, GOP id 2 = the
  frames ``tests/test_gpu_configs.py::test_4k_gop32_one_rank_share`` codes): per backend the
  per-latent symbol flips against ``onednn8``, dPSNR and relative dbpp;
* ``p1080_frame1``: the same at 1920x1080 -> 1088 (GOP id 0, frame 1);
* ``p1080_gop12``: BASELINE configs[2]'s closed loop -- one 1080p GOP-12 (GOP id 0) through the
  ``parallel_compression`` DVC-pretrained loop (``models.py:368-383``; frame 0 passed through as the
  I-frame), per backend (``onednn8``, ``native``, ``fp64``, ``chlast``, ``onednn4``, ``onednn1``) and per P-frame: PSNR
  (``models.py:379``), bpp and its three parts, symbol statistics, and the flips / PSNR drift
  against the ``onednn8`` chain.

The reference never leaves this container; only the JSON is committed.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (shims + reference import; chdir /root/reference)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fastvideocodec_amd.synthetic import gop_seed, make_gop  # noqa: E402
from fastvideocodec_amd.weights import seeded_torch_state_dict  # noqa: E402

OUT = os.path.join(G.OUT, "ref_fullsize_parity.json")
BAND_BYTES = 2 << 30
GOP_VARIANTS = ("native", "fp64", "chlast", "onednn4", "onednn1")
LATENTS = (("quant_mv", "mv"), ("compressed_feature", "feature"), ("compressed_z", "z"))

_orig_conv_forward = torch.nn.Conv2d._conv_forward


def _cpu_torch_warp_any_dtype(x, flow):
    """gen_golden's CPU torch_warp with the grid built in x's dtype (identical for float32; the
    float64 run needs a float64 grid for grid_sample)."""
    B, _, H, W = flow.shape
    gh = torch.linspace(-1.0, 1.0, W, dtype=x.dtype).view(1, 1, 1, W).expand(B, -1, H, -1)
    gv = torch.linspace(-1.0, 1.0, H, dtype=x.dtype).view(1, 1, H, 1).expand(B, -1, -1, W)
    grid = torch.cat([gh, gv], 1)
    flow = flow.to(x.dtype)
    f = torch.cat([flow[:, 0:1] / ((x.size(3) - 1.0) / 2.0), flow[:, 1:2] / ((x.size(2) - 1.0) / 2.0)], 1)
    return F.grid_sample(x, (grid + f).permute(0, 2, 3, 1), mode="bilinear",
                         padding_mode="border", align_corners=False)


G.E.torch_warp = _cpu_torch_warp_any_dtype


def _banded_conv_forward(self, x, weight, bias):
    """Conv2d on output-row bands (explicit zero padding, padding 0 per band)."""
    if self.padding_mode != "zeros" or self.groups != 1 or tuple(self.dilation) != (1, 1) \
            or isinstance(self.padding, str):
        return _orig_conv_forward(self, x, weight, bias)
    n, c, h, w = x.shape
    kh, kw = self.kernel_size
    sh, sw = self.stride
    ph, pw = self.padding
    ho = (h + 2 * ph - kh) // sh + 1
    wo = (w + 2 * pw - kw) // sw + 1
    row_bytes = n * c * kh * kw * wo * x.element_size()
    rows = max(1, BAND_BYTES // row_bytes)
    if rows >= ho:
        return _orig_conv_forward(self, x, weight, bias)
    xp = F.pad(x, (pw, pw, ph, ph))
    outs = []
    for r0 in range(0, ho, rows):
        r1 = min(ho, r0 + rows)
        outs.append(F.conv2d(xp[:, :, r0 * sh:(r1 - 1) * sh + kh], weight, bias, self.stride, 0))
    return torch.cat(outs, 2)


class Backend:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.threads = torch.get_num_threads()
        self.mkldnn = torch.backends.mkldnn.enabled
        # onednnN: the default oneDNN path on N threads (8 for every other backend)
        torch.set_num_threads(int(self.name[6:]) if self.name.startswith("onednn") else 8)
        if self.name in ("native", "fp64"):
            torch.backends.mkldnn.enabled = False
            torch.nn.Conv2d._conv_forward = _banded_conv_forward
        elif self.name == "native_unbanded":
            torch.backends.mkldnn.enabled = False
        return self

    def __exit__(self, *exc):
        torch.set_num_threads(self.threads)
        torch.backends.mkldnn.enabled = self.mkldnn
        torch.nn.Conv2d._conv_forward = _orig_conv_forward


_models = {}


def model_for(name):
    key = "fp64" if name == "fp64" else "fp32"
    if key not in _models:
        m = G.build()
        if key == "fp64":
            m = m.double()
        _models[key] = m
    return _models[key]


def forward(name, cur, ref):
    """One reference forward under backend ``name``: symbols (numpy float32 NCHW) + scalars."""
    m = model_for(name)
    cur_t, ref_t = torch.from_numpy(cur), torch.from_numpy(ref)
    if name == "fp64":
        cur_t, ref_t = cur_t.double(), ref_t.double()
    if name == "chlast":
        cur_t = cur_t.contiguous(memory_format=torch.channels_last)
        ref_t = ref_t.contiguous(memory_format=torch.channels_last)
        m = m.to(memory_format=torch.channels_last)
    t0 = time.time()
    with Backend(name):
        d = G.run_pair(m, cur_t, ref_t)
    if name == "chlast":
        m.to(memory_format=torch.contiguous_format)
    d["seconds"] = time.time() - t0
    return d


# gen_golden.run_pair takes numpy arrays; accept tensors too (dtype / memory format preserved)
def _run_pair(m, cur, ref):
    acts = {}

    def hook(name):
        def f(mod, inp, out):
            acts[name] = out
        return f

    hs = [getattr(m, n).register_forward_hook(hook(k)) for n, k in
          [("mvEncoder", "mvfeature"), ("resEncoder", "feature"), ("respriorEncoder", "z")]]
    with torch.no_grad():
        out = m(cur, ref)
    for h in hs:
        h.remove()
    d = {"quant_mv": torch.round(acts["mvfeature"]).float().contiguous().numpy(),
         "compressed_feature": torch.round(acts["feature"]).float().contiguous().numpy(),
         "compressed_z": torch.round(acts["z"]).float().contiguous().numpy()}
    names = ["clipped", "mse_loss", "warploss", "interloss", "bpp_feature", "bpp_z", "bpp_mv", "bpp"]
    for n, o in zip(names, out):
        d[n] = o.float().contiguous().numpy() if n == "clipped" else float(o)
    return d


G.run_pair = _run_pair


def psnr(mse):
    # models.py:379: 10 log(1/mse) / log(10) on the fp32 mse the forward returns
    return float(10.0 * np.log10(1.0 / np.float64(np.float32(mse))))


def sym_stats(d):
    s = {}
    for g, short in LATENTS:
        q = d[g]
        s[short] = {"n": int(q.size), "nonzero": int(np.count_nonzero(q)), "abs_sum": int(np.abs(q).sum()),
                    "sha16": hashlib.sha256(np.ascontiguousarray(q, np.int32).tobytes()).hexdigest()[:16]}
    return s


def compare(d, a):
    """Flips of run d against anchor run a, per latent, plus dPSNR / dbpp."""
    fl = {}
    tot = n = 0
    for g, short in LATENTS:
        k = int((d[g] != a[g]).sum())
        fl[short] = k
        n += k
        tot += d[g].size
    fl["total"] = n
    return {"flips": fl, "n_symbols": tot, "flip_rate": n / tot,
            "dpsnr_db": abs(psnr(d["mse_loss"]) - psnr(a["mse_loss"])),
            "dbpp_rel": abs(d["bpp"] - a["bpp"]) / a["bpp"],
            "max_abs_dclipped": float(np.abs(d["clipped"].astype(np.float64) - a["clipped"]).max())}


def frame1(frames, variants, tag):
    cur, ref = frames[1:2].copy(), frames[0:1].copy()
    runs = {}
    res = {"variants": {}}
    for v in variants:
        t0 = time.time()
        runs[v] = forward(v, cur, ref)
        print(f"[{tag}] {v}: {time.time() - t0:.1f}s psnr {psnr(runs[v]['mse_loss']):.6f} "
              f"bpp {runs[v]['bpp']:.6f}", flush=True)
        if v != "onednn8":
            res["variants"][v] = compare(runs[v], runs["onednn8"])
            print(f"[{tag}] {v} vs onednn8: {res['variants'][v]}", flush=True)
        else:
            res["onednn8"] = {"psnr_db": psnr(runs[v]["mse_loss"]), "bpp": runs[v]["bpp"],
                              "symbols": sym_stats(runs[v])}
    return res, runs


def oracle_vs(frames, anchor, tag):
    """The build's oracle restatement (oracle/dvc_ref.py) against the reference at full size."""
    sys.path.insert(0, G.REPO)
    from oracle import dvc_ref
    cur, ref = torch.from_numpy(frames[1:2].copy()), torch.from_numpy(frames[0:1].copy())
    torch.set_num_threads(8)
    t0 = time.time()
    (clip, mse, _, _, bf, bz, bmv, bpp), inter = dvc_ref.forward(seeded_torch_state_dict(), cur, ref,
                                                                return_intermediates=True)
    d = {"quant_mv": inter["quant_mv"].numpy(), "compressed_feature": inter["compressed_feature"].numpy(),
         "compressed_z": inter["compressed_z"].numpy(), "mse_loss": float(mse), "bpp": float(bpp),
         "clipped": clip.numpy()}
    r = compare(d, anchor)
    print(f"[{tag}] oracle/dvc_ref vs onednn8 ({time.time() - t0:.1f}s): {r}", flush=True)
    return r


def gop_chain(frames, name, anchor_chain=None):
    """models.py:368-383: x_prev = data[0]; x_prev = forward(data[i], x_prev)[0] for i >= 1."""
    x_prev = frames[0:1].copy()
    per = []
    runs = []
    for i in range(1, frames.shape[0]):
        t0 = time.time()
        d = forward(name, frames[i:i + 1].copy(), x_prev)
        x_prev = d["clipped"]
        rec = {"frame": i, "psnr_db": psnr(d["mse_loss"]), "mse": float(np.float32(d["mse_loss"])),
               "bpp": d["bpp"], "bpp_mv": d["bpp_mv"], "bpp_z": d["bpp_z"], "bpp_feature": d["bpp_feature"],
               "symbols": sym_stats(d)}
        if anchor_chain is not None:
            a = anchor_chain[i - 1]
            c = compare(d, a)
            rec.update({"vs_onednn8": c})
        runs.append({k: d[k] for k in ("quant_mv", "compressed_feature", "compressed_z", "mse_loss", "bpp",
                                       "clipped")})
        per.append(rec)
        print(f"[gop1080 {name}] frame {i}: {time.time() - t0:.1f}s psnr {rec['psnr_db']:.6f} bpp {rec['bpp']:.6f}"
              + (f" flips {rec['vs_onednn8']['flips']} dpsnr {rec['vs_onednn8']['dpsnr_db']:.3e}"
                 if anchor_chain is not None else ""), flush=True)
    return per, runs


def load():
    if os.path.exists(OUT):
        with open(OUT) as f:
            return json.load(f)
    return {}


def save(res):
    res["generator"] = "tests/golden/gen_fullsize_parity.py"
    res["torch"] = torch.__version__
    res["threads_default"] = 8
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", OUT, flush=True)


def main(which):
    res = load()
    if which == "gop-add":
        # add chains of the GOP_VARIANTS missing from an existing fixture (same anchor chain)
        frames = make_gop(1080, 1920, 12, gop_seed(0))
        g = res["p1080_gop12"]
        _, anchor_runs = gop_chain(frames, "onednn8")
        for v in GOP_VARIANTS:
            if v not in g["chains"]:
                g["chains"][v], _ = gop_chain(frames, v, anchor_runs)
                g["psnr_drift_db"][v] = [c["vs_onednn8"]["dpsnr_db"] for c in g["chains"][v]]
        save(res)
        return
    if which in ("1080", "all"):
        frames = make_gop(1080, 1920, 12, gop_seed(0))
        r, runs = frame1(frames, ["onednn8", "native_unbanded", "native", "onednn1", "chlast", "fp64"], "p1080f1")
        r["oracle_vs_onednn8"] = oracle_vs(frames, runs["onednn8"], "p1080f1")
        r["frames"] = "make_gop(1080, 1920, 12, gop_seed(0)) frames 0 -> 1 (padded to 1088x1920)"
        res["p1080_frame1"] = r
        save(res)
        del runs
        chains = {}
        anchor_per, anchor_runs = gop_chain(frames, "onednn8")
        chains["onednn8"] = anchor_per
        for v in GOP_VARIANTS:
            chains[v], _ = gop_chain(frames, v, anchor_runs)
        drift = {v: [c["vs_onednn8"]["dpsnr_db"] for c in chains[v]] for v in GOP_VARIANTS}
        res["p1080_gop12"] = {"frames": "make_gop(1080, 1920, 12, gop_seed(0)), closed loop models.py:368-383",
                              "chains": chains, "psnr_drift_db": drift}
        save(res)
    if which in ("4k", "all"):
        frames = make_gop(2160, 3840, 32, gop_seed(2))[:2].copy()
        r, runs = frame1(frames, ["onednn8", "native", "chlast", "fp64", "onednn1"], "k4f1")
        r["oracle_vs_onednn8"] = oracle_vs(frames, runs["onednn8"], "k4f1")
        r["frames"] = "make_gop(2160, 3840, 32, gop_seed(2)) frames 0 -> 1 (padded to 2176x3840)"
        res["k4_frame1"] = r
        save(res)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "all")  # 4k | 1080 | all | gop-add
