"""Build libfvc.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo).

Each source compiles to its own object (in parallel, only when stale), then one link step.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
VARIANT_SRCS = ("fvc_conv_x3.hip", "fvc_deconv_x3.hip", "fvc_conv_wino.hip", "fvc_conv_wr7.hip", "fvc_conv_stem.hip",
                "fvc_elem.hip")
SRCS = ["fvc_conv.hip", "fvc_conv_x3.hip", "fvc_deconv_x3.hip", "fvc_conv_wino.hip", "fvc_conv_wr7.hip", "fvc_conv_stem.hip", "fvc_elem.hip", "fvc_coder.hip", "fvc_iframe.hip",
        "fvc_torchac.hip"]
# per-source flags: the Winograd transforms stay scalar f32 (packed f32 VALU issues slower beside MFMAs)
SRC_FLAGS = {"fvc_conv_wino.hip": ["-fno-slp-vectorize"], "fvc_conv_wr7.hip": ["-fno-slp-vectorize"]}
OUT = os.path.join(HERE, "libfvc.so")
OBJDIR = os.path.join(HERE, "build")
HEADERS = [os.path.join(HERE, "csrc", "fvc_common.h"), os.path.join(HERE, "csrc", "fvc_dist.h"),
           os.path.join(HERE, "csrc", "fvc_dx.h"),
           os.path.join(os.path.dirname(HERE), "include", "fvc.h")]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"]


def _hipcc():
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _obj(src, tag=""):
    return os.path.join(OBJDIR, os.path.splitext(src)[0] + tag + ".o")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, verbose, extra=(), tag=""):
    path = os.path.join(HERE, "csrc", src)
    obj = _obj(src, tag)
    cmd = [_hipcc()] + FLAGS + SRC_FLAGS.get(src, []) + list(extra) + ["-c", path, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)


def build(force=False, verbose=True, variant=None, defines=(), only=None):
    """Build libfvc.so; variant="name" with extra -D defines builds an experiment library
    libfvc_<name>.so instead (loaded with FVC_LIB_PATH; never the product)."""
    os.makedirs(OBJDIR, exist_ok=True)
    tag = f"_{variant}" if variant else ""
    out = OUT if not variant else os.path.join(HERE, f"libfvc{tag}.so")
    extra = [f"-D{d}" for d in defines]
    # experiment variants recompile only the conv kernels (the -D switches are theirs) and link
    # the product objects of every other source
    vsrcs = [s for s in SRCS if not variant or (s in VARIANT_SRCS and (not only or s in only))]
    if variant:
        build(force=False, verbose=verbose)
    todo = [s for s in vsrcs if force or _stale(_obj(s, tag), [os.path.join(HERE, "csrc", s)] + HEADERS)]
    if todo:
        with ThreadPoolExecutor(max_workers=min(len(todo), 4)) as ex:
            list(ex.map(lambda s: _compile(s, verbose, extra, tag), todo))
    objs = [_obj(s, tag if s in vsrcs else "") for s in SRCS]
    if force or todo or _stale(out, objs):
        cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", default=None)
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--only", action="append", default=None, help="variant: recompile only these sources")
    a = ap.parse_args()
    build(force=a.force, variant=a.variant, defines=a.defines, only=a.only)
