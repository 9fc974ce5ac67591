"""Generate the LSVC tree-graph fixture by running the REFERENCE's own graph helpers (build
container only).

Run from the repo root:  python tests/golden/gen_tree_golden.py

Imports /root/reference/models.py and calls ``generate_graph`` (models.py:683-728),
``graph_from_batch`` (models.py:923-940) and ``refidx_from_graph`` (models.py:942-949). The
module's import-time dependencies that are absent here (cv2, torchvision, compressai,
pytorch_msssim, torchac, super_precision) are satisfied by permissive stand-in modules whose
attributes are placeholder classes; none of them is called by these three functions. Output:
tests/golden/tree_graphs.json (plain data: graphs with int keys written as strings). The
reference never leaves this container; only the data file is committed.
"""
import importlib.abc
import importlib.machinery
import json
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "tests", "golden", "tree_graphs.json")
sys.dont_write_bytecode = True

import torch.nn as nn  # noqa: E402

_STUB_ROOTS = {"cv2", "torchvision", "compressai", "pytorch_msssim", "torchac", "super_precision"}


class _Placeholder(nn.Module):
    def __init__(self, *a, **k):
        super().__init__()


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Placeholder


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if fullname.split(".")[0] in _STUB_ROOTS:
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _StubModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


def main():
    sys.meta_path.insert(0, _StubFinder())
    sys.path.insert(0, "/root/reference")
    cwd = os.getcwd()
    os.chdir("/root/reference")
    try:
        import models as M
    finally:
        os.chdir(cwd)
    out = {"generate_graph": {}, "graph_from_batch": {}, "refidx_from_graph": {}}
    enc = lambda g: {str(k): v for k, v in g.items()}
    for kind in ("default", "onehop", "2layers", "3layers", "4layers", "5layers"):
        g, layers, parents = M.generate_graph(kind)
        out["generate_graph"][kind] = {"g": enc(g), "layers": layers, "parents": enc(parents)}
    for bs in range(1, 31):
        for lin, one in ((False, False), (True, False), (False, True)):
            g, layers, parents = M.graph_from_batch(bs, isLinear=lin, isOnehop=one)
            key = f"{bs}{'-L' if lin else ''}{'-O' if one else ''}"
            out["graph_from_batch"][key] = {"layers": layers, "parents": enc(parents)}
            out["refidx_from_graph"][key] = M.refidx_from_graph(g, bs)
    try:
        M.graph_from_batch(31)
        out["graph_from_batch_31"] = "returned"
    except Exception as e:  # the reference prints and then fails on an unbound name
        out["graph_from_batch_31"] = type(e).__name__
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
