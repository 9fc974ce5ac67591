"""CPU: the Winograd kernel's inline-asm MFMA blocks rely on hand-counted wait states
(fvc_conv_wino.hip: VALU writes of MFMA sources >= 2 states before the MFMA, no reader of an MFMA
destination within 12 states). hipcc pads nothing inside an asm statement, so a toolchain or
source change that moves compiler code into those windows would silently corrupt results. This
test compiles the kernel source for gfx950 exactly as the product build does (device assembly
only) and runs scripts/check_wino_hazards.py over every conv_wino_kernel instantiation."""
import importlib.util
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _checker():
    spec = importlib.util.spec_from_file_location("check_wino_hazards",
                                                  os.path.join(REPO, "scripts", "check_wino_hazards.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="hipcc not available")
def test_wino_asm_wait_states(tmp_path):
    from fastvideocodec_amd import build as B
    src = os.path.join(REPO, "fastvideocodec_amd", "csrc", "fvc_conv_wino.hip")
    out = tmp_path / "wino.s"
    flags = [f for f in B.FLAGS if f != "-fPIC"] + B.SRC_FLAGS.get("fvc_conv_wino.hip", [])
    subprocess.run([HIPCC] + flags + ["--cuda-device-only", "-S", src, "-o", str(out)], check=True,
                   stderr=subprocess.DEVNULL)
    s = out.read_text()
    mod = _checker()
    import re
    names = re.findall(r"^(_Z\S*conv_wino_kernel\S*):", s, re.M)
    assert len(names) >= 12, names  # every instantiation the launcher dispatches
    for n in names:
        start = s.index(n + ":")
        bad = mod.check(s[start:s.index(".Lfunc_end", start)])
        assert not bad, (n, bad[:5])


def test_checker_flags_real_hazards():
    """The audit is not vacuous: an asm MFMA whose destination is read right after, and a VALU
    write of an MFMA source right before it, are both reported; a compiler (non-asm) MFMA is not."""
    mod = _checker()
    body = ("\tv_add_f32_e32 v4, v1, v2\n\t;;#ASMSTART\n\tv_mfma_f32_16x16x32_f16 v[0:3], a[0:3], v[4:7], 0\n"
            "\t;;#ASMEND\n\tv_add_f32_e32 v8, v0, v1\n")
    bad = mod.check(body)
    assert any("source" in b for b in bad) and any("dst touched" in b for b in bad), bad
    ok = "\tv_mfma_f32_16x16x32_f16 v[0:3], a[0:3], v[4:7], 0\n\ts_nop 4\n\tv_add_f32_e32 v8, v0, v1\n"
    assert mod.check(ok) == []


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="hipcc not available")
def test_wr7_asm_wait_states(tmp_path):
    """The same audit over every conv_wr7_kernel instantiation (fvc_conv_wr7.hip: inline-asm MFMAs
    with U in AGPRs, the transformed-row ring written by VALU a step before its MFMAs read it)."""
    from fastvideocodec_amd import build as B
    src = os.path.join(REPO, "fastvideocodec_amd", "csrc", "fvc_conv_wr7.hip")
    out = tmp_path / "wr7.s"
    flags = [f for f in B.FLAGS if f != "-fPIC"] + B.SRC_FLAGS.get("fvc_conv_wr7.hip", [])
    subprocess.run([HIPCC] + flags + ["--cuda-device-only", "-S", src, "-o", str(out)], check=True,
                   stderr=subprocess.DEVNULL)
    s = out.read_text()
    mod = _checker()
    import re
    names = re.findall(r"^(_Z\S*conv_wr7_kernel\S*):", s, re.M)
    assert len(names) == 18, names  # nt 1 / 2 x three modes x three activations
    for n in names:
        start = s.index(n + ":")
        body = s[start:s.index(".Lfunc_end", start)]
        bad = mod.check(body)
        assert not bad, (n, bad[:5])
        # U stays in AGPRs: loaded once, never copied in or out by the compiler
        assert "v_accvgpr_write" not in body and "v_accvgpr_read" not in body, n
        assert "scratch_" not in body, n
