"""Audit a hipcc -save-temps .s of fvc_conv_wino.hip for the MFMA-operand wait states the inline-asm
blocks rely on (the MFMAs inside inline-asm strings; hipcc pads its own builtin MFMAs): no VALU /
v_accvgpr_write may write an MFMA source (A, B) within 2 wait states before it (cdna_hip_programming.md §5.7 item 2), and no non-MFMA instruction may read or write an
MFMA destination within 12 states after it unless an MFMA accumulate chain takes it. Counts one
state per instruction and N+1 per s_nop N (a lower bound on the hardware's distance).

usage: python scripts/check_wino_hazards.py path/to/fvc_conv_wino-hip-amdgcn-amd-amdhsa-gfx950.s
"""
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(4) is not None:
            out.add((k, int(m.group(4))))
        else:
            out.update((k, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(lines):
    """(opcode, operands, text, inside an inline-asm block) per instruction."""
    ins = []
    in_asm = False
    for l in lines:
        if ";;#ASMSTART" in l:
            in_asm = True
        elif ";;#ASMEND" in l:
            in_asm = False
        t = l.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        op, _, rest = t.partition(" ")
        ops = [x.strip() for x in rest.split(",")] if rest else []
        ins.append((op, ops, t, in_asm))
    return ins


def check(body):
    ins = parse(body.splitlines())
    bad = []
    for k, (op, ops, t, asm) in enumerate(ins):
        # hipcc pads its own MFMAs (builtins) through its hazard recognizer; only the MFMAs inside
        # inline-asm strings are hand-padded
        if not op.startswith("v_mfma") or not asm:
            continue
        src = regs(ops[1]) | regs(ops[2])
        dist = 0
        for j in range(k - 1, -1, -1):
            pop, pops, pt, _ = ins[j]
            if dist >= 2:
                break
            if (pop.startswith("v_") and not pop.startswith("v_mfma")) and pops and regs(pops[0]) & src:
                bad.append(f"VALU write -> MFMA source within {dist} states: '{pt}' then '{t}'")
            if pop.startswith("s_nop"):
                dist += int(pop == "s_nop" and pops[0], 0) + 1 if pops else 1
            elif pop.startswith("s_waitcnt") or pop.startswith("s_barrier"):
                dist += 1
            else:
                dist += 1
        dst = regs(ops[0])
        dist = 0
        for j in range(k + 1, len(ins)):
            nop_, nops, nt, _ = ins[j]
            if dist >= 12:
                break
            if nop_.startswith("v_mfma"):
                if regs(nops[0]) & dst and nops[3] == ops[0]:
                    break  # accumulate chain takes it over
                if (regs(nops[1]) | regs(nops[2])) & dst:
                    bad.append(f"MFMA dst read as source within {dist} states: '{t}' then '{nt}'")
            elif nop_.startswith(("v_", "ds_", "global_", "buffer_")) and regs(" ".join(nops)) & dst:
                bad.append(f"MFMA dst touched within {dist} states: '{t}' then '{nt}'")
                break
            if nop_ == "s_nop":
                dist += int(nops[0], 0) + 1
            elif nop_.startswith("s_cbranch") or nop_.startswith("s_branch"):
                break
            else:
                dist += 1
    return bad


def main(path):
    s = open(path).read()
    names = re.findall(r"^(_Z\S*conv_wino_kernel\S*):", s, re.M)
    nbad = 0
    for n in names:
        start = s.index(n + ":")
        end = s.index(".Lfunc_end", start)
        bad = check(s[start:end])
        nbad += len(bad)
        print(f"{n[:70]}: {len(bad)} hazards")
        for b in bad[:10]:
            print("   ", b)
    return 1 if nbad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
