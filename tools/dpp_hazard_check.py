"""Static check of a built kernel's ISA for the DPP read hazard that inline asm
hides from the compiler: a VALU instruction writing a VGPR, followed within 2
wait states by a DPP instruction whose swizzled source (src0) is that VGPR
(CDNA3/4 manual wait states: the DPP reads the value from before the write).

pgp_gobi.hip issues its row_newbcast multiply-adds as inline asm
(v_fmac_f32_dpp); the compiler inserts the wait states for its own DPP
builtins, not for those.  This walks the assembly in program order and, for
every `*_dpp` instruction, looks back for the nearest writer of its src0:
a VALU writer fewer than 2 wait states back (s_nop N counts N + 1) is a
violation; a label inside that window (another predecessor could reach the
DPP) is reported as well, conservatively.

usage: python tools/dpp_hazard_check.py <file.s>   (exit 1 on any finding)
  the .s: hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --offload-device-only
  (basic-block labels kept); also takes llvm-objdump -d text (no block labels:
  tests/test_roofline_isa.py runs it on the built library's gobi_kernel)
"""
import re
import sys

REG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def vgprs(tok):
    m = REG.match(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def parse(lines):
    """(kind, opcode, operands) per line: kind 'label' or 'inst'."""
    out = []
    for raw in lines:
        line = raw.split(";")[0].split("//")[0].strip()
        if not line or line.startswith("."):
            continue
        if line.endswith(":"):  # a basic-block label (.s) or a symbol (llvm-objdump -d)
            out.append(("label", line, []))
            continue
        parts = line.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        out.append(("inst", parts[0], ops))
    return out


def valu_dst(op, ops):
    """VGPRs a VALU instruction writes (its first operand), or the empty set."""
    if not op.startswith("v_") or not ops:
        return set()
    if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    return vgprs(ops[0].split()[0])


def check(path):
    return check_insts(parse(open(path).read().split("\n")))


def check_insts(insts):
    findings = []
    n_dpp = 0
    for i, (kind, op, ops) in enumerate(insts):
        if kind != "inst" or not op.endswith("_dpp") or len(ops) < 2:
            continue
        n_dpp += 1
        src = vgprs(ops[1].split()[0])
        waits = 0
        j = i - 1
        while j >= 0 and waits < 2:
            k, o, a = insts[j]
            if k == "label":
                findings.append((i, op, ops, f"label {o} within 2 wait states"))
                break
            if valu_dst(o, a) & src:
                findings.append((i, op, ops, f"{o} {', '.join(a)} writes the source {waits} wait state(s) back"))
                break
            m = re.match(r"s_nop\s*$", o)
            waits += (int(a[0], 0) + 1) if (m and a) else 1
            j -= 1
    return n_dpp, findings


def main(path):
    n, found = check(path)
    print(f"{path}: {n} DPP instructions, {len(found)} findings")
    for i, op, ops, why in found[:40]:
        print(f"  #{i} {op} {', '.join(ops)}: {why}")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
