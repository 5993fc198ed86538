"""Count instructions per host-loop iteration of the encoder kernel (K2) in the
BUILT library: the gfx950 code objects are unbundled from
preganplus_amd/_lib/libpreganplus.so (llvm-objdump --offloading, in a scratch
directory) and disassembled.  The host loop is `#pragma unroll 1` and holds all
of the kernel's MFMAs, so the kernel-wide v_mfma count is the per-host count.
These counts are preganplus_amd/roofline.py ENC_MFMA_PER_HOST (bench.py's
executed-work `frac`); tests/test_roofline_isa.py holds the two equal.  The same
holds for the fused tuning-encoder kernels' per-unit counts (TUNE_MFMA_PER_UNIT).
usage: python tools/isa_count.py [H ...]"""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "preganplus_amd", "_lib", "libpreganplus.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _disasm(lib, needle):
    """Disassembly of the library's gfx950 code objects that mention `needle`."""
    with tempfile.TemporaryDirectory() as td:
        shutil.copy(lib, os.path.join(td, "lib.so"))
        subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=td, check=True, capture_output=True)
        asm = ""
        for co in sorted(glob.glob(os.path.join(td, "lib.so.*gfx950"))):
            d = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                               text=True).stdout
            if needle in d:
                asm += d
    return asm


def tune_counts(Hs=(16, 50), lib=LIB, op="_f32_16x16x4"):
    """{H: {kernel: mfma}} for the fused tuning-encoder kernels (pgp_tunef.hip),
    MFMAs of opcode suffix `op` (the split forms' bf16: "_f32_16x16x32_bf16"):
    the unit loop is `#pragma unroll 1` and holds every MFMA, so the static
    count is the per-unit count (tf_fwd_kernel's includes layer 0's time
    encoder, which layer 1 skips)."""
    asm = _disasm(lib, "tf_fwd_kernel")
    out = {}
    for H in Hs:
        out[H] = {}
        for name in ("tf_fwd_kernel", "tf_bwd_ffn_kernel", "tf_bwd_att_kernel"):
            m = re.search(rf"<_ZN3pgp12_GLOBAL__N_1\d+{name}ILi{H}EEEvNS_6TfArgsE>:\n(.*?)s_endpgm", asm, re.S)
            if m is None:
                raise RuntimeError(f"{name}<{H}> not found in {lib}")
            out[H][name] = len(re.findall(r"^\s+v_mfma" + op, m.group(1), re.M))
    return out


def _encoder_body(asm, H, split, lib):
    m = re.search(rf"<_ZN3pgp12_GLOBAL__N_114encoder_kernelILi{H}ELb{int(split)}EEEvNS_7FwdArgsE>:\n(.*?)s_endpgm",
                  asm, re.S)
    if m is None:
        raise RuntimeError(f"encoder_kernel<{H}, {split}> not found in {lib}")
    return m.group(1)


def encoder_counts(Hs=(16, 50), lib=LIB):
    """{H: (mfma, other_valu)} for encoder_kernel<H> (the fp32 form) in the built library."""
    asm = _disasm(lib, "encoder_kernel")
    out = {}
    for H in Hs:
        body = _encoder_body(asm, H, False, lib)
        mfma = len(re.findall(r"^\s+v_mfma", body, re.M))
        valu = len(re.findall(r"^\s+v_", body, re.M)) - mfma
        out[H] = (mfma, valu)
    return out


def encoder_split_counts(Hs=(50,), lib=LIB):
    """{H: (f32 16x16x4 MFMAs, bf16 16x16x32 MFMAs, other VALU)} per host and
    wave of the split-feed-forward form encoder_kernel<H, true>."""
    asm = _disasm(lib, "encoder_kernel")
    out = {}
    for H in Hs:
        body = _encoder_body(asm, H, True, lib)
        f32 = len(re.findall(r"^\s+v_mfma_f32_16x16x4", body, re.M))
        bf = len(re.findall(r"^\s+v_mfma_f32_16x16x32_bf16", body, re.M))
        valu = len(re.findall(r"^\s+v_", body, re.M)) - len(re.findall(r"^\s+v_mfma", body, re.M))
        out[H] = (f32, bf, valu)
    return out


_ASM_CACHE = {}


def _all_asm(lib):
    """Disassembly of every gfx950 code object of `lib` (cached per path and mtime)."""
    key = (os.path.abspath(lib), os.path.getmtime(lib))
    if key not in _ASM_CACHE:
        _ASM_CACHE[key] = _disasm(lib, "")
    return _ASM_CACHE[key]


def kernel_isa_hash(name, H=None, lib=LIB, targs=None):
    """sha256 of kernel `name` (template argument H if given) as BUILT in `lib`:
    its instruction text with addresses and encodings stripped, so it changes
    when that kernel's code changes and not when another kernel moves it.  The
    PMC traffic files (profiles/pmc_*.json) carry it; bench.py reports a
    file's traffic only while the loaded library's kernel still hashes the
    same.  None when the kernel is not found."""
    import hashlib
    asm = _all_asm(lib)
    # targs: every integer template argument (e.g. gan_kernel<16, 16>: the same
    # H has several instantiations); otherwise the first whose first is H
    if targs:
        targ = "I" + "".join(f"Lb{int(t)}E" if isinstance(t, bool) else f"Li{int(t)}E" for t in targs) + "E"
    else:
        targ = rf"ILi{H}E" if H is not None else ""
    m = re.search(rf"^[0-9a-f]+ <(_ZN3pgp12_GLOBAL__N_1\d+{name}{targ}[^>]*)>:\n(.*?)(?=^[0-9a-f]+ <|\Z)", asm,
                  re.S | re.M)
    if m is None:
        return None
    lines = []
    for line in m.group(2).splitlines():
        t = line.split("//")[0].strip()
        # the last kernel of a code object runs into the next object's header,
        # which names the temporary file: not part of the kernel
        if t and "file format" not in t and not t.startswith("Disassembly of section"):
            lines.append(re.sub(r"\s+", " ", t))
    return hashlib.sha256("\n".join(lines).encode()).hexdigest()


if __name__ == "__main__":
    Hs = [int(h) for h in sys.argv[1:]] or [16, 50]
    for H, (mfma, valu) in encoder_counts(Hs).items():
        print(f"H={H}: {mfma} MFMA (16x16x4 f32), {valu} other VALU per host and wave")
    for H, (f32, bf, valu) in encoder_split_counts([h for h in Hs if h == 50]).items():
        print(f"H={H} split FFN: {f32} MFMA 16x16x4 f32 + {bf} MFMA 16x16x32 bf16, {valu} other VALU per host and wave")
    for H, d in tune_counts(Hs).items():
        print(f"H={H}: fused tuning kernels, MFMA per unit: {d}")


def load_cover(name, H, lib=LIB):
    """For each vector-memory load of kernel `name`<H> (program order), the
    MFMAs issued between the load and the s_waitcnt that first requires it
    (vmcnt counts loads and stores in order: `vmcnt(N)` requires all but the
    newest N).  A prefetch whose value is selected right after the load shows
    0 here (the compiler waits at once)."""
    asm = _disasm(lib, name)
    m = re.search(rf"<_ZN3pgp12_GLOBAL__N_1\d+{name}ILi{H}EE[^>]*>:\n(.*?)s_endpgm", asm, re.S)
    if m is None:
        raise RuntimeError(f"{name}<{H}> not found in {lib}")
    pend, cover = [], []  # pend: [is_load, mfma_since]
    for line in m.group(1).splitlines():
        t = line.strip().split("//")[0].strip()
        op = t.split(" ")[0] if t else ""
        if op.startswith("v_mfma"):
            for p in pend:
                p[1] += 1
        elif op.startswith(("global_load", "buffer_load")):
            pend.append([True, 0])
        elif op.startswith(("global_store", "buffer_store", "global_atomic")):
            pend.append([False, 0])
        elif op == "s_waitcnt":
            w = re.search(r"vmcnt\((\d+)\)", t)
            if w:
                n = int(w.group(1))
                while len(pend) > n:
                    p = pend.pop(0)
                    if p[0]:
                        cover.append(p[1])
    return cover
