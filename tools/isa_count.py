"""Count instructions per host-loop iteration of the encoder kernel (K2) in the
BUILT library: the gfx950 code objects are unbundled from
preganplus_amd/_lib/libpreganplus.so (llvm-objdump --offloading, in a scratch
directory) and disassembled.  The host loop is `#pragma unroll 1` and holds all
of the kernel's MFMAs, so the kernel-wide v_mfma count is the per-host count.
These counts are preganplus_amd/roofline.py ENC_MFMA_PER_HOST (bench.py's
executed-work `frac`); tests/test_roofline_isa.py holds the two equal.
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


def encoder_counts(Hs=(16, 50), lib=LIB):
    """{H: (mfma, other_valu)} for encoder_kernel<H> in the built library."""
    with tempfile.TemporaryDirectory() as td:
        shutil.copy(lib, os.path.join(td, "lib.so"))
        subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=td, check=True, capture_output=True)
        asm = ""
        for co in sorted(glob.glob(os.path.join(td, "lib.so.*gfx950"))):
            d = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                               text=True).stdout
            if "encoder_kernel" in d:
                asm += d
    out = {}
    for H in Hs:
        m = re.search(rf"<_ZN3pgp12_GLOBAL__N_114encoder_kernelILi{H}EEEvNS_7FwdArgsE>:\n(.*?)s_endpgm", asm, re.S)
        if m is None:
            raise RuntimeError(f"encoder_kernel<{H}> not found in {lib}")
        body = m.group(1)
        mfma = len(re.findall(r"^\s+v_mfma", body, re.M))
        valu = len(re.findall(r"^\s+v_", body, re.M)) - mfma
        out[H] = (mfma, valu)
    return out


if __name__ == "__main__":
    Hs = [int(h) for h in sys.argv[1:]] or [16, 50]
    for H, (mfma, valu) in encoder_counts(Hs).items():
        print(f"H={H}: {mfma} MFMA (16x16x4 f32), {valu} other VALU per host and wave")
