"""Count instructions per host-loop iteration of the encoder kernel (K2) from the
gfx950 ISA (hipcc --save-temps).  The host loop is `#pragma unroll 1` and holds
all of the kernel's MFMAs, so the kernel-wide v_mfma count is the per-host count.
usage: python tools/isa_count.py [H ...]   (prints MFMA / VALU counts; the MFMA
counts feed preganplus_amd/roofline.py ENC_MFMA_PER_HOST)"""
import os, re, subprocess, sys, tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
Hs = [int(h) for h in sys.argv[1:]] or [16, 50]
with tempfile.TemporaryDirectory() as td:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--save-temps", "-c",
                    "-o", os.path.join(td, "e.o"), os.path.join(ROOT, "preganplus_amd/csrc/pgp_encoder.hip")],
                   cwd=td, check=True, capture_output=True)
    asm = open(os.path.join(td, "pgp_encoder-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
for H in Hs:
    m = re.search(rf"^_ZN3pgp12_GLOBAL__N_114encoder_kernelILi{H}EEEvNS_7FwdArgsE:(.*?)s_endpgm", asm, re.S | re.M)
    body = m.group(1)
    mfma = len(re.findall(r"^\s+v_mfma", body, re.M))
    valu = len(re.findall(r"^\s+v_", body, re.M)) - mfma
    print(f"H={H}: {mfma} MFMA (16x16x4 f32), {valu} other VALU per host and wave")
