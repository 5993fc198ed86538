"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output per kernel."""
import re, subprocess, sys
import glob
out = ""
files = sys.argv[1:] or sorted(glob.glob("preganplus_amd/csrc/*.hip"))
for f in files:
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-o", "/tmp/pgp_k.o",
           f, "-Rpass-analysis=kernel-resource-usage"]
    out += subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s*(.+?): (.+?) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    print(f"{r['name'][:60]:60s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>4} "
          f"spillV {r.get('VGPRs Spill','?'):>3} occ {r.get('Occupancy [waves/SIMD]','?'):>2} "
          f"LDS {r.get('LDS Size [bytes/block]','?'):>6} SGPR {r.get('TotalSGPRs','?')}")
