"""Phase timing of the GOBI kernel (pgp_gobi.hip) per workgroup, summed over a run.

  make variant NAME=gprof VFLAGS=-DPGP_GOBI_PROF          (here, before the call)
  PGP_LIB=preganplus_amd/_lib/var/libpreganplus_gprof.so python tools/gobi_phases.py
Per workgroup (the first 256), wave 0's wall clock: phases 0 layer 1, 1 layer 2,
2 layer 3, 3 head, 4 dh2, 5 dh1, 6 dx + AdamW + one-hot, 7 prologue (weights,
init); slots 8-11 / 12-15 the time / count of iterations with 1-4 active
environments; 16-22 phases 0-6 of the iterations with one active; slot 31 its
iterations.  Printed for workgroup 0 and the
workgroup with the most iterations (the one that sets the launch's time).
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from preganplus_amd import _native  # noqa: E402
from preganplus_amd.gobi import GOBIOptimizer  # noqa: E402

NAMES = ["layer1", "layer2", "layer3", "head", "dh2", "dh1", "dx_adam_onehot", "prologue"]
WG, SLOTS = 256, 32


def main():
    L = _native.lib()
    L.pgp_gobi_prof_read.argtypes = [ctypes.c_void_p]
    z = np.load("tests/golden/gobi_h16.npz")
    E = 1024
    inits = np.concatenate([z["inits"]] * (E // z["inits"].shape[0] + 1))[:E]
    g = GOBIOptimizer()
    x = torch.tensor(inits, device="cuda")
    for _ in range(3):
        g.optimize(x)
    torch.cuda.synchronize()
    L.pgp_gobi_prof_reset.argtypes = []
    L.pgp_gobi_prof_reset()
    n = 10
    for _ in range(n):
        g.optimize(x)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (WG * SLOTS))()
    L.pgp_gobi_prof_read(ctypes.addressof(buf))
    a = np.frombuffer(buf, dtype=np.uint64).reshape(WG, SLOTS).astype(np.float64) / n
    out = {}
    for tag, w in (("workgroup 0", 0), ("slowest workgroup", int(np.argmax(a[:, 31])))):
        its = a[w, 31] * n  # set (not summed) per launch
        us = {NAMES[i]: a[w, i] * 0.01 for i in range(8)}  # 100 MHz wall clock
        print(f"{tag} ({w}): {its:.0f} iterations; {sum(us.values()):.1f} us per launch")
        for k, v in us.items():
            print(f"  {k:16s} {v:9.1f} us/launch  {v / (its if k != 'prologue' else 1):7.2f} us/iteration")
        one = a[w, 12]
        if one:
            print("  phases of the iterations with 1 active (us/iteration): " +
                  ", ".join(f"{NAMES[i]} {a[w, 16 + i] * 0.01 / one:.2f}" for i in range(7)))
        for m in range(1, 5):
            cnt = a[w, 11 + m]
            if cnt:
                print(f"  iterations with {m} active: {cnt:4.0f} x {a[w, 7 + m] * 0.01 / cnt:6.2f} us")
        out[tag] = {"workgroup": w, "iterations": its, "us_per_launch": us,
                    "by_active": {m: [a[w, 11 + m], a[w, 7 + m] * 0.01] for m in range(1, 5)}}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/gobi_phases.json", "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
