"""Phase timing of the GOBI kernel (pgp_gobi.hip), workgroup 0, summed over a run.

  make variant NAME=gprof VFLAGS=-DPGP_GOBI_PROF          (here, before the call)
  PGP_LIB=preganplus_amd/_lib/var/libpreganplus_gprof.so python tools/gobi_phases.py
Phases: 0 layer 1, 1 layer 2, 2 layer 3, 3 head, 4 dh2, 5 dh1, 6 dx + AdamW +
one-hot, 7 prologue (weights, init); slot 15 = iterations of workgroup 0.
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
    buf = (ctypes.c_ulonglong * 16)()
    L.pgp_gobi_prof_read(ctypes.addressof(buf))
    its = buf[15]
    us = {NAMES[i]: buf[i] * 0.01 / n for i in range(8)}
    per_it = {k: (v / its if k != "prologue" else v) for k, v in us.items()}
    total = sum(us.values())
    print(f"iterations of workgroup 0: {its}; total {total:.1f} us per launch")
    for k, v in us.items():
        print(f"  {k:16s} {v:9.1f} us/launch  {per_it[k]:7.2f} us/iteration")
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/gobi_phases.json", "w") as f:
        json.dump({"iterations_wg0": its, "us_per_launch": us, "us_per_iteration": per_it}, f)


if __name__ == "__main__":
    main()
