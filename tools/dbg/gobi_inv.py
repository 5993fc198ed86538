"""GOBI batch invariance probe: each environment's result, iteration count and
fitness from sub-batches (1, 3, 65 envs) against the full 240-env batch, and
the per-step pre-projection values (max_iters 1-4) of env 7 alone vs in the
batch.  usage: [PGP_LIB=...] python tools/dbg/gobi_inv.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from preganplus_amd.gobi import GOBIOptimizer  # noqa: E402


def main():
    z = np.load("tests/golden/gobi_h16.npz")
    g = GOBIOptimizer()
    full = [t.cpu().numpy() for t in g.optimize(z["inits"])]
    for sl in (slice(7, 8), slice(100, 103), slice(0, 65)):
        part = [t.cpu().numpy() for t in g.optimize(z["inits"][sl])]
        bad = [i for i in range(part[0].shape[0]) if not np.array_equal(part[0][i], full[0][sl][i])]
        print(sl, "result mismatches", bad, "its", part[1][:4], full[1][sl][:4], "fit", part[2][:2], full[2][sl][:2])
    for step in range(1, 6):
        pf = torch.empty((240, 16, 16), device="cuda")
        p1 = torch.empty((1, 16, 16), device="cuda")
        g.optimize(z["inits"], max_iters=step, pre=pf)
        g.optimize(z["inits"][7:8], max_iters=step, pre=p1)
        a, b = pf.cpu().numpy()[7], p1.cpu().numpy()[0]
        d = np.argwhere(a != b)
        print("step", step, "pre mismatches", len(d), d[:4].tolist(), (a[tuple(d[0])], b[tuple(d[0])]) if len(d) else "")


if __name__ == "__main__":
    main()
