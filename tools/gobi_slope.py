"""Per-iteration cost of the GOBI kernel: time pgp_gobi_optimize with
max_iters in {1, 11, 21, 31} (every environment then runs exactly that many
steps: the stop rule needs >= 31 unchanged ones) for a few batch sizes."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from preganplus_amd.gobi import GOBIOptimizer  # noqa: E402

z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/gobi_h16.npz"))
g = GOBIOptimizer()
for E in (64, 256, 1024):
    inits = torch.tensor(np.concatenate([z["inits"]] * (-(-E // 240)))[:E], device="cuda")
    out = (torch.empty_like(inits), torch.empty(E, dtype=torch.int32, device="cuda"),
           torch.empty(E, dtype=torch.float32, device="cuda"))
    row = []
    for mi in (1, 11, 21, 31):
        for _ in range(3):
            g.optimize(inits, out=out, max_iters=mi)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            g.optimize(inits, out=out, max_iters=mi)
        torch.cuda.synchronize()
        row.append((time.perf_counter() - t0) / 20 * 1e6)
    slope = (row[3] - row[0]) / 30
    print(f"E={E}: us at max_iters 1/11/21/31 = {[round(r, 1) for r in row]}, per iteration {slope:.2f} us", flush=True)
