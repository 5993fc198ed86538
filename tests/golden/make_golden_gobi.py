"""Golden fixtures for GOBI, the schedule producer of the decision path
(SURVEY §8f row f3): the reference's own optimiser, run here.

  scheduler/GOBI.py:19-42          run_GOBI: init = [host cpu, container ips, one-hot alloc]
  scheduler/BaGTI/src/opt.py:9-33  opt(): AdamW(lr 0.8) + CosineAnnealingLR(T_max 10) on the
                                   input, one-hot projection per step, stop after 31
                                   unchanged steps or 200 iterations
  scheduler/BaGTI/src/models.py:8-27 energy_latency_16 surrogate (288-128-128-64-2)

Imports /root/reference/scheduler/BaGTI (read-only; run with python -B so no
bytecode is written there), loads the shipped checkpoint with
torch.load(weights_only=True), and writes
  tests/golden/gobi_h16.npz                   inits, results, iterations, fitness
  preganplus_amd/data/gobi_energy_latency_16.npz  surrogate weights + max container IPS
Inits: the 200 rows of the reference's own scheduling dataset
(datasets/energy_latency_16_scheduling.csv) mapped as run_GOBI maps a live
environment (unplaced containers get a seeded random host, as GOBI.py:31 draws
one), plus 40 synthetic rows.
"""
import os
import sys

import numpy as np
import torch

REF = "/root/reference/scheduler/BaGTI"
OUT = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(os.path.dirname(os.path.dirname(OUT)), "preganplus_amd", "data")
H = 16


def main():
    sys.path.insert(0, REF)
    sys.argv = ["make_golden_gobi", "-", "-"]  # models.py:25 reads argv[0], argv[2]
    from src.models import energy_latency_16  # noqa: E402
    from src.opt import opt  # noqa: E402

    model = energy_latency_16()
    ck = torch.load(os.path.join(REF, "checkpoints", "energy_latency_16_Trained.ckpt"), weights_only=True,
                    map_location="cpu")
    model.load_state_dict(ck["model_state_dict"])
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}

    data = np.loadtxt(os.path.join(REF, "datasets", "energy_latency_16_scheduling.csv"), delimiter=",")
    max_ips = float(data[:, H:2 * H].max())  # utils.py:61
    rng = np.random.Generator(np.random.PCG64(2024))
    inits = []
    for row in data:
        cpu = row[:H] / 100.0
        cpuc = row[H:2 * H] / max_ips
        alloc = np.zeros((H, H))
        for c in range(H):
            hid = int(row[2 * H + c])
            alloc[c, hid if hid >= 0 else rng.integers(0, H)] = 1.0
        inits.append(np.concatenate([cpu[:, None], cpuc[:, None], alloc], axis=1))
    for _ in range(40):
        cpu = rng.uniform(0, 1, H)
        cpuc = rng.uniform(0, 1, H) * (rng.uniform(size=H) < 0.7)
        alloc = np.zeros((H, H))
        alloc[np.arange(H), rng.integers(0, H, H)] = 1.0
        inits.append(np.concatenate([cpu[:, None], cpuc[:, None], alloc], axis=1))
    inits = np.stack(inits)

    results, iters, fitness = [], [], []
    for x in inits:
        init = torch.tensor(x, dtype=torch.float, requires_grad=True)  # GOBI.py:33
        res, it, fit = opt(init, model, [], "energy_latency_16")
        results.append(res.numpy().copy())
        iters.append(it)
        fitness.append(float(fit))
    np.savez_compressed(os.path.join(OUT, "gobi_h16.npz"), inits=inits.astype(np.float32),
                        results=np.stack(results), iterations=np.array(iters), fitness=np.array(fitness),
                        max_ips=max_ips)
    np.savez_compressed(os.path.join(DATA, "gobi_energy_latency_16.npz"), max_ips=max_ips,
                        **{k: v for k, v in sd.items()})
    print("inits", inits.shape, "iterations min/mean/max", min(iters), np.mean(iters), max(iters))


if __name__ == "__main__":
    main()
