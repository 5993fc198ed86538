"""Where one PreGANPlusRecovery.run_model call spends its time (host clock,
GPU synchronised around each section), on the recorded plugin intervals."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from preganplus_amd import weights as W  # noqa: E402
from preganplus_amd.recovery import PreGANPlusRecovery  # noqa: E402

w, extra = W.load_npz(os.path.join(ROOT, "preganplus_amd/data/simulator_16.npz"))
z = np.load(os.path.join(ROOT, "tests/golden/plugin_h16.npz"))
tr = extra["train_time_data"]
rec = PreGANPlusRecovery(16, "", training=True, weights=w, extra=extra)
acc = {}


def timed(name, fn):
    def wrap(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
        return r
    return wrap


for name in ("train_gan", "_tune_launch", "_tune_finish", "sync_inference_weights", "recover_decision", "input_window"):
    setattr(rec, name, timed(name, getattr(rec, name)))
rec.infer.forward = timed("forward", rec.infer.forward)
N = 40
for k in range(N + 4):
    if k == 4:
        acc.clear()
        t_all = time.perf_counter()
    step = k % 4
    rec.setEnvironment(bench._plugin_env(z, step, tr))
    rec.run_model(None, [tuple(x) for x in z[f"s{step}/decision_in"]])
torch.cuda.synchronize()
tot = (time.perf_counter() - t_all) / N * 1e3
print(f"run_model {tot:.3f} ms/call")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:24s} {v / N * 1e3:.3f} ms")
