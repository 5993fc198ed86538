"""Host enqueue time vs wall time of one backprop() call (10 sequential
batch-1 tuning steps, H=16, recorded plugin windows).  Run under
rocprofv3 --kernel-trace --stats for the device time per kernel."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from preganplus_amd import train as TR, weights as W

w, extra = W.load_npz(os.path.join(ROOT, "preganplus_amd/data/simulator_16.npz"))
z = np.load(os.path.join(ROOT, "tests/golden/tune_h16.npz"))
tr = TR.Trainer(16, w, extra)
st = TR.TuneState(z["protos0"], float(z["factor0"]))
wins, anom, cls = z["windows"], z["anom"], z["cls"]
stage = {}
orig = {k: getattr(tr, k) for k in ("tune_forward", "tune_targets", "tune_backward", "adam_step")}
for k, f in orig.items():
    def wrap(*a, _f=f, _k=k, **kw):
        t0 = time.perf_counter()
        r = _f(*a, **kw)
        stage[_k] = stage.get(_k, 0.0) + time.perf_counter() - t0
        return r
    setattr(tr, k, wrap)
N = 50
for i in range(N + 5):
    if i == 5:
        stage.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    TR.backprop(tr, st, wins, anom, cls)
torch.cuda.synchronize()
tot = (time.perf_counter() - t0) / N * 1e3
print(f"backprop {tot:.3f} ms/call (10 steps)")
for k, v in stage.items():
    print(f"  host time in {k:14s} {v / N * 1e3:.3f} ms/call")
