"""Phase timing of the fused batch-1 tuning kernel (pgp_tune1.hip).

Run on the GPU box with the timing variant:
  make variant NAME=t1prof VFLAGS=-DPGP_T1_PROF     (here, before the call)
  PGP_LIB=preganplus_amd/_lib/var/libpreganplus_t1prof.so python tools/t1_phases.py
Prints, per barrier-delimited phase, the median wall-clock time (100 MHz
counter) over repeated steps, and the kernel total.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from preganplus_amd import _native  # noqa: E402
from preganplus_amd import train as TR  # noqa: E402
from preganplus_amd import weights as W  # noqa: E402


def main():
    H = int(os.environ.get("T1_HOSTS", "16"))
    w, extra = W.load_npz("preganplus_amd/data/simulator_16.npz") if H == 16 else (W.synth_weights(H, 1), None)
    tr = TR.Trainer(H, w, extra, max_batch=1)
    L = _native.lib()
    L.pgp_tune1_prof_read.argtypes = [ctypes.c_void_p]
    dev = tr.device
    rng = np.random.default_rng(0)
    st = TR.TuneState(rng.uniform(0.1, 0.9, (H, 2)))
    state = st.to_device(dev)
    loss = torch.zeros(2, dtype=torch.float64, device=dev)
    buf = (ctypes.c_ulonglong * 128)()
    rows = []
    for it in range(60):
        win = torch.tensor(rng.uniform(0, 1, (3, 3 * H)), dtype=torch.float32, device=dev)
        y = torch.tensor((rng.random(H) < 0.4).astype(np.int32), device=dev)
        c = torch.tensor(rng.integers(0, 3, H).astype(np.int32), device=dev)
        tr.tune_step1(win, y, c, state, loss)
        torch.cuda.synchronize()
        assert L.pgp_tune1_prof_read(ctypes.addressof(buf)) == 0
        t = np.array(buf[:], dtype=np.int64)
        n = int(np.argmax(t == 0)) if (t == 0).any() else 128
        if it >= 10:
            rows.append(np.diff(t[:n]) * 0.01)  # 100 MHz ticks -> us
    d = np.median(np.stack(rows), axis=0)
    for i, v in enumerate(d):
        print(f"phase {i:2d}: {v:7.2f} us")
    print(f"total   : {d.sum():7.2f} us")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/t1_phases_h{H}.json", "w") as f:
        json.dump({"H": H, "phase_us": d.tolist(), "total_us": float(d.sum())}, f)


if __name__ == "__main__":
    main()
