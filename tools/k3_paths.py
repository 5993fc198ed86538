"""K3 (stage 3) time with one-hot schedules (gather path) vs soft schedules
(dense MFMA path), H = 16 and 50, 65,536 windows."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from preganplus_amd import weights as W  # noqa: E402
from preganplus_amd.model import DecisionModel  # noqa: E402

for H in (16, 50):
    B = 65536
    w = W.synth_weights(H, seed=1)
    m = DecisionModel(H, w)
    m.reserve(B)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.rand((B, 3, 3 * H), generator=g, device="cuda") * 0.6).contiguous()
    idx = torch.randint(0, H, (B, H), generator=g, device="cuda")
    s1 = torch.zeros((B, H, H), device="cuda").scatter_(2, idx.unsqueeze(-1), 1.0).contiguous()
    s2 = s1.clone()
    s2[:, 0, 0] += 0.5  # one soft value per window: every workgroup takes the dense path
    out = m.alloc_outputs(B)
    for name, s in (("one-hot", s1), ("dense", s2)):
        for st in (0, 1, 2, 3):
            m.forward(x, s, out=out, stage=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            m.forward(x, s, out=out, stage=3)
        e1.record()
        torch.cuda.synchronize()
        print(f"H={H} {name}: K3 {e0.elapsed_time(e1) / 10:.3f} ms", flush=True)
