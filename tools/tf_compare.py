"""A/B of the tuning step's forward + backward between two builds of the
library (PGP_LIB), on the same seeded inputs: `dump OUT H B` writes logits,
protos, latent and the transformer gradient; `compare A B` prints the largest
relative difference per parameter tensor.  A debugging aid for kernel
rewrites (the parity tests proper compare against the reference fixtures)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(out, H, B):
    import torch
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    w = W.synth_weights(H, seed=0)
    tr = TR.Trainer(H, w, max_batch=B)
    rng = np.random.Generator(np.random.PCG64(7))
    x = rng.uniform(0, 0.6, size=(B, 3, 3 * H)).astype(np.float32)
    y = (rng.uniform(size=(B, H)) < 0.2).astype(np.int32)
    mult = rng.uniform(0.5, 2.0, size=(B, H)).astype(np.float32)
    tgt = rng.uniform(size=(B, H, 2)).astype(np.float32)
    lat = torch.zeros((B, 3 * H * H), device=tr.device)
    logits, protos = tr.tune_forward(torch.tensor(x, device=tr.device), lat)
    tr.tune_backward(B, y, mult, tgt)
    torch.cuda.synchronize()
    g = tr.G.cpu().numpy()
    res = {"logits": logits.cpu().numpy(), "protos": protos.cpu().numpy(), "latent": lat.cpu().numpy()}
    for t in tr.tensors:
        if t["section"] == "transformer":
            res["G/" + t["name"]] = g[t["offset"]:t["offset"] + t["n"]]
    np.savez(out, **res)


def compare(a, b):
    za, zb = np.load(a), np.load(b)
    worst = 0.0
    for k in za.files:
        x, y = za[k].astype(np.float64), zb[k].astype(np.float64)
        scale = max(np.abs(y).max(), 1e-30)
        d = np.abs(x - y).max() / scale
        worst = max(worst, d) if not k.endswith("pe") else worst
        print(f"{k:45s} max|a-b|/max|b| = {d:.3e}   max|b| = {scale:.3e}")
    print("worst", worst)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    else:
        compare(sys.argv[2], sys.argv[3])
