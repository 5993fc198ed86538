"""Golden fixture for PreGAN's offline FPE_16 training (build container only).

Run:  cd /tmp && python /root/repo/tests/golden/make_golden_fpetrain.py

With no FPE checkpoint, PreGANRecovery.load_models creates a new FPE_16
(utils.py:60-79: epoch -1) and trains it (PreGAN.py:26-27, 39-49): epochs of
train.backprop (train.py:42-57, sequential batch-1 steps, AdamW lr 1e-4 wd
1e-5) + train.accuracy over utils.load_dataset's whole series (utils.py:36-42).
The reference's framework environment ships no FPE checkpoint
(recovery/PreGANSrc/checkpoints/), so this is the path it takes there.

Recorded here with the reference's own modules (via refshim): a seeded new
FPE_16 (its torch initialisation and prototypes), two epochs over the first
N_WIN windows of data/framework/time_series.npy, every GRU state the forwards
draw (torch.randn inside encode, models.py:70: recorded by wrapping torch.randn,
so the kernels can take them as inputs), the losses, factor, counters,
parameters and AdamW moments after each epoch, and accuracy()'s scores.
Writes tests/golden/fpe_train_h16.npz (numeric arrays only).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import refshim  # noqa: E402

models, utils, train = refshim.import_reference()
N_WIN = 24
EPOCHS = 2


def main():
    torch.manual_seed(7)
    f = models.FPE_16().double()
    opt = torch.optim.AdamW(f.parameters(), lr=f.lr, weight_decay=1e-5)      # utils.py:65
    rec = {f"init/{k}": v.detach().numpy().copy() for k, v in f.state_dict().items()}
    rec["init/prototypes"] = np.stack([p.numpy() for p in f.prototype])
    folder = refshim.ckpt_path("data/framework")
    wins, sched, anom, cls = utils.load_dataset(folder, f)                     # utils.py:36-42
    wins, sched, anom, cls = wins[:N_WIN], sched[:N_WIN], anom[:N_WIN], cls[:N_WIN]
    rec["wins"] = wins.numpy()
    rec["anom"] = np.asarray(anom, dtype=np.int64)
    rec["cls"] = np.asarray(cls, dtype=np.int64)
    draws = []
    randn = torch.randn

    def recording_randn(*a, **k):
        t = randn(*a, **k)
        draws.append(t.detach().numpy().reshape(-1).copy())
        return t

    torch.randn = recording_randn
    torch.manual_seed(11)
    train.PROTO_UPDATE_FACTOR = 0.2   # the module global starts at PROTO_UPDATE_FACTOR (train.py:1)
    try:
        for ep in range(EPOCHS):
            n0 = len(draws)
            loss, factor = train.backprop(ep, f, wins, sched, anom, cls, opt)
            n1 = len(draws)
            asc, csc = train.accuracy(f, wins, sched, anom, cls, None)
            n2 = len(draws)
            assert n1 - n0 == N_WIN and n2 - n1 == N_WIN, (n0, n1, n2)
            rec[f"ep{ep}/h0_backprop"] = np.stack(draws[n0:n1])
            rec[f"ep{ep}/h0_accuracy"] = np.stack(draws[n1:n2])
            rec[f"ep{ep}/loss"] = np.float64(loss)
            rec[f"ep{ep}/factor"] = np.float64(factor)
            rec[f"ep{ep}/ascore"] = np.float64(asc)
            rec[f"ep{ep}/cscore"] = np.float64(csc)
            rec[f"ep{ep}/num_zero"] = np.float64(train.num_zero)
            rec[f"ep{ep}/num_ones"] = np.float64(train.num_ones)
            rec[f"ep{ep}/proto_factor"] = np.float64(train.PROTO_UPDATE_FACTOR)
            rec[f"ep{ep}/prototypes"] = np.stack([p.detach().numpy() for p in f.prototype])
            for k, v in f.state_dict().items():
                rec[f"ep{ep}/p/{k}"] = v.detach().numpy().copy()
            names = [k for k, _ in f.named_parameters()]
            for i, (k, q) in enumerate(f.named_parameters()):
                st = opt.state[q]
                rec[f"ep{ep}/m/{k}"] = st["exp_avg"].numpy().copy()
                rec[f"ep{ep}/v/{k}"] = st["exp_avg_sq"].numpy().copy()
                rec[f"ep{ep}/step/{k}"] = np.float64(float(st["step"]))
            print(f"epoch {ep}: loss {loss:.6f} factor {factor:.6f} AScore {asc:.4f} CScore {csc:.4f}", names[:2])
    finally:
        torch.randn = randn
    np.savez_compressed(os.path.join(HERE, "fpe_train_h16.npz"), **rec)


if __name__ == "__main__":
    main()
