"""H=50 golden fixtures for the online training steps (build container only).

Run:  cd /tmp && python /root/repo/tests/golden/make_golden_train50.py

Every number is computed by the REFERENCE's own modules: the H=50 instance of
``Transformer_16`` (``make_golden.build_transformer``), the
reference ``Gen_50`` / ``Disc_50`` (``models.py:258-291``), ``train.custom_loss``
/ ``train.anomaly_loss`` / ``train.mse_loss`` (``train.py:7-40``), the reference
on-the-fly dataset functions (``utils.py:7-24, 94-95``) and
``PreGANPlusRecovery.train_gan`` (``PreGANPlus.py:60-81``), with dropout p = 0
(the reference never calls eval()) and fresh AdamW optimisers as
``load_model`` builds them (``utils.py:65``: lr = model.lr, weight decay 1e-5).
Weights: ``preganplus_amd.weights.synth_weights(50, seed=0)``.  Large tensors are
stored as digests (tests/golden/digest.py).

  tests/golden/tune_h50.npz   backprop (train.py:42-57) over the 10-window
                              on-the-fly dataset of a synthetic 50-host series:
                              losses, gradients of step 0, parameters after
                              step 0 and step 9, prototypes, factor, counters
  tests/golden/gan_h50.npz    train_gan for both label outcomes: Gen/Disc
                              parameters after the step
  tests/golden/dp_h50_b1024.npz  C3's local batch: 1,024 windows through the
                              reference modules with the data-parallel loss
                              (every window scored against the
                              step-start state, loss summed over the batch):
                              per-window losses, transformer gradients, the
                              prototype-EMA increments; and the batched GAN
                              step's Disc / Gen gradients (sums of the
                              per-window BCE losses, PreGANPlus.py:60-74)
"""
import os
import sys
import tempfile

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import make_golden as MG  # noqa: E402  (imports the reference through refshim)
from digest import digest  # noqa: E402
from preganplus_amd import weights as W  # noqa: E402

models, utils, train = MG.models, MG.utils, MG.train
import recovery.PreGANPlus as plugin_mod  # noqa: E402

H = 50
torch.set_default_dtype(torch.float64)


def no_dropout(m):
    for mod in m.modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
        if isinstance(mod, nn.MultiheadAttention):
            mod.dropout = 0.0


def transformer(w):
    t = MG.build_transformer(H).double()
    t.load_state_dict(MG.to_sd(w["transformer"]))
    t.prototype = [torch.tensor(p) for p in np.asarray(w["prototypes"])]
    no_dropout(t)
    return t, torch.optim.AdamW(t.parameters(), lr=t.lr, weight_decay=1e-5)


def gan(w):
    g, d = models.Gen_50().double(), models.Disc_50().double()
    g.load_state_dict(MG.to_sd(w["gen"]))
    d.load_state_dict(MG.to_sd(w["disc"]))
    return (g, torch.optim.AdamW(g.parameters(), lr=g.lr, weight_decay=1e-5),
            d, torch.optim.AdamW(d.parameters(), lr=d.lr, weight_decay=1e-5))


def params(m):
    return {n: p.detach().numpy().copy() for n, p in m.named_parameters()}


def digests(prefix, d):
    """Digest per tensor; the sample indices are keyed by the parameter name, so
    a parameter's gradient and values share them."""
    out = {}
    for k, v in d.items():
        out.update(digest(f"{prefix}/{k}", v, key=k))
    return out


def synth_series(rng, T):
    """A 50-host [cpu, ram, disk] series with per-column scales and sparse
    contention spikes (the raw stats.time_series shape, Stats.py:46-48)."""
    scale = rng.uniform(20, 100, size=3 * H)
    x = rng.uniform(0.05, 0.6, size=(T, 3 * H)) * scale
    spike = rng.uniform(size=x.shape) < 0.03
    return np.where(spike, rng.uniform(0.8, 1.0, size=x.shape) * scale, x)


def make_tune(w):
    t, opt = transformer(w)
    rng = np.random.Generator(np.random.PCG64(50))
    train_time = synth_series(rng, 60)
    ts = train_time[40:55].copy()
    # utils.load_on_the_fly_dataset (utils.py:40-47) without its npy read: the
    # training series is passed in directly
    time_data = utils.normalize_test_time_data(ts[-10:], train_time)
    wins = utils.convert_to_windows(time_data, t)
    anom, cls = utils.form_test_dataset(time_data)
    sched = np.zeros((10, H, H))
    sched[np.arange(10)[:, None], np.arange(H)[None, :], rng.integers(0, H, (10, H))] = 1.0
    train.PROTO_UPDATE_FACTOR = 0.2
    train.num_zero, train.num_ones = 1, 1
    res = {}
    losses, protos_steps = [], []
    for i in range(wins.shape[0]):
        out = t(wins[i], torch.tensor(sched[i]))
        aloss, tloss = train.custom_loss(t, out, anom[i], cls[i])
        opt.zero_grad()
        (aloss + tloss).backward()
        if i == 0:
            res.update(digests("g0", {n: (q.grad.numpy() if q.grad is not None else np.zeros(q.shape))
                                      for n, q in t.named_parameters()}))
        opt.step()
        if i == 0:
            res.update(digests("p1", params(t)))
        losses.append((float(aloss), float(tloss)))
        protos_steps.append(np.stack([p.detach().numpy() for p in t.prototype[:3]]))
    res.update(digests("p10", params(t)))
    res.update(train_time=train_time, time_series=ts, windows=wins.numpy(), sched=sched, anom=anom, cls=cls,
               losses=np.array(losses), protos_steps=np.stack(protos_steps), factor0=np.float64(0.2),
               factor_end=np.float64(train.PROTO_UPDATE_FACTOR), num_zero=np.float64(train.num_zero),
               num_ones=np.float64(train.num_ones), weights_seed=np.int32(0),
               weights_checksum=np.float64(W.weights_checksum(w)))
    np.savez_compressed(os.path.join(HERE, "tune_h50.npz"), **res)
    print("tune_h50: losses", np.array(losses)[:2], "anomalous hosts", int(anom.sum()))


class _Obj:
    pass


class _Stats:
    def __init__(self, scores):
        self.scores = list(scores)
        self.calls = []

    def runSimulation(self, s):
        self.calls.append(np.asarray(s.detach().numpy() if torch.is_tensor(s) else s).copy())
        return self.scores.pop(0)


def make_gan(w):
    z = np.load(os.path.join(HERE, "fwd_h50.npz"))
    i = int(np.argmax(np.abs(z["emb"]).sum(axis=(1, 2))))     # the window with the most anomalous hosts
    emb, sched = z["emb"][i], z["sched"][i]
    out = {"emb": emb, "sched": sched}
    for tag, scores in (("better", [(1.0, 1.0), (2.0, 2.0)]), ("worse", [(3.0, 3.0), (1.0, 1.0)])):
        g, gopt, d, dopt = gan(w)
        obj = _Obj()
        obj.gen, obj.disc, obj.gopt, obj.dopt = g, d, gopt, dopt
        obj.ganloss = nn.BCELoss()
        obj.save_gan = False
        obj.env = _Obj()
        obj.env.stats = _Stats(scores)
        plugin_mod.PreGANPlusRecovery.train_gan(obj, torch.tensor(emb), torch.tensor(sched))
        out.update(digests(f"{tag}/gen", params(g)))
        out.update(digests(f"{tag}/disc", params(d)))
        out[f"{tag}/sim_new"] = obj.env.stats.calls[0]
    np.savez_compressed(os.path.join(HERE, "gan_h50.npz"), **out)
    print("gan_h50: window", i, "anomalous hosts", int((np.abs(emb).sum(-1) > 0).sum()))


def make_dp(w, B=1024):
    t, _ = transformer(w)
    rng = np.random.Generator(np.random.PCG64(1024))
    x = MG.c2_windows(rng, B, H)
    y = (rng.uniform(size=(B, H)) < 0.3).astype(np.int64)
    c = rng.integers(0, 3, size=(B, H))
    P = np.asarray(w["prototypes"], dtype=np.float64)
    num_zero, num_ones, factor = 500.0, 37.0, 0.2
    f = factor + 0.02                                           # PROTO_UPDATE_FACTOR + PROTO_UPDATE_MIN
    total = 0
    losses = np.zeros((B, 2))
    logits = np.zeros((B, H, 2))
    protos = np.zeros((B, H, 2))
    delta, count = np.zeros((3, 2)), np.zeros(3)
    Pt = [torch.tensor(p) for p in P]
    for b in range(B):
        sa_list, sp_list = t(torch.tensor(x[b]), None)
        aloss = 0
        tloss = torch.tensor(0.0)
        for h in range(H):                                      # train.py:31-35, start-of-step counters
            mult = 1 if y[b, h] == 0 else num_zero / num_ones
            aloss = aloss + train.anomaly_loss(sa_list[h], torch.tensor([int(y[b, h])])) * mult
        for h in range(H):                                      # train.py:36-38 / triplet_loss :13-25
            if y[b, h] > 0:
                cc = int(c[b, h])
                pos = train.mse_loss(sp_list[h], Pt[cc].detach().clone())
                negs = [train.mse_loss(sp_list[h], Pt[nc]) for nc in (0, 1, 2) if nc != cc]
                tloss = tloss + pos - torch.sum(torch.tensor([float(v) for v in negs]))
                if pos <= negs[0] and pos <= negs[1]:           # the EMA as an increment
                    delta[cc] += f * (sp_list[h].detach().numpy() - P[cc])
                    count[cc] += 1
        total = total + aloss + tloss
        losses[b] = (float(aloss), float(tloss))
        logits[b] = torch.cat(sa_list, 0).detach().numpy()
        protos[b] = torch.stack(sp_list).detach().numpy()
    t.zero_grad()
    total.backward()
    res = digests("grad", {n: (q.grad.numpy() if q.grad is not None else np.zeros(q.shape))
                           for n, q in t.named_parameters()})
    res.update(digest("logits", logits))
    res.update(digest("protos", protos))
    res.update(windows_seed=np.int64(1024), y=y, c=c, losses=losses, num_zero=np.float64(num_zero),
               num_ones=np.float64(num_ones), factor=np.float64(factor), delta=delta, count=count)
    # batched GAN step (PreGANPlus.py:60-74 summed over windows): Disc BCE toward
    # per-window targets on detached schedules, then Gen BCE toward [0, 1]
    g, _, d, _ = gan(w)
    emb = np.where(rng.uniform(size=(B, H, 1)) < 0.3, rng.uniform(size=(B, H, 2)), 0.0)
    s = np.zeros((B, H, H))
    s[np.arange(B)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(B, H))] = 1.0
    lab = rng.uniform(size=B) < 0.5
    target = np.stack([1.0 - lab, lab], axis=1)
    bce = nn.BCELoss()
    ns = [g(torch.tensor(emb[b]), torch.tensor(s[b])) for b in range(B)]
    dl = sum(bce(d(torch.tensor(s[b]), ns[b].detach()), torch.tensor(target[b])) for b in range(B))
    d.zero_grad()
    dl.backward()
    res.update(digests("gan/dgrad", {n: q.grad.numpy() for n, q in d.named_parameters()}))
    d.zero_grad()
    gl = sum(bce(d(torch.tensor(s[b]), ns[b]), torch.tensor([0.0, 1.0])) for b in range(B))
    g.zero_grad()
    gl.backward()
    res.update(digests("gan/ggrad", {n: q.grad.numpy() for n, q in g.named_parameters()}))
    res.update(digest("gan/ns", np.stack([v.detach().numpy() for v in ns])))
    res.update({"gan/emb": emb, "gan/sidx": s.argmax(-1), "gan/target": target})
    np.savez_compressed(os.path.join(HERE, "dp_h50_b1024.npz"), **res)
    print("dp_h50_b1024: loss", float(total), "EMA counts", count)


def main():
    w = W.synth_weights(H, seed=0)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            make_tune(w)
            make_gan(w)
            make_dp(w)
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()
