"""Golden fixtures for PreGAN's FPE path at 50 hosts (BASELINE config C4 "50
hosts"; build container only).

Run:  cd /tmp && python /root/repo/tests/golden/make_golden_fpe50.py

The reference's ``FPE_50`` (recovery/PreGANSrc/src/models.py:156-210) cannot
run: its encode feeds a 2-D tensor into ``GATHead`` (models.py:186-187), whose
forward unpacks four dimensions (dlutils.py:306).  Its ``FPE_16`` class,
however, is host-count generic: ``encode``/``forward`` (models.py:65-115) take
every shape from ``self.n_hosts`` / ``self.n_feats``.  So, exactly as
make_golden.py does for ``Transformer_16`` at H=50, the fixture model is an
instance of the reference ``FPE_16`` with only its ``__init__`` constants set
for 50 hosts (the same submodule classes and structure, models.py:11-63); its
``forward`` is the reference's own method.  This is an extrapolation of the
FPE_16 architecture to H=50, NOT the reference's FPE_50.
Gen_50 / Disc_50 (models.py:258-291) are the reference's own classes.

Weights: preganplus_amd.weights.synth_fpe_weights(50, seed=0) (fp32-
representable doubles), fp64, eval mode.  Each window runs under
torch.manual_seed(1000 + b); the GRU state draw of encode (models.py:70) is
recorded as the fixture's h0 so the kernels can take it as an input.

Windows: C2's distribution (make_golden.c2_windows) plus low-load and
high-load windows so the fixture holds windows with and without any flagged
host; one-hot and dense schedules (dense ones move the discriminator gate).
Margins of every decision are stored next to it.

Writes tests/golden/fpe_h50.npz.
"""
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import refshim  # noqa: E402
from preganplus_amd import weights as W  # noqa: E402
import make_golden as MG  # noqa: E402

models, utils, train = refshim.import_reference()

H = 50
SEED = 0


def build_fpe(n_hosts):
    """An n_hosts instance of the reference ``FPE_16`` (models.py:10-63):
    same submodules and structure, constants set for n_hosts."""
    m = models.FPE_16.__new__(models.FPE_16)
    nn.Module.__init__(m)
    m.name, m.lr = f"FPE_{n_hosts}", 0.0001
    m.n_hosts = n_hosts
    m.n_feats = 3 * n_hosts
    m.n_window = 3
    m.n_latent = 10
    m.n_hidden = 16
    m.gru = nn.GRU(input_size=m.n_feats, hidden_size=m.n_window, num_layers=1, batch_first=False)
    src = torch.tensor([i for i in range(n_hosts) for _ in range(n_hosts)])
    dst = torch.tensor([j for _ in range(n_hosts) for j in range(n_hosts)])
    m.gat_graph = models.dgl.graph((src, dst))
    m.gat_input_feats = 3
    m.gat_output_feats = n_hosts
    m.gat = models.GAT(m.gat_graph, m.gat_input_feats, m.gat_output_feats)
    m.mha = nn.MultiheadAttention(embed_dim=m.n_window + m.gat_output_feats, num_heads=1)
    m.encoder = nn.Sequential(
        nn.Linear(m.n_window * (m.n_window + m.gat_output_feats), m.n_hosts * m.n_latent),
        nn.LeakyReLU(True))
    m.anomaly_decoder = nn.Sequential(nn.Linear(m.n_latent, 2), nn.Softmax(dim=0))
    m.prototype_decoder = nn.Sequential(nn.Linear(m.n_latent, models.PROTO_DIM), nn.Sigmoid())
    m.prototype = [torch.rand(models.PROTO_DIM, dtype=torch.double) for _ in range(3)]
    return m


def to_sd(d):
    return {k: torch.tensor(np.asarray(v, dtype=np.float64)) for k, v in d.items()}


def second_gap(v, largest):
    """fp64 margin of a first-arg-extremum decision: |best - runner-up|."""
    s = np.sort(v, axis=-1)
    return (s[..., -1] - s[..., -2]) if largest else (s[..., 1] - s[..., 0])


def make_models(w):
    f = build_fpe(H).double()
    g, d = models.Gen_50().double(), models.Disc_50().double()
    f.load_state_dict(to_sd(w["fpe"]))
    g.load_state_dict(to_sd(w["gen"]))
    d.load_state_dict(to_sd(w["disc"]))
    f.prototype = [torch.tensor(p) for p in np.asarray(w["prototypes"])]
    for m in (f, g, d):
        m.eval()
    return f, g, d


def run_reference(w, windows, sched, seed0):
    f, g, d = make_models(w)
    out = {k: [] for k in ["h0", "probs", "protos", "emb", "cls", "any", "new_sched", "gprobs", "keep",
                           "final_target", "gen_target"]}
    with torch.no_grad():
        for b in range(windows.shape[0]):
            torch.manual_seed(seed0 + b)
            h0 = torch.randn(1, 1, 3, dtype=torch.double)
            torch.manual_seed(seed0 + b)
            win, s = torch.tensor(windows[b]), torch.tensor(sched[b])
            anomaly, prototype = f(win, s)                                   # models.py:111-115
            probs = torch.cat(anomaly, 0).numpy()
            emb = [torch.zeros_like(p) if torch.argmax(anomaly[i]).item() == 0 else p
                   for i, p in enumerate(prototype)]                           # PreGAN.py:119
            cls = utils.get_classes(emb, f)                                  # utils.py:102-109
            e = torch.stack(emb)
            ns = g(e, s)                                                     # models.py:271-273
            gp = d(s, ns)                                                    # models.py:289-291
            out["h0"].append(h0.numpy().reshape(3))
            out["probs"].append(probs)
            out["protos"].append(torch.stack(prototype).numpy())
            out["emb"].append(e.numpy())
            out["cls"].append(np.array(cls, np.int32))
            out["any"].append(any(torch.argmax(a).item() == 1 for a in anomaly))
            out["new_sched"].append(ns.numpy())
            out["gprobs"].append(gp.numpy())
            out["keep"].append(bool(gp[0] > gp[1]))
            out["final_target"].append(np.array([r.index(max(r)) for r in s.tolist()], np.int32))
            out["gen_target"].append(np.array([r.index(max(r)) for r in ns.tolist()], np.int32))
    res = {k: np.stack([np.asarray(v) for v in vals]) for k, vals in out.items()}
    P = np.asarray(w["prototypes"])
    dist = ((res["emb"][:, :, None, :] - P[None, None]) ** 2).mean(-1)
    res["margin_anomaly"] = np.abs(res["probs"][..., 1] - res["probs"][..., 0])
    res["margin_class"] = second_gap(dist, largest=False)
    res["margin_keep"] = np.abs(res["gprobs"][:, 0] - res["gprobs"][:, 1])
    res["margin_gen"] = second_gap(res["new_sched"], largest=True)
    flagged = (res["probs"][..., 1] > res["probs"][..., 0]).sum(1)
    print("fpe50: windows", windows.shape[0], "any", int(res["any"].sum()), "keep", int(res["keep"].sum()),
          "flagged hosts per window min/median/max", int(flagged.min()), int(np.median(flagged)),
          int(flagged.max()))
    print("  min margins: anomaly %.3g class %.3g keep %.3g gen %.3g" % (
        res["margin_anomaly"].min(), np.nanmin(res["margin_class"]), res["margin_keep"].min(),
        res["margin_gen"].min()))
    return res


def shifted(w, shift):
    """The same weights with the shared anomaly decoder's bias moved by
    (+shift, -shift): few hosts flagged, so windows without any flagged host
    (the early return, PreGAN.py:112-113) and the class -1 rows occur."""
    import copy
    w2 = copy.deepcopy(w)
    w2["fpe"]["anomaly_decoder.0.bias"] = w2["fpe"]["anomaly_decoder.0.bias"] + np.array([shift, -shift])
    return w2


BIAS_SHIFT = 0.046875


def main():
    w = W.synth_fpe_weights(H, seed=SEED)
    rng = np.random.Generator(np.random.PCG64(5050))
    syn = MG.c2_windows(rng, 48, H)
    low = rng.uniform(0, 0.05, size=(8, 3, 3 * H))           # idle fleet
    high = rng.uniform(0.8, 1.3, size=(8, 3, 3 * H))         # saturated fleet
    wide = rng.uniform(-1.0, 2.0, size=(8, 3, 3 * H))         # out-of-range loads
    windows = np.concatenate([syn, low, high, wide])
    n = windows.shape[0]
    sched = MG.onehot_sched(rng, n, H)
    dense = rng.permutation(n)[:12]
    sched[dense] = rng.uniform(0, 1, size=(12, H, H))
    res = run_reference(w, windows, sched, 1000)
    # set b: shifted anomaly bias, C2 windows
    wb = shifted(w, BIAS_SHIFT)
    win_b = MG.c2_windows(rng, 40, H)
    sched_b = MG.onehot_sched(rng, 40, H)
    sched_b[-8:] = rng.uniform(0, 1, size=(8, H, H))
    res_b = run_reference(wb, win_b, sched_b, 3000)
    assert 0 < res_b["any"].sum() < len(win_b)
    np.savez_compressed(os.path.join(HERE, "fpe_h50.npz"), windows=windows, sched=sched,
                        weights_seed=np.int32(SEED), n_hosts=np.int32(H),
                        model_note=np.array("reference FPE_16 class instantiated at n_hosts=50 "
                                            "(extrapolation; the reference FPE_50 raises at dlutils.py:306)"),
                        **res, **{"b/windows": win_b, "b/sched": sched_b, "b/bias_shift": np.float64(BIAS_SHIFT)},
                        **{f"b/{k}": v for k, v in res_b.items()})


if __name__ == "__main__":
    main()
