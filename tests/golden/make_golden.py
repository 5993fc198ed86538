"""Generate the golden fixtures from the reference itself (build container only).

Run:  cd /tmp && python /root/repo/tests/golden/make_golden.py
(cwd outside /root/reference so nothing is written there; bytecode writing off.)

Every output below is computed by the REFERENCE's own modules
(``recovery/PreGANSrc/src/models.py`` Transformer_16 / Gen_* / Disc_*, and
``utils.get_classes``), in ``eval()`` mode, fp64, through ``refshim`` (DGL
stand-in, safe checkpoint loading).  The fixtures are data: inputs + expected
outputs.  They are committed; the reference never travels to the GPU box.

Fixtures:
  preganplus_amd/data/simulator_16.npz  shipped H=16 checkpoints, converted
                                        (+ data/simulator/time_series.npy for
                                        normalisation)
  tests/golden/fwd_h16.npz   256 windows: 199 real run_encoder windows from the
                             shipped simulator series + 57 synthetic; real +
                             synthetic schedules (one-hot and dense)
  tests/golden/fwd_h50.npz   64 synthetic windows at H=50, weights =
                             preganplus_amd.weights.synth_weights(50, seed=0)
                             loaded into an H=50 instance of the reference
                             Transformer_16 code (constants overridden) and the
                             reference Gen_50/Disc_50
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

models, utils, train = refshim.import_reference()


def build_transformer(H):
    """An H-host instance of the reference ``Transformer_16`` (models.py:314-416):
    same submodule classes and structure, constants set for H hosts.
    forward/encode are the reference's own methods."""
    m = models.Transformer_16.__new__(models.Transformer_16)
    nn.Module.__init__(m)
    m.name, m.lr = f"Transformer_{H}", 0.0001
    m.n_hosts, m.n_window, m.gat_input_feats = H, 3, 3
    m.gat_output_feats = m.d_model = H
    m.nhead, m.dim_feedforward, m.num_layers = 2, 64, 2
    m.latent_dim = H * H * 3
    src = torch.tensor([i for i in range(H) for _ in range(H)])
    dst = torch.tensor([j for _ in range(H) for j in range(H)])
    m.gat_graph = models.dgl.graph((src, dst))
    m.gat = models.GAT(m.gat_graph, 3, H)
    m.time_encoder = nn.Linear(H, H)
    m.pos_encoder = models.PositionalEncoding(H, 0.1, 3)
    layer = nn.TransformerEncoderLayer(d_model=H, nhead=2, dim_feedforward=64, dropout=0.1)
    m.transformer_encoder = nn.TransformerEncoder(layer, num_layers=2)
    m.anomaly_decoder = nn.Sequential(nn.Linear(m.latent_dim, 2 * H), nn.LeakyReLU(True),
                                      nn.Unflatten(1, (H, 2)))
    m.prototype_decoder = nn.Sequential(nn.Linear(m.latent_dim, 2 * H), nn.Sigmoid(),
                                        nn.Unflatten(1, (H, 2)))
    m.prototype = [torch.rand(2, dtype=torch.double) for _ in range(H)]
    return m


def to_sd(d):
    return {k: torch.tensor(np.asarray(v, dtype=np.float64)) for k, v in d.items()}


def make_models(weights, H):
    if H == 16:
        t = models.Transformer_16()
        g, d = models.Gen_16(), models.Disc_16()
    else:
        t = build_transformer(H)
        g, d = getattr(models, f"Gen_{H}")(), getattr(models, f"Disc_{H}")()
    t, g, d = t.double(), g.double(), d.double()
    t.load_state_dict(to_sd(weights["transformer"]))
    g.load_state_dict(to_sd(weights["gen"]))
    d.load_state_dict(to_sd(weights["disc"]))
    t.prototype = [torch.tensor(p) for p in np.asarray(weights["prototypes"])]
    for m in (t, g, d):
        m.eval()
    return t, g, d


def c2_windows(rng, n, H):
    """SURVEY §8(d) C2 distribution: U(0,0.6) load, 2% spikes U(0.9,1.3)."""
    x = rng.uniform(0, 0.6, size=(n, 3, 3 * H))
    spike = rng.uniform(0, 1, size=x.shape) < 0.02
    x[spike] = rng.uniform(0.9, 1.3, size=int(spike.sum()))
    return x


def onehot_sched(rng, n, H):
    s = np.zeros((n, H, H))
    idx = rng.integers(0, H, size=(n, H))
    for b in range(n):
        s[b, np.arange(H), idx[b]] = 1.0
    return s


@torch.no_grad()
def run_reference(t, g, d, windows, sched):
    out = {k: [] for k in ["latent", "logits", "protos", "emb", "cls", "any",
                           "new_sched", "probs", "keep", "final_target", "gen_target"]}
    for b in range(windows.shape[0]):
        win = torch.tensor(windows[b])
        s = torch.tensor(sched[b])
        out["latent"].append(t.encode(win, s).numpy()[0])
        anomaly, prototype = t(win, s)                    # models.py:402-416
        logits = torch.cat(anomaly, 0).numpy()
        protos = torch.stack(prototype).numpy()
        anoms = [torch.argmax(a).item() for a in anomaly]          # PreGANPlus.py:120-121
        emb = [torch.zeros_like(p) if torch.argmax(anomaly[i]).item() == 0 else p
               for i, p in enumerate(prototype)]                    # PreGANPlus.py:129
        cls = utils.get_classes(emb, t)                             # utils.py:102-109
        emb_t = torch.stack(emb)
        ns = g(emb_t, s)                                            # models.py:131-133
        probs = d(s, ns)                                            # models.py:149-151
        out["logits"].append(logits)
        out["protos"].append(protos)
        out["emb"].append(emb_t.numpy())
        out["cls"].append(np.array(cls, dtype=np.int32))
        out["any"].append(any(a == 1 for a in anoms))
        out["new_sched"].append(ns.numpy())
        out["probs"].append(probs.numpy())
        out["keep"].append(bool(probs[0] > probs[1]))               # PreGANPlus.py:87
        out["final_target"].append(np.array([r.index(max(r)) for r in s.tolist()], np.int32))
        out["gen_target"].append(np.array([r.index(max(r)) for r in ns.tolist()], np.int32))
    return {k: np.stack([np.asarray(v) for v in vals]) for k, vals in out.items()}


def real_windows_h16(train_time):
    """Windows exactly as run_encoder builds them (PreGANPlus.py:107-112) for
    env.stats.time_series = series[:t+1], t = 2..201."""
    series = train_time
    wins = []
    for tt in range(3, series.shape[0]):
        td = utils.normalize_test_time_data(series[:tt], train_time)
        if td.shape[0] >= 3:
            td = td[-3:]
        wins.append(utils.convert_to_windows(td, models.Transformer_16())[-1].numpy())
    return np.stack(wins)


def main():
    rng = np.random.Generator(np.random.PCG64(1234))
    # ---------------- H = 16, shipped checkpoints ----------------
    wt = W.load_reference_checkpoints(refshim.ckpt_path("checkpointsplus"), "simulator", 16)
    train_time = np.load(refshim.ckpt_path("data/simulator/time_series.npy"))
    sched_series = np.load(refshim.ckpt_path("data/simulator/schedule_series.npy"))
    os.makedirs(os.path.join(REPO, "preganplus_amd", "data"), exist_ok=True)
    W.save_npz(os.path.join(REPO, "preganplus_amd", "data", "simulator_16.npz"), wt,
               extra={"train_time_data": train_time})
    t, g, d = make_models(wt, 16)
    real = real_windows_h16(train_time)                               # [199,3,48]
    real_s = sched_series[3:3 + real.shape[0]]
    syn = c2_windows(rng, 57, 16)
    syn_s = onehot_sched(rng, 57, 16)
    syn_s[-8:] = rng.uniform(0, 1, size=(8, 16, 16))                  # dense schedules
    windows = np.concatenate([real, syn])
    sched = np.concatenate([real_s, syn_s])
    ref = run_reference(t, g, d, windows, sched)
    np.savez_compressed(os.path.join(HERE, "fwd_h16.npz"), windows=windows, sched=sched,
                        n_real=np.int32(real.shape[0]), **ref)
    print("H16: any-anomaly windows", int(ref["any"].sum()), "/", len(windows),
          " keep", int(ref["keep"].sum()))
    # ---------------- H = 50, seeded weights ----------------
    w50 = W.synth_weights(50, seed=0)
    t, g, d = make_models(w50, 50)
    windows = c2_windows(rng, 64, 50)
    sched = onehot_sched(rng, 64, 50)
    sched[-4:] = rng.uniform(0, 1, size=(4, 50, 50))
    ref = run_reference(t, g, d, windows, sched)
    ref["latent"] = ref["latent"][:8]
    np.savez_compressed(os.path.join(HERE, "fwd_h50.npz"), windows=windows, sched=sched,
                        weights_seed=np.int32(0),
                        weights_checksum=np.float64(W.weights_checksum(w50)), **ref)
    print("H50: any-anomaly windows", int(ref["any"].sum()), "/", len(windows),
          " keep", int(ref["keep"].sum()))


if __name__ == "__main__":
    main()
