"""Golden fixtures for PreGAN's FPE_16 path (BASELINE config 4; build container only).

Run:  cd /tmp && python /root/repo/tests/golden/make_golden_fpe.py

Reference modules: FPE_16 (models.py:10-115) with the shipped
checkpoints/simulator_FPE_16.ckpt, Gen_16/Disc_16 from checkpoints/ (PreGAN's
own GAN, PreGAN.py:23-37), eval mode.  FPE's encode draws the GRU state with
torch.randn (models.py:70); each window is run under torch.manual_seed(1000+b)
and the same draw is recorded as the fixture's h0, so the kernels can take it as
an input.  Writes preganplus_amd/data/pregan_simulator_16.npz (converted
weights + Gen/Disc AdamW state), tests/golden/fpe_h16.npz (per-window forward)
and tests/golden/pregan_plugin_h16.npz (PreGANRecovery.run_model over 4
intervals on a fake env, training on; torch.manual_seed(2000+step) before each
call pins the GRU h0 draw; checkpoints written by save_gan go to a temp dir).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import tempfile  # noqa: E402

import torch.nn as nn  # noqa: E402

import refshim  # noqa: E402
from preganplus_amd import weights as W  # noqa: E402
import make_golden as MG  # noqa: E402

models, utils, train = refshim.import_reference()
import recovery.PreGAN as plugin_mod  # noqa: E402
from make_golden_train import FakeContainer, FakeStats, Obj, opt_state_arrays, params  # noqa: E402

H = 16
DATA = refshim.ckpt_path("data")


def load_pregan():
    """FPE_16 + Gen_16/Disc_16 from checkpoints/ with AdamW as load_model/load_gan
    build them (utils.py:60-79), via the safe loader."""
    out = {}
    for name, cls in (("FPE", models.FPE_16), ("Gen", models.Gen_16), ("Disc", models.Disc_16)):
        ck = refshim.safe_load_ckpt(refshim.ckpt_path(f"checkpoints/simulator_{name}_16.ckpt"))
        m = cls().double()
        opt = torch.optim.AdamW(m.parameters(), lr=m.lr, weight_decay=1e-5)
        m.load_state_dict(ck["model_state_dict"])
        if name == "FPE":
            m.prototype = [p.detach().clone() for p in ck["model_prototypes"]]
        opt.load_state_dict(ck["optimizer_state_dict"])
        out[name] = (m, opt, ck)
    return out


def make_plugin_golden(train_time):
    ms = load_pregan()
    f, fopt, fck = ms["FPE"]
    g, gopt, gck = ms["Gen"]
    d, dopt, _ = ms["Disc"]
    utils.freeze(f)                                                          # PreGAN.py:29
    ss_all = np.load(os.path.join(DATA, "simulator/schedule_series.npy"))
    rng = np.random.Generator(np.random.PCG64(12))
    obj = plugin_mod.PreGANRecovery.__new__(plugin_mod.PreGANRecovery)
    obj.model, obj.optimizer, obj.epoch, obj.accuracy_list = f, fopt, gck["epoch"], []
    obj.gen, obj.disc, obj.gopt, obj.dopt = g, d, gopt, dopt
    obj.gan_plotter = sys.modules["recovery.PreGANSrc.src.plotter"].GAN_Plotter()
    obj.ganloss = nn.BCELoss()
    obj.train_time_data = train_time
    obj.hosts, obj.env_name, obj.training = H, "simulator", True
    obj.model_name, obj.gen_name, obj.disc_name = "FPE_16", "Gen_16", "Disc_16"
    env = Obj()
    env.hostlist = list(range(H))
    obj.env = env
    rec = {}
    T0 = 120
    for step in range(4):
        tt = T0 + step
        sched = ss_all[tt].astype(np.float32)
        placement = rng.integers(0, H, size=H)
        placement[rng.integers(0, H)] = -1
        containers = [FakeContainer(c, int(placement[c])) for c in range(H)]
        containers[5] = None
        env.containerlist = containers
        env.scheduler = Obj()
        env.scheduler.result_cache = sched
        scores = [(float(rng.uniform(0, 2)), float(rng.uniform(0, 2))) for _ in range(2)]
        env.stats = FakeStats(train_time[:tt + 1], ss_all[:tt + 1], scores)
        decision = [(c, int(placement[c])) for c in range(H) if placement[c] >= 0 and c != 5][:10]
        torch.manual_seed(2000 + step)
        res = obj.run_model(None, decision)
        rec[f"s{step}/sched"] = sched
        rec[f"s{step}/placement"] = placement
        rec[f"s{step}/scores"] = np.array(scores)
        rec[f"s{step}/decision_in"] = np.array(decision, dtype=np.int64).reshape(-1, 2)
        rec[f"s{step}/decision_out"] = np.array(res, dtype=np.int64).reshape(-1, 2)
        rec[f"s{step}/n_sim_calls"] = np.int64(len(env.stats.calls))
        print(f"pregan plugin step {step}: {len(res)} decisions, sim calls {len(env.stats.calls)}")
    rec.update({f"end/g/{k}": v for k, v in params(g).items()})
    rec.update({f"end/d/{k}": v for k, v in params(d).items()})
    rec["T0"] = np.int64(T0)
    rec["container_none"] = np.int64(5)
    rec["end/epoch"] = np.int64(obj.epoch)
    rec["end/accuracy_list"] = np.array(obj.accuracy_list, dtype=np.float64)   # 4 x (gen_loss, disc_loss)
    rec["schedule_series"] = ss_all[:T0 + 4]
    np.savez_compressed(os.path.join(HERE, "pregan_plugin_h16.npz"), **rec)


def main():
    ck = {n: refshim.safe_load_ckpt(refshim.ckpt_path(f"checkpoints/simulator_{n}_16.ckpt"))
          for n in ("FPE", "Gen", "Disc")}
    f, g, d = models.FPE_16().double(), models.Gen_16().double(), models.Disc_16().double()
    f.load_state_dict(ck["FPE"]["model_state_dict"])
    g.load_state_dict(ck["Gen"]["model_state_dict"])
    d.load_state_dict(ck["Disc"]["model_state_dict"])
    f.prototype = [p.detach().clone() for p in ck["FPE"]["model_prototypes"]]
    for m in (f, g, d):
        m.eval()
    conv = lambda sd: {k: v.detach().numpy().astype(np.float64) for k, v in sd.items()}
    wts = {"fpe": conv(f.state_dict()), "gen": conv(g.state_dict()), "disc": conv(d.state_dict()),
           "prototypes": np.stack([p.numpy() for p in f.prototype])}
    flat = {f"fpe/{k}": v for k, v in wts["fpe"].items()}
    flat.update({f"gen/{k}": v for k, v in wts["gen"].items()})
    flat.update({f"disc/{k}": v for k, v in wts["disc"].items()})
    flat["prototypes"] = wts["prototypes"]
    flat["train_time_data"] = np.load(refshim.ckpt_path("data/simulator/time_series.npy"))
    # the FPE_16 training curve (AScore per epoch): the only reference-held
    # evidence on DGL's softmax_edges semantics (tests/test_gat_semantics.py)
    flat.update(W.accuracy_list_to_arrays(ck["FPE"]["accuracy_list"], "meta/fpe/accuracy_list"))
    ms = load_pregan()
    for name, pre in (("Gen", "gen"), ("Disc", "disc")):
        m, opt, ckk = ms[name]
        flat.update(opt_state_arrays(m, opt, pre))
        flat[f"meta/{pre}/epoch"] = np.int64(ckk["epoch"])
        if name == "Gen":   # load_gan's accuracy_list, kept by the plugin (PreGAN.py:31-32)
            flat.update(W.accuracy_list_to_arrays(ckk["accuracy_list"], "meta/gen/accuracy_list"))
    np.savez_compressed(os.path.join(REPO, "preganplus_amd", "data", "pregan_simulator_16.npz"), **flat)

    train_time = np.load(refshim.ckpt_path("data/simulator/time_series.npy"))
    real = MG.real_windows_h16(train_time)[:120]
    rng = np.random.Generator(np.random.PCG64(4321))
    syn = MG.c2_windows(rng, 40, 16)
    windows = np.concatenate([real, syn])
    sched = MG.onehot_sched(rng, windows.shape[0], 16)
    sched[-6:] = rng.uniform(0, 1, size=(6, 16, 16))
    out = {k: [] for k in ["h0", "probs", "protos", "emb", "cls", "any", "new_sched", "gprobs", "keep",
                           "final_target", "gen_target"]}
    with torch.no_grad():
        for b in range(windows.shape[0]):
            torch.manual_seed(1000 + b)
            h0 = torch.randn(1, 1, 3, dtype=torch.double)
            torch.manual_seed(1000 + b)
            win, s = torch.tensor(windows[b]), torch.tensor(sched[b])
            anomaly, prototype = f(win, s)                                   # models.py:111-115
            probs = torch.cat(anomaly, 0).numpy()
            anoms = [torch.argmax(a).item() for a in anomaly]                # PreGAN.py:110-111
            emb = [torch.zeros_like(p) if torch.argmax(anomaly[i]).item() == 0 else p
                   for i, p in enumerate(prototype)]                           # PreGAN.py:119
            cls = utils.get_classes(emb, f)
            e = torch.stack(emb)
            ns = g(e, s)
            gp = d(s, ns)
            out["h0"].append(h0.numpy().reshape(3))
            out["probs"].append(probs)
            out["protos"].append(torch.stack(prototype).numpy())
            out["emb"].append(e.numpy())
            out["cls"].append(np.array(cls, np.int32))
            out["any"].append(any(a == 1 for a in anoms))
            out["new_sched"].append(ns.numpy())
            out["gprobs"].append(gp.numpy())
            out["keep"].append(bool(gp[0] > gp[1]))
            out["final_target"].append(np.array([r.index(max(r)) for r in s.tolist()], np.int32))
            out["gen_target"].append(np.array([r.index(max(r)) for r in ns.tolist()], np.int32))
    res = {k: np.stack([np.asarray(v) for v in vals]) for k, vals in out.items()}
    np.savez_compressed(os.path.join(HERE, "fpe_h16.npz"), windows=windows, sched=sched, **res)
    print("fpe: any", int(res["any"].sum()), "/", len(windows), "keep", int(res["keep"].sum()))
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "recovery/PreGANSrc/checkpoints"))   # save_gan target (temp only)
        os.symlink(DATA, os.path.join(td, "recovery/PreGANSrc/data"))
        os.chdir(td)
        try:
            make_plugin_golden(train_time)
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()
