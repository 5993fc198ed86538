"""Golden fixtures for the online steps of PreGANPlusRecovery (build container only).

Run:  cd /tmp && python /root/repo/tests/golden/make_golden_train.py

Captured from the reference's own code (dropout p set to 0 so the reference is
deterministic — it never calls eval()):

  tests/golden/tune_h16.npz    train.backprop (train.py:42-57) on the 10-window
                               on-the-fly dataset (utils.py:40-47) of a fake
                               stats object: per-step losses, the parameter
                               gradients of step 0, parameters after step 0 and
                               after all 10 steps, prototypes, PROTO_UPDATE_FACTOR
  tests/golden/gan_h16.npz     PreGANPlusRecovery.train_gan (PreGANPlus.py:60-81)
                               for both label outcomes, weights after each
  tests/golden/plugin_h16.npz  PreGANPlusRecovery.run_model (PreGANPlus.py:115-136)
                               over 4 consecutive intervals of a fake environment
                               (GAN step, tuning, decision assembly)

The shipped checkpoints' optimizer states (AdamW exp_avg / exp_avg_sq / step)
are added to preganplus_amd/data/simulator_16.npz so the build can continue
training exactly where the checkpoint left off (utils.py:73).
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

import refshim  # noqa: E402
from preganplus_amd import weights as W  # noqa: E402

models, utils, train = refshim.import_reference()
import recovery.PreGANPlus as plugin_mod  # noqa: E402

H = 16
DATA = refshim.ckpt_path("data")


def no_dropout(m):
    for mod in m.modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
        if isinstance(mod, nn.MultiheadAttention):
            mod.dropout = 0.0


def load_all():
    """Models + optimizers exactly as load_model does (utils.py:60-79), but with
    the safe loader."""
    out = {}
    for name, cls in (("Transformer", models.Transformer_16), ("Gen", models.Gen_16),
                      ("Disc", models.Disc_16)):
        ck = refshim.safe_load_ckpt(refshim.ckpt_path(f"checkpointsplus/simulator_{name}_16.ckpt"))
        m = cls().double()
        opt = torch.optim.AdamW(m.parameters(), lr=m.lr, weight_decay=1e-5)
        m.load_state_dict(ck["model_state_dict"])
        if name == "Transformer":
            m.prototype = [p.detach().clone() for p in ck["model_prototypes"]]
        opt.load_state_dict(ck["optimizer_state_dict"])
        no_dropout(m)
        out[name] = (m, opt, ck)
    return out


def opt_state_arrays(m, opt, prefix):
    """AdamW state per named parameter (state keyed by param order)."""
    arrs = {}
    for i, (n, p) in enumerate(m.named_parameters()):
        st = opt.state[p]
        arrs[f"opt/{prefix}/{n}/exp_avg"] = st["exp_avg"].detach().numpy().astype(np.float64)
        arrs[f"opt/{prefix}/{n}/exp_avg_sq"] = st["exp_avg_sq"].detach().numpy().astype(np.float64)
        arrs[f"opt/{prefix}/{n}/step"] = np.float64(float(st["step"]))
    return arrs


def params(m):
    return {n: p.detach().numpy().copy() for n, p in m.named_parameters()}


class FakeStats:
    def __init__(self, ts, ss, scores):
        self.time_series = ts
        self.schedule_series = ss
        self._scores = list(scores)
        self.calls = []

    def runSimulation(self, schedule):
        s = np.asarray(schedule.detach().numpy() if torch.is_tensor(schedule) else schedule)
        self.calls.append(s.copy())
        return self._scores.pop(0)


class FakeContainer:
    def __init__(self, cid, hid):
        self.id, self._h = cid, hid

    def getHostID(self):
        return self._h


class Obj:
    pass


def make_tune_golden(ms, train_time):
    t, topt, _ = ms["Transformer"]
    rng = np.random.Generator(np.random.PCG64(7))
    ts = train_time[60:75].copy()
    ss = np.load(os.path.join(DATA, "simulator/schedule_series.npy"))[60:75]
    stats = FakeStats(ts, ss, [])
    folder = os.path.join(DATA, "simulator")
    wins, sched, anom, cls = utils.load_on_the_fly_dataset(t, folder, stats)   # utils.py:40-47
    train.PROTO_UPDATE_FACTOR = 0.2
    factor0 = train.PROTO_UPDATE_FACTOR
    protos0 = np.stack([p.detach().numpy() for p in t.prototype])
    p0 = params(t)
    # step 0 by hand (same calls as backprop's loop body) to capture gradients
    train.num_zero, train.num_ones = 1, 1
    grads0, losses, protos_steps, params1 = None, [], [], None
    for i in range(wins.shape[0]):
        out = t(wins[i], sched[i])
        aloss, tloss = train.custom_loss(t, out, anom[i], cls[i])
        loss = aloss + tloss
        topt.zero_grad()
        loss.backward()
        if i == 0:
            grads0 = {n: (q.grad.detach().numpy().copy() if q.grad is not None else np.zeros_like(q.detach().numpy()))
                      for n, q in t.named_parameters()}
        topt.step()
        if i == 0:
            params1 = params(t)
        losses.append((float(aloss), float(tloss)))
        protos_steps.append(np.stack([p.detach().numpy() for p in t.prototype]))
    res = {f"p0/{k}": v for k, v in p0.items()}
    res.update({f"g0/{k}": v for k, v in grads0.items()})
    res.update({f"p1/{k}": v for k, v in params1.items()})
    res.update({f"p10/{k}": v for k, v in params(t).items()})
    res.update(windows=wins.numpy(), sched=np.asarray(sched, np.float64), anom=anom, cls=cls,
               time_series=ts, losses=np.array(losses), protos0=protos0,
               protos_steps=np.stack(protos_steps), factor0=np.float64(factor0),
               factor_end=np.float64(train.PROTO_UPDATE_FACTOR),
               num_zero=np.float64(train.num_zero), num_ones=np.float64(train.num_ones))
    np.savez_compressed(os.path.join(HERE, "tune_h16.npz"), **res)
    print("tune: losses", np.array(losses)[:3], "factor", train.PROTO_UPDATE_FACTOR)


def make_gan_golden(ms, emb, sched):
    out = {}
    for tag, scores in (("better", [(1.0, 1.0), (2.0, 2.0)]), ("worse", [(3.0, 3.0), (1.0, 1.0)])):
        g, gopt, _ = ms["Gen"]
        d, dopt, _ = ms["Disc"]
        g0, d0 = params(g), params(d)
        obj = Obj()
        obj.gen, obj.disc, obj.gopt, obj.dopt = g, d, gopt, dopt
        obj.ganloss = nn.BCELoss()
        obj.save_gan = False
        obj.env = Obj()
        obj.env.stats = FakeStats(None, None, scores)
        plugin_mod.PreGANPlusRecovery.train_gan(obj, torch.tensor(emb), torch.tensor(sched))
        out.update({f"{tag}/gen/{k}": v for k, v in params(g).items()})
        out.update({f"{tag}/disc/{k}": v for k, v in params(d).items()})
        out[f"{tag}/sim_new"] = obj.env.stats.calls[0]
        # restore for the next outcome
        for m, p in ((g, g0), (d, d0)):
            with torch.no_grad():
                for n, q in m.named_parameters():
                    q.copy_(torch.tensor(p[n]))
        ms2 = load_all()
        ms["Gen"], ms["Disc"] = ms2["Gen"], ms2["Disc"]
    out["emb"], out["sched"] = emb, sched
    np.savez_compressed(os.path.join(HERE, "gan_h16.npz"), **out)
    print("gan: fixtures written")


def make_plugin_golden(train_time):
    """run_model over 4 consecutive intervals on a fake env."""
    ms = load_all()
    t, topt, tck = ms["Transformer"]
    g, gopt, gck = ms["Gen"]
    d, dopt, _ = ms["Disc"]
    ss_all = np.load(os.path.join(DATA, "simulator/schedule_series.npy"))
    rng = np.random.Generator(np.random.PCG64(11))
    obj = plugin_mod.PreGANPlusRecovery.__new__(plugin_mod.PreGANPlusRecovery)
    obj.model, obj.optimizer, obj.epoch, obj.accuracy_list = t, topt, tck["epoch"], []
    obj.gen, obj.disc, obj.gopt, obj.dopt = g, d, gopt, dopt
    obj.gan_plotter = sys.modules["recovery.PreGANSrc.src.plotter"].GAN_Plotter()
    obj.ganloss = nn.BCELoss()
    obj.train_time_data = train_time
    # save_gan is always True in the reference (PreGANPlus.py:20): train_gan
    # appends (gen_loss, disc_loss) and counts the epoch; the checkpoint write
    # itself is replaced by a no-op so nothing is written
    obj.hosts, obj.env_name, obj.training, obj.save_gan = H, "simulator", True, True
    plugin_mod.save_gan = lambda *a, **k: None
    obj.model_name, obj.gen_name, obj.disc_name = "Transformer_16", "Gen_16", "Disc_16"
    env = Obj()
    env.hostlist = list(range(H))
    obj.env = env
    train.PROTO_UPDATE_FACTOR = 0.2
    rec = {}
    T0 = 100
    for step in range(4):
        tt = T0 + step
        sched = ss_all[tt].astype(np.float32)
        placement = rng.integers(0, H, size=H)
        placement[rng.integers(0, H)] = -1          # one unplaced container
        containers = [FakeContainer(c, int(placement[c])) for c in range(H)]
        containers[3] = None                        # a None slot, as containerlist allows
        env.containerlist = containers
        env.scheduler = Obj()
        env.scheduler.result_cache = sched
        scores = [(float(rng.uniform(0, 2)), float(rng.uniform(0, 2))) for _ in range(2)]
        env.stats = FakeStats(train_time[:tt + 1], ss_all[:tt + 1], scores)
        decision = [(c, int(placement[c])) for c in range(H) if placement[c] >= 0 and c != 3][:10]
        res = obj.run_model(None, decision)
        rec[f"s{step}/sched"] = sched
        rec[f"s{step}/placement"] = placement
        rec[f"s{step}/scores"] = np.array(scores)
        rec[f"s{step}/decision_in"] = np.array(decision, dtype=np.int64).reshape(-1, 2)
        rec[f"s{step}/decision_out"] = np.array(res, dtype=np.int64).reshape(-1, 2)
        rec[f"s{step}/n_sim_calls"] = np.int64(len(env.stats.calls))
        print(f"plugin step {step}: {len(res)} decisions, sim calls {len(env.stats.calls)}")
    rec.update({f"end/t/{k}": v for k, v in params(t).items()})
    rec.update({f"end/g/{k}": v for k, v in params(g).items()})
    rec.update({f"end/d/{k}": v for k, v in params(d).items()})
    rec["end/protos"] = np.stack([p.detach().numpy() for p in t.prototype])
    # per interval: (gen_loss, disc_loss) from train_gan, then (loss, factor,
    # AScore, CScore) from tune_model's accuracy() (PreGANPlus.py:56-58, 77)
    rec["end/accuracy_list"] = np.concatenate([np.asarray(x, dtype=np.float64) for x in obj.accuracy_list])
    rec["end/accuracy_list_lens"] = np.array([len(x) for x in obj.accuracy_list], dtype=np.int64)
    rec["end/epoch"] = np.int64(obj.epoch)
    rec["start/epoch"] = np.int64(gck["epoch"])
    rec["end/factor"] = np.float64(train.PROTO_UPDATE_FACTOR)
    rec["T0"] = np.int64(T0)
    rec["schedule_series"] = ss_all[:T0 + 4]
    np.savez_compressed(os.path.join(HERE, "plugin_h16.npz"), **rec)


def main():
    train_time = np.load(os.path.join(DATA, "simulator/time_series.npy"))
    ms = load_all()
    # optimizer states into the packaged weights
    wpath = os.path.join(REPO, "preganplus_amd", "data", "simulator_16.npz")
    w, extra = W.load_npz(wpath)
    for name, pre in (("Transformer", "transformer"), ("Gen", "gen"), ("Disc", "disc")):
        m, opt, ck = ms[name]
        extra.update(opt_state_arrays(m, opt, pre))
        extra[f"meta/{pre}/epoch"] = np.int64(ck["epoch"])
        if name == "Gen":   # load_gan's accuracy_list, kept by the plugin (PreGANPlus.py:32-34)
            extra.update(W.accuracy_list_to_arrays(ck["accuracy_list"], "meta/gen/accuracy_list"))
    W.save_npz(wpath, w, extra=extra)
    make_tune_golden(ms, train_time)
    z = np.load(os.path.join(HERE, "fwd_h16.npz"))
    make_gan_golden(load_all(), z["emb"][5], z["sched"][5])
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "recovery/PreGANSrc"))
        os.symlink(DATA, os.path.join(td, "recovery/PreGANSrc/data"))
        os.chdir(td)
        try:
            make_plugin_golden(train_time)
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()
