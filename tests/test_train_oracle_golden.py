"""Pin the training oracle (torch-autograd restatement) against fixtures
produced by the reference's own training code (tests/golden/make_golden_train.py)."""
import numpy as np
import pytest
import torch

from oracle import pregan_oracle as O
from oracle import pregan_train_oracle as TO
from preganplus_amd import weights as W

GOLD = "tests/golden"


def load16():
    return W.load_npz("preganplus_amd/data/simulator_16.npz")


def test_tuning_step_matches_reference():
    w, extra = load16()
    z = np.load(f"{GOLD}/tune_h16.npz")
    wins, sched, anom, cls = TO.on_the_fly_dataset(z["time_series"], z["sched"], extra["train_time_data"])
    np.testing.assert_allclose(wins, z["windows"], rtol=0, atol=1e-15)
    assert np.array_equal(anom, z["anom"]) and np.array_equal(cls, z["cls"])
    tw = TO.leaf_params(w["transformer"])
    opt = TO.AdamW({k: v for k, v in tw.items() if v.requires_grad}, 1e-4,
                   TO.opt_state_from_npz(extra, "transformer"))
    st = TO.TuneState(z["protos0"], float(z["factor0"]))
    rec = {}
    losses = TO.backprop(tw, opt, st, wins, sched, anom, cls, record=rec)
    np.testing.assert_allclose(np.array(losses), z["losses"], rtol=1e-10, atol=1e-12)
    for k in w["transformer"]:
        if k == "pos_encoder.pe":
            continue
        np.testing.assert_allclose(rec["g0"][k], z[f"g0/{k}"], rtol=1e-8, atol=1e-12, err_msg=k)
        np.testing.assert_allclose(rec["p1"][k], z[f"p1/{k}"], rtol=1e-10, atol=1e-13, err_msg=k)
        np.testing.assert_allclose(tw[k].detach().numpy(), z[f"p10/{k}"], rtol=1e-8, atol=1e-11, err_msg=k)
    np.testing.assert_allclose(np.stack([p.numpy() for p in st.protos]), z["protos_steps"][-1], atol=1e-12)
    assert abs(st.factor - float(z["factor_end"])) < 1e-15
    assert st.num_zero == z["num_zero"] and st.num_ones == z["num_ones"]


@pytest.mark.parametrize("tag,scores", [("better", [1.0, 2.0]), ("worse", [3.0, 1.0])])
def test_gan_step_matches_reference(tag, scores):
    w, extra = load16()
    z = np.load(f"{GOLD}/gan_h16.npz")
    gw, dw = TO.leaf_params(w["gen"], skip=()), TO.leaf_params(w["disc"], skip=())
    gopt = TO.AdamW(gw, 5e-5, TO.opt_state_from_npz(extra, "gen"))
    dopt = TO.AdamW(dw, 5e-5, TO.opt_state_from_npz(extra, "disc"))
    it = iter(scores)
    _, _, ns = TO.train_gan(gw, dw, gopt, dopt, z["emb"], z["sched"], lambda s: next(it))
    np.testing.assert_allclose(ns, z[f"{tag}/sim_new"], atol=1e-12)
    for k in w["gen"]:
        np.testing.assert_allclose(gw[k].detach().numpy(), z[f"{tag}/gen/{k}"], rtol=1e-10, atol=1e-13)
    for k in w["disc"]:
        np.testing.assert_allclose(dw[k].detach().numpy(), z[f"{tag}/disc/{k}"], rtol=1e-10, atol=1e-13)


class _Obj:
    pass


class FakeContainer:
    def __init__(self, cid, hid):
        self.id, self._h = cid, hid

    def getHostID(self):
        return self._h


def fake_env(z, step, train_time, ss_all_rows):
    T0 = int(z["T0"])
    tt = T0 + step
    env = _Obj()
    env.hostlist = list(range(16))
    placement = z[f"s{step}/placement"]
    cl = [FakeContainer(c, int(placement[c])) for c in range(16)]
    cl[int(z["container_none"]) if "container_none" in z.files else 3] = None
    env.containerlist = cl
    env.scheduler = _Obj()
    env.scheduler.result_cache = z[f"s{step}/sched"]
    env.stats = _Obj()
    env.stats.time_series = train_time[:tt + 1]
    env.stats.schedule_series = ss_all_rows[:tt + 1]
    sc = [tuple(x) for x in z[f"s{step}/scores"]]
    env.stats.runSimulation = lambda sched: sc.pop(0)
    return env


def test_plugin_run_model_matches_reference():
    w, extra = load16()
    z = np.load(f"{GOLD}/plugin_h16.npz")
    tr = extra["train_time_data"]
    ss = z["schedule_series"]
    po = TO.PluginOracle(w, extra, tr)
    for step in range(4):
        env = fake_env(z, step, tr, ss)
        dec = po.run_model(env, [tuple(x) for x in z[f"s{step}/decision_in"]])
        assert [tuple(map(int, d)) for d in dec] == [tuple(x) for x in z[f"s{step}/decision_out"].tolist()]
    for k in w["transformer"]:
        if k != "pos_encoder.pe":
            np.testing.assert_allclose(po.tw[k].detach().numpy(), z[f"end/t/{k}"], rtol=1e-7, atol=1e-10, err_msg=k)
    for k in w["gen"]:
        np.testing.assert_allclose(po.gw[k].detach().numpy(), z[f"end/g/{k}"], rtol=1e-7, atol=1e-10)
    np.testing.assert_allclose(np.stack([p.numpy() for p in po.st.protos]), z["end/protos"], atol=1e-10)
