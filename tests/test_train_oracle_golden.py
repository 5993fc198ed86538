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


# ---------------------------------------------------------------------------
# H = 50 (tests/golden/make_golden_train50.py: the reference's modules on the
# H=50 instance, seeded weights, fresh AdamW)
# ---------------------------------------------------------------------------
def _close(rtol, atol):
    def f(got, want, what):
        np.testing.assert_allclose(got, want, rtol=rtol, atol=atol, err_msg=what)
    return f


def test_tuning_step_matches_reference_h50():
    from tests.golden import digest as D
    w = W.synth_weights(50, 0)
    z = np.load(f"{GOLD}/tune_h50.npz")
    assert abs(W.weights_checksum(w) - float(z["weights_checksum"])) == 0
    wins, sched, anom, cls = TO.on_the_fly_dataset(z["time_series"], z["sched"], z["train_time"])
    np.testing.assert_allclose(wins, z["windows"], rtol=0, atol=1e-15)
    assert np.array_equal(anom, z["anom"]) and np.array_equal(cls, z["cls"])
    tw = TO.leaf_params(w["transformer"])
    opt = TO.AdamW({k: v for k, v in tw.items() if v.requires_grad}, 1e-4)
    st = TO.TuneState(w["prototypes"], float(z["factor0"]))
    rec = {}
    losses = TO.backprop(tw, opt, st, wins, sched, anom, cls, record=rec)
    np.testing.assert_allclose(np.array(losses), z["losses"], rtol=1e-10, atol=1e-12)
    for k in w["transformer"]:
        if k == "pos_encoder.pe":
            continue
        g = rec["g0"][k] if rec["g0"][k] is not None else np.zeros_like(w["transformer"][k])
        D.check(z, f"g0/{k}", g, _close(1e-8, 1e-12), sum_rel=1e-9, key=k)
        # an entry whose gradient is rounding noise (|g| ~ 1e-15) still takes an
        # AdamW step of up to lr: those differ by more than the parameters' ulps
        D.check(z, f"p1/{k}", rec["p1"][k], _close(1e-10, 1e-11), sum_rel=1e-9, key=k)
        D.check(z, f"p10/{k}", tw[k].detach().numpy(), _close(1e-8, 1e-10), sum_rel=1e-8, key=k)
    np.testing.assert_allclose(np.stack([p.numpy() for p in st.protos[:3]]), z["protos_steps"][-1], atol=1e-12)
    assert abs(st.factor - float(z["factor_end"])) < 1e-15
    assert st.num_zero == z["num_zero"] and st.num_ones == z["num_ones"]


@pytest.mark.parametrize("tag,scores", [("better", [1.0, 2.0]), ("worse", [3.0, 1.0])])
def test_gan_step_matches_reference_h50(tag, scores):
    from tests.golden import digest as D
    w = W.synth_weights(50, 0)
    z = np.load(f"{GOLD}/gan_h50.npz")
    gw, dw = TO.leaf_params(w["gen"], skip=()), TO.leaf_params(w["disc"], skip=())
    gopt, dopt = TO.AdamW(gw, 3e-5), TO.AdamW(dw, 3e-5)
    it = iter(scores)
    _, _, ns = TO.train_gan(gw, dw, gopt, dopt, z["emb"], z["sched"], lambda s: next(it))
    np.testing.assert_allclose(ns, z[f"{tag}/sim_new"], atol=1e-12)
    for k in w["gen"]:
        D.check(z, f"{tag}/gen/{k}", gw[k].detach().numpy(), _close(1e-10, 1e-13), sum_rel=1e-10, key=k)
    for k in w["disc"]:
        D.check(z, f"{tag}/disc/{k}", dw[k].detach().numpy(), _close(1e-10, 1e-13), sum_rel=1e-10, key=k)


def dp_inputs(z, H=50):
    """The 1,024 C2 windows of dp_h50_b1024.npz (make_golden.c2_windows, seeded)."""
    rng = np.random.Generator(np.random.PCG64(int(z["windows_seed"])))
    B = z["y"].shape[0]
    x = rng.uniform(0, 0.6, size=(B, 3, 3 * H))
    spike = rng.uniform(0, 1, size=x.shape) < 0.02
    x[spike] = rng.uniform(0.9, 1.3, size=int(spike.sum()))
    return x


def test_dp_batch_h50_matches_reference():
    """C3's local batch (1,024 windows, H=50) under the data-parallel loss:
    the training oracle's batched autograd reproduces the reference modules'
    gradients, and the product's host restatement of the step's bookkeeping
    (train.loss_targets_dp) reproduces the reference-computed CE weights,
    losses and prototype-EMA increments."""
    from preganplus_amd import train as TR
    from tests.golden import digest as D
    w = W.synth_weights(50, 0)
    z = np.load(f"{GOLD}/dp_h50_b1024.npz")
    x, y, c = dp_inputs(z), z["y"], z["c"]
    B, H = y.shape
    tw = TO.leaf_params(w["transformer"])
    logits, protos = TO.decode_t(tw, TO.encode_t(tw, torch.tensor(x)))
    D.check(z, "logits", logits.detach().numpy(), _close(1e-10, 1e-12), sum_rel=1e-10)
    D.check(z, "protos", protos.detach().numpy(), _close(1e-10, 1e-12), sum_rel=1e-10)
    st = TR.TuneState(w["prototypes"], float(z["factor"]))
    st.num_zero, st.num_ones = float(z["num_zero"]), float(z["num_ones"])
    mult, tgt, aloss, tloss, inc = TR.loss_targets_dp(logits.detach().numpy(), protos.detach().numpy(), y, c, st)
    np.testing.assert_allclose(np.stack([aloss, tloss], 1), z["losses"], rtol=1e-10, atol=1e-9)
    np.testing.assert_allclose(inc.delta[:3], z["delta"], rtol=1e-10, atol=1e-12)
    np.testing.assert_array_equal(inc.count[:3], z["count"])
    assert inc.count[3:].sum() == 0 and inc.num_zero == B * H and inc.num_ones == y.sum()
    ce = torch.nn.functional.cross_entropy(logits.reshape(-1, 2), torch.tensor(y.reshape(-1)), reduction="none")
    loss = (ce.reshape(B, H) * torch.tensor(mult)).sum()
    loss = loss + (((protos - torch.tensor(tgt)) ** 2).mean(-1) * torch.tensor(y > 0)).sum()
    loss.backward()
    for k in w["transformer"]:
        if k != "pos_encoder.pe":
            D.check(z, f"grad/{k}", tw[k].grad.numpy(), _close(1e-8, 1e-9), sum_rel=1e-8, key=k)


def fpe_train_fixture():
    z = np.load("tests/golden/fpe_train_h16.npz")
    init = {k[len("init/"):]: z[k] for k in z.files if k.startswith("init/") and k != "init/prototypes"}
    return z, init


def test_fpe_offline_training_matches_reference():
    """The torch restatement of PreGAN's offline FPE training (fpe_backprop,
    PreGAN.py:39-49 / train.py:42-57 on FPE_16) against the reference's own
    modules (tests/golden/make_golden_fpetrain.py): two epochs over 24 windows
    of the framework series with the recorded GRU states; parameters, AdamW
    moments, prototypes, factor, counters after each epoch, and accuracy()'s
    scores (train.py:94-109) from the same forwards."""
    from preganplus_amd import train as TR
    z, init = fpe_train_fixture()
    fw = TO.leaf_params(init, skip=())
    opt = TO.AdamW(fw, 1e-4)
    st = TO.TuneState(z["init/prototypes"], 0.2)
    wins, anom, cls = z["wins"], z["anom"], z["cls"]
    for ep in range(2):
        losses = TO.fpe_backprop(fw, opt, st, wins, z[f"ep{ep}/h0_backprop"], anom, cls)
        loss = np.mean([a for a, _ in losses]) + np.mean([t for _, t in losses])
        assert loss == pytest.approx(float(z[f"ep{ep}/loss"]), rel=1e-12)
        assert st.factor + O.PROTO_UPDATE_MIN == pytest.approx(float(z[f"ep{ep}/factor"]), rel=1e-14)
        assert (st.num_zero, st.num_ones) == (z[f"ep{ep}/num_zero"], z[f"ep{ep}/num_ones"])
        for k, q in fw.items():
            np.testing.assert_allclose(q.detach().numpy(), z[f"ep{ep}/p/{k}"], rtol=1e-10, atol=1e-13, err_msg=k)
            np.testing.assert_allclose(opt.m[k].numpy(), z[f"ep{ep}/m/{k}"], rtol=1e-9, atol=1e-14, err_msg=k)
            assert opt.step[k] == float(z[f"ep{ep}/step/{k}"])
        np.testing.assert_allclose(np.stack([p.numpy() for p in st.protos]), z[f"ep{ep}/prototypes"], rtol=1e-12)
        with torch.no_grad():
            probs, protos = TO.fpe_t(fw, torch.tensor(wins), torch.tensor(z[f"ep{ep}/h0_accuracy"]))
        asc, csc = TR.accuracy_scores(probs.numpy(), protos.numpy(), anom, cls,
                                      np.stack([p.numpy() for p in st.protos]))
        assert asc == pytest.approx(float(z[f"ep{ep}/ascore"]), rel=1e-12)
        assert csc == pytest.approx(float(z[f"ep{ep}/cscore"]), rel=1e-12)
