"""PreGAN's offline FPE_16 training on the device (PreGAN.py:26-27, 39-49;
preganplus_amd/fpetrain.py, csrc/pgp_fpetrain.hip) against the reference's own
modules: tests/golden/fpe_train_h16.npz (make_golden_fpetrain.py) holds a new
FPE_16, two epochs of train.backprop + accuracy over 24 windows of the
framework series, and every GRU state the forwards drew.  fp32 device training
vs the fp64 reference: parameters after each epoch within fp32 tolerance (the
AdamW rule of the tuning tests: entries whose gradient is rounding noise take
an lr-sized step of either sign), prototypes / factor / counters / scores from
the same bookkeeping."""
import numpy as np
import pytest
import torch

from oracle import pregan_oracle as O
from oracle import pregan_train_oracle as TO

pytestmark = pytest.mark.gpu


def _fixture():
    z = np.load("tests/golden/fpe_train_h16.npz")
    init = {k[len("init/"):]: z[k] for k in z.files if k.startswith("init/") and k != "init/prototypes"}
    return z, init


def test_fpe_step_gradient_matches_autograd():
    """One device step (forward, bookkeeping, backward) == torch autograd of
    the FPE restatement (pinned to the reference), from the same weights, h0
    and state: losses, the gradient of every parameter, the updated state."""
    from preganplus_amd import fpetrain as FT
    from preganplus_amd import train as TR
    z, init = _fixture()
    ft = FT.FPETrainer(init)
    wins, anom, cls = z["wins"], z["anom"], z["cls"]
    i = int(np.argmax(anom.sum(1) > 0))            # a window with a positive label
    h0 = z["ep0/h0_backprop"][i:i + 1]
    st = TR.TuneState(z["init/prototypes"], 0.2)
    st.num_zero, st.num_ones = 7, 3
    state = torch.tensor(st.vector(), dtype=torch.float64, device="cuda")
    dev = lambda a, dt: torch.as_tensor(np.asarray(a), dtype=dt).cuda().contiguous()
    w, h = dev(wins[i], torch.float32), dev(h0, torch.float32)
    y, c = dev(anom[i], torch.int32), dev(np.clip(cls[i], 0, 2), torch.int32)
    loss = torch.zeros(2, dtype=torch.float64, device="cuda")
    ft._L.pgp_fpe_train_step(16, 3, w.data_ptr(), h.data_ptr(), y.data_ptr(), c.data_ptr(), ft.P.data_ptr(),
                             ft.G.data_ptr(), state.data_ptr(), TR.PROTO_UPDATE_MIN, TR.PROTO_FACTOR_DECAY,
                             loss.data_ptr(), ft._stream())
    torch.cuda.synchronize()
    fw = TO.leaf_params(init, skip=())
    sto = TO.TuneState(z["init/prototypes"], 0.2)
    sto.num_zero, sto.num_ones = 7, 3
    probs, protos = TO.fpe_t(fw, torch.tensor(wins[i:i + 1]), torch.tensor(h0))
    aloss, tloss = TO.custom_loss(probs[0], protos[0], anom[i], cls[i], sto)
    (aloss + tloss).backward()
    lo = loss.cpu().numpy()
    assert lo[0] == pytest.approx(float(aloss), rel=1e-4) and lo[1] == pytest.approx(float(tloss), rel=1e-3, abs=1e-6)
    g = ft.G.cpu().numpy()
    for t in ft.tensors:
        want = fw[t["name"]].grad
        want = np.zeros(t["n"]) if want is None else want.numpy().reshape(-1)
        got = g[t["offset"]:t["offset"] + t["n"]]
        tol = 1e-3 * np.abs(want) + 1e-4 * (np.abs(want).max() + 1e-30)
        assert np.all(np.abs(got - want) <= tol), (t["name"], np.abs(got - want).max(), np.abs(want).max())
    sv = state.cpu().numpy()
    np.testing.assert_allclose(sv[:6].reshape(3, 2), np.stack([p.numpy() for p in sto.protos]), rtol=1e-6)
    assert sv[6] == pytest.approx(sto.factor, rel=1e-15) and (sv[7], sv[8]) == (sto.num_zero, sto.num_ones)


def test_fpe_offline_training_epochs_match_reference():
    from preganplus_amd import fpetrain as FT
    from preganplus_amd import train as TR
    z, init = _fixture()
    ft = FT.FPETrainer(init)
    st = TR.TuneState(z["init/prototypes"], 0.2)
    wins, anom, cls = z["wins"], z["anom"], z["cls"]
    for ep in range(2):
        losses = ft.backprop(st, wins, z[f"ep{ep}/h0_backprop"], anom, cls)
        loss = np.mean([a for a, _ in losses]) + np.mean([t for _, t in losses])
        assert loss == pytest.approx(float(z[f"ep{ep}/loss"]), rel=1e-4)
        assert st.factor + O.PROTO_UPDATE_MIN == pytest.approx(float(z[f"ep{ep}/factor"]), rel=1e-14)
        assert (st.num_zero, st.num_ones) == (z[f"ep{ep}/num_zero"], z[f"ep{ep}/num_ones"])
        np.testing.assert_allclose(st.protos, z[f"ep{ep}/prototypes"], rtol=1e-4, atol=1e-6)
        pw = ft.weights_numpy()
        lr = FT.FPE_LR
        fails = []
        for t in ft.tensors:
            want = z[f"ep{ep}/p/{t['name']}"].reshape(-1)
            got = pw[t["name"]].reshape(-1)
            # fp32 tolerance for all but entries whose gradient is rounding noise: those take
            # AdamW steps of arbitrary sign on both sides, at most 2 lr apart per step.  The
            # attention's key bias (in_proj_bias[E:2E]) is such an entry everywhere: its exact
            # gradient is zero (softmax is invariant to a shift of all scores of a query), as
            # in the tuning tests (DESIGN §8 "Parity")
            noise = np.zeros(t["n"], dtype=bool)
            if t["name"] == "mha.in_proj_bias":
                E = t["n"] // 3
                noise[E:2 * E] = True
            tol = 1e-4 * np.abs(want) + 1e-5 * np.abs(want).max()
            bad = (np.abs(got - want) > tol) & ~noise
            if bad.mean() >= 0.01:
                fails.append((t["name"], int(bad.sum()), float(np.abs(got - want).max())))
            if not np.all(np.abs(got - want) <= 2 * lr * 24 * (ep + 1)):
                fails.append((t["name"], "beyond the lr bound", float(np.abs(got - want).max())))
            if t["step"] != float(z[f"ep{ep}/step/{t['name']}"]):
                fails.append((t["name"], "step", t["step"]))
        assert not fails, (ep, fails)
        asc, csc = ft.accuracy(st, wins, z[f"ep{ep}/h0_accuracy"], anom, cls)
        assert asc == pytest.approx(float(z[f"ep{ep}/ascore"]), abs=1.0 / (16 * 24) + 1e-12)
        _cscore_within_decision_bounds(ft, st, z, ep, wins, anom, cls, csc)


def _cscore_within_decision_bounds(ft, st, z, ep, wins, anom, cls, csc):
    """class_accuracy (train.py:75-92) counts, per positive host, whether its
    prototype output is closest to its own class.  The device model is the
    reference's up to fp32 training, so a host's verdict may differ only where
    the reference's own distance margin is inside what that difference can
    move: |d_k(a') - d_k(a)| <= |a' - a|_inf * (|a - P_k|_1 + |a' - a|_1 / 2)
    per distance (d_k = mean over the 2 dims of (a - P_k)^2), plus the device
    prototypes' deviation from the reference's.  The reference's forward is
    restated in fp64 (oracle, pinned) on ITS epoch-end weights and the recorded
    GRU states; its CScore must equal the fixture's, and the device CScore must
    equal the reference's with exactly the in-bound flips applied."""
    from preganplus_amd import train as TR
    n, H = wins.shape[0], 16
    fw = {k[len(f"ep{ep}/p/"):]: torch.tensor(z[k]) for k in z.files if k.startswith(f"ep{ep}/p/")}
    h0 = z[f"ep{ep}/h0_accuracy"]
    with torch.no_grad():
        rp, rq = TO.fpe_t(fw, torch.tensor(wins), torch.tensor(h0))
    rp, rq = rp.numpy().reshape(n, H, 2), rq.numpy().reshape(n, H, 2)
    Pref = np.asarray(z[f"ep{ep}/prototypes"], dtype=np.float64)[:3]
    _, csc_ref = TR.accuracy_scores(rp, rq, anom, cls, Pref)
    assert csc_ref == pytest.approx(float(z[f"ep{ep}/cscore"]), rel=1e-12, abs=1e-12)
    _, dq = ft.forward_many(wins, h0)
    P = np.asarray(st.protos, dtype=np.float64)[:3]

    def hits(q, PP):
        d = np.mean((q[:, :, None, :] - PP[None, None]) ** 2, axis=-1)       # [n,H,3]
        c = np.clip(cls, 0, 2)
        pos = np.take_along_axis(d, c[..., None], -1)[..., 0]
        negs = np.where(np.arange(3)[None, None] == c[..., None], np.inf, d).min(-1)
        return (anom > 0) & (pos <= negs), negs - pos, d

    h_ref, margin, d_ref = hits(rq, Pref)
    h_dev, _, _ = hits(dq, P)
    da = np.abs(dq - rq).max(-1)                                                # per host, inf-norm
    dP = np.abs(P - Pref).max()
    span = np.abs(rq[:, :, None, :] - Pref[None, None]).sum(-1).max(-1)        # max_k |a - P_k|_1
    bound = 2 * ((da + dP) * (span + (da + dP)))                               # pos and neg both move
    flip = h_ref != h_dev
    assert np.all(np.abs(margin[flip]) <= bound[flip]), (np.abs(margin[flip]), bound[flip])
    # the device score is the reference's with those flips: the count is exact
    cc, tot = 0.0, 0
    for i in range(n):
        npos = int(np.sum(anom[i] > 0))
        if npos:
            tot += 1
            cc += int(np.sum(h_dev[i])) / (1e-4 + npos)
    assert csc == pytest.approx(cc / tot, rel=1e-12)
    assert int(flip.sum()) <= max(2, int((np.abs(margin) <= bound).sum()))


def test_fpe_optimizer_state_round_trip():
    """FPETrainer(state=...) restores the AdamW moments and step counts that
    checkpoint() writes (torch's optimizer_state_dict: keyed by parameter
    index): a restored trainer's next step equals the original's."""
    from preganplus_amd import fpetrain as FT
    from preganplus_amd import train as TR
    z, init = _fixture()
    wins, anom, cls = z["wins"][:6], z["anom"][:6], z["cls"][:6]
    h0 = z["ep0/h0_backprop"][:6]
    a = FT.FPETrainer(init)
    st = TR.TuneState(z["init/prototypes"], 0.2)
    a.backprop(st, wins[:4], h0[:4], anom[:4], cls[:4])
    ck = a.checkpoint(0, [], st.protos)
    b = FT.FPETrainer({k: np.asarray(v) for k, v in ck["model_state_dict"].items()},
                      state=ck["optimizer_state_dict"]["state"])
    assert [t["step"] for t in b.tensors] == [t["step"] for t in a.tensors] and a.tensors[0]["step"] > 0
    np.testing.assert_array_equal(b.m.cpu().numpy(), a.m.cpu().numpy())
    np.testing.assert_array_equal(b.v.cpu().numpy(), a.v.cpu().numpy())
    st2 = TR.TuneState(st.protos, st.factor)
    a.backprop(st, wins[4:], h0[4:], anom[4:], cls[4:])
    b.backprop(st2, wins[4:], h0[4:], anom[4:], cls[4:])
    np.testing.assert_array_equal(b.P.cpu().numpy(), a.P.cpu().numpy())


def test_pregan_new_model_trains_offline(tmp_path, monkeypatch):
    """No FPE checkpoint, no packaged weights (the framework environment):
    PreGANRecovery trains a new FPE for num_epochs (here 2, on 30 rows of the
    framework series), rewriting {env}_FPE_16.ckpt each epoch in the
    reference's format, then runs the plugin on the trained encoder."""
    from preganplus_amd import recovery as RC
    from preganplus_amd import weights as W
    rng = np.random.default_rng(4)
    d = tmp_path / "recovery" / "PreGANSrc" / "data" / "framework"
    d.mkdir(parents=True)
    np.save(d / "time_series.npy", rng.uniform(0, 100, size=(30, 48)))
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(RC, "NUM_EPOCHS", 2)
    torch.manual_seed(5)
    rec = RC.PreGANRecovery(16, "framework", training=False, model_folder=str(tmp_path / "ck"))
    assert rec.fpe_epoch == 1 and len(rec.fpe_accuracy_list) == 2
    ck = W._safe_load(str(tmp_path / "ck" / "framework_FPE_16.ckpt"))
    assert int(ck["epoch"]) == 1 and len(ck["accuracy_list"]) == 2 and len(ck["model_prototypes"]) == 3
    fw = rec.fpe_trainer.weights_numpy()
    for k, v in ck["model_state_dict"].items():
        np.testing.assert_array_equal(np.asarray(v), fw[k])
    assert rec.epoch == -1            # a new GAN (load_gan without checkpoints)
    np.testing.assert_array_equal(rec.weights["fpe"]["encoder.0.weight"], fw["encoder.0.weight"])
    # the folder now holds the FPE checkpoint and no GAN ones (training=False never saves
    # them): a second plugin loads the trained FPE and, as load_gan does for absent files
    # (utils.py:81-84), a new GAN at epoch -1
    rec2 = RC.PreGANRecovery(16, "framework", training=True, model_folder=str(tmp_path / "ck"))
    assert rec2.epoch == -1 and rec2.accuracy_list == []
    np.testing.assert_array_equal(rec2.weights["fpe"]["encoder.0.weight"], fw["encoder.0.weight"])
    np.testing.assert_array_equal(rec2.weights["gen"]["delta.0.weight"], rec.weights["gen"]["delta.0.weight"])
