"""GPU parity of the online training steps (HIP kernels through the C-ABI)
against the reference-generated fixtures and the torch training oracle."""
import numpy as np
import pytest
import torch

from oracle import pregan_train_oracle as TO
from preganplus_amd import weights as W

pytestmark = pytest.mark.gpu
GOLD = "tests/golden"


def load16():
    return W.load_npz("preganplus_amd/data/simulator_16.npz")


def close(got, want, rel=2e-4, abs_scale=2e-4, what=""):
    """fp32 HIP vs fp64 reference: |got - want| <= rel*|want| + abs_scale*max|want|."""
    want = np.asarray(want, dtype=np.float64)
    got = np.asarray(got, dtype=np.float64)
    tol = rel * np.abs(want) + abs_scale * (np.abs(want).max() + 1e-30)
    bad = np.abs(got - want) > tol
    assert not bad.any(), f"{what}: {bad.sum()} of {bad.size} off, max err {np.abs(got - want).max():.3e}"


def key_bias_mask(name, n, d=16):
    """The attention key bias has an identically-zero gradient (softmax over the
    keys is invariant to a shift q.b_k shared by all keys), so both the fp64
    reference and the fp32 kernels hold rounding noise there, which AdamW turns
    into O(lr) steps of arbitrary sign: those elements are compared with an
    lr-sized tolerance instead."""
    m = np.zeros(n, dtype=bool)
    if name.endswith("self_attn.in_proj_bias"):
        m[d:2 * d] = True
    return m


def close_params(got, want, name, steps, rel, abs_scale, what):
    got, want = np.asarray(got).reshape(-1), np.asarray(want).reshape(-1)
    kb = key_bias_mask(name, want.size)
    close(got[~kb], want[~kb], rel=rel, abs_scale=abs_scale, what=what)
    assert np.all(np.abs(got[kb] - want[kb]) <= 2e-4 * steps), what + " (key bias)"


def test_tuning_step_matches_reference():
    from preganplus_amd import train as TR
    w, extra = load16()
    z = np.load(f"{GOLD}/tune_h16.npz")
    tr = TR.Trainer(16, w, extra)
    st = TR.TuneState(z["protos0"], float(z["factor0"]))
    wins, anom, cls = z["windows"], z["anom"], z["cls"]
    st.num_zero, st.num_ones = 1, 1
    losses = []
    for i in range(wins.shape[0]):
        logits, protos = tr.tune_forward(torch.tensor(wins[i:i + 1], dtype=torch.float32))
        mult, tgt, aloss, tloss = TR.loss_targets(logits[0].cpu().numpy(), protos[0].cpu().numpy(),
                                                  anom[i], cls[i], st)
        tr.tune_backward(1, anom[i][None], mult[None], tgt[None])
        if i == 0:
            g = tr.G.cpu().numpy()
            for t in tr.tensors:
                if t["section"] == "transformer" and t["trainable"]:
                    close(g[t["offset"]:t["offset"] + t["n"]], z[f"g0/{t['name']}"].reshape(-1),
                          rel=1e-3, abs_scale=1e-4, what="grad " + t["name"])
        inactive = () if np.any(anom[i] > 0) else ("prototype_decoder.0.weight", "prototype_decoder.0.bias")
        tr.adam_step("transformer", inactive)
        if i == 0:
            pw = tr.weights_numpy()["transformer"]
            for k, v in pw.items():
                if k != "pos_encoder.pe":
                    close_params(v, z[f"p1/{k}"], k, 1, rel=1e-5, abs_scale=1e-6, what="p1 " + k)
        losses.append((aloss, tloss))
    np.testing.assert_allclose(np.array(losses), z["losses"], rtol=1e-4, atol=1e-5)
    pw = tr.weights_numpy()["transformer"]
    for k, v in pw.items():
        if k != "pos_encoder.pe":
            close_params(v, z[f"p10/{k}"], k, 10, rel=1e-4, abs_scale=2e-5, what="p10 " + k)
    np.testing.assert_allclose(st.protos, z["protos_steps"][-1], atol=1e-5)
    assert abs(st.factor - float(z["factor_end"])) < 1e-12
    assert st.num_zero == z["num_zero"] and st.num_ones == z["num_ones"]


@pytest.mark.parametrize("tag,scores", [("better", [1.0, 2.0]), ("worse", [3.0, 1.0])])
def test_gan_step_matches_reference(tag, scores):
    from preganplus_amd import train as TR
    w, extra = load16()
    z = np.load(f"{GOLD}/gan_h16.npz")
    tr = TR.Trainer(16, w, extra)
    it = iter(scores)
    ns, _, _, _, _ = TR.train_gan(tr, z["emb"], z["sched"], lambda s: next(it))
    np.testing.assert_allclose(ns, z[f"{tag}/sim_new"], rtol=1e-4, atol=1e-5)
    pw = tr.weights_numpy()
    for k, v in pw["gen"].items():
        close(v, z[f"{tag}/gen/{k}"], rel=1e-5, abs_scale=1e-6, what="gen " + k)
    for k, v in pw["disc"].items():
        close(v, z[f"{tag}/disc/{k}"], rel=1e-5, abs_scale=1e-6, what="disc " + k)


def test_plugin_run_model_matches_reference():
    from preganplus_amd.recovery import PreGANPlusRecovery
    from tests.test_train_oracle_golden import fake_env
    w, extra = load16()
    z = np.load(f"{GOLD}/plugin_h16.npz")
    tr_time = extra["train_time_data"]
    rec = PreGANPlusRecovery(16, "", training=True, weights=w, extra=extra)
    for step in range(4):
        env = fake_env(z, step, tr_time, z["schedule_series"])
        rec.setEnvironment(env)
        dec = rec.run_model(None, [tuple(x) for x in z[f"s{step}/decision_in"]])
        assert [tuple(map(int, d)) for d in dec] == [tuple(x) for x in z[f"s{step}/decision_out"].tolist()], step
    pw = rec.trainer.weights_numpy()
    for k, v in pw["transformer"].items():
        if k != "pos_encoder.pe":
            close_params(v, z[f"end/t/{k}"], k, 40, rel=1e-3, abs_scale=1e-4, what="t " + k)
    for k, v in pw["gen"].items():
        close(v, z[f"end/g/{k}"], rel=1e-4, abs_scale=1e-5, what="g " + k)
    np.testing.assert_allclose(rec.tune_state.protos, z["end/protos"], atol=1e-4)
    check_accuracy_list(rec.accuracy_list, z)
    assert rec.epoch == int(extra["meta/gen/epoch"]) + 4     # one GAN epoch per call (PreGANPlus.py:77)


def check_accuracy_list(got, z):
    """accuracy_list entries appended by run_model (PreGANPlus.py:58, 77): per
    call (gen_loss, disc_loss), then (loss, factor, AScore, CScore) — the
    scores are ratios of counts and must be exact."""
    lens = z["end/accuracy_list_lens"].tolist()
    assert [len(e) for e in got[-len(lens):]] == lens
    flat = np.concatenate([np.asarray(e, dtype=np.float64) for e in got[-len(lens):]])
    want = z["end/accuracy_list"]
    o = 0
    for n in lens:
        g, w = flat[o:o + n], want[o:o + n]
        if n == 2:
            np.testing.assert_allclose(g, w, rtol=1e-4, atol=1e-6, err_msg="(gen_loss, disc_loss)")
        else:
            np.testing.assert_allclose(g[:2], w[:2], rtol=1e-4, atol=1e-5, err_msg="(loss, factor)")
            np.testing.assert_array_equal(g[2:], w[2:], err_msg="(AScore, CScore)")
        o += n


def _batched_case(H, B, seed):
    w = W.synth_weights(H, seed=seed)
    rng = np.random.Generator(np.random.PCG64(9 + H + B))
    x = rng.uniform(0, 0.8, size=(B, 3, 3 * H))
    spike = rng.uniform(size=x.shape) < 0.03
    x = np.where(spike, rng.uniform(0.9, 1.3, size=x.shape), x)
    y = (rng.uniform(size=(B, H)) < 0.3).astype(np.int32)
    mult = rng.uniform(0.5, 2.0, size=(B, H))
    tgt = rng.uniform(0, 1, size=(B, H, 2))
    return w, x, y, mult, tgt


def _autograd(w, x, y, mult, tgt):
    B, H = y.shape
    tw = TO.leaf_params(w["transformer"])
    lat = TO.encode_t(tw, torch.tensor(x))
    logits, protos = TO.decode_t(tw, lat)
    ce = torch.nn.functional.cross_entropy(logits.reshape(-1, 2), torch.tensor(y.reshape(-1), dtype=torch.long),
                                           reduction="none").reshape(B, H)
    loss = (ce * torch.tensor(mult)).sum()
    loss = loss + (((protos - torch.tensor(tgt)) ** 2).mean(-1) * torch.tensor(y > 0)).sum()
    loss.backward()
    return tw, lat.detach().numpy(), logits.detach().numpy(), protos.detach().numpy()


@pytest.mark.parametrize("H,B", [(8, 5), (16, 37), (32, 9), (50, 3), (50, 21), (64, 4), (16, 300), (50, 256)])
def test_batched_tuning_step_matches_autograd(H, B):
    """Token-major MFMA tuning step (pgp_tune.hip) on a ragged batch: logits,
    protos and the latent tap within fp32 tolerance of the fp64 forward, and
    every transformer gradient == autograd of the summed per-window losses
    (fixed labels / CE weights / targets) — the DP tuning semantics."""
    from preganplus_amd import train as TR
    w, x, y, mult, tgt = _batched_case(H, B, seed=3)
    tr = TR.Trainer(H, w, max_batch=B)
    lat = torch.empty((B, 3 * H * H), dtype=torch.float32, device=tr.device)
    logits, protos = tr.tune_forward(torch.tensor(x, dtype=torch.float32), latent=lat)
    tr.tune_backward(B, y, mult, tgt)
    g = tr.G.cpu().numpy()
    tw, lat_r, logits_r, protos_r = _autograd(w, x, y, mult, tgt)
    close(lat.cpu().numpy(), lat_r, rel=1e-4, abs_scale=1e-5, what="latent")
    close(logits.cpu().numpy(), logits_r, rel=1e-4, abs_scale=1e-5, what="logits")
    close(protos.cpu().numpy(), protos_r, rel=1e-4, abs_scale=1e-5, what="protos")
    for t in tr.tensors:
        if t["section"] == "transformer" and t["trainable"]:
            ref = tw[t["name"]].grad.numpy().reshape(-1)
            close(g[t["offset"]:t["offset"] + t["n"]], ref, rel=1e-3, abs_scale=1e-4, what=t["name"])
    assert np.all(g[tr.sec_end["transformer"]:] == 0)


def test_batched_tuning_step_is_deterministic():
    """Weight gradients are reduced from fixed partial slabs in a fixed order:
    two identical steps give bit-identical gradients."""
    from preganplus_amd import train as TR
    H, B = 50, 130
    w, x, y, mult, tgt = _batched_case(H, B, seed=5)
    tr = TR.Trainer(H, w, max_batch=B)
    xs = torch.tensor(x, dtype=torch.float32)
    gs = []
    for _ in range(2):
        tr.tune_forward(xs)
        tr.tune_backward(B, y, mult, tgt)
        gs.append(tr.G.cpu().numpy().copy())
    assert np.array_equal(gs[0], gs[1])


@pytest.mark.parametrize("H,B", [(16, 1), (16, 7), (16, 103), (50, 3), (50, 103), (50, 256)])
def test_split_gan_forward_repeats_bit_identical(H, B):
    """The GAN forward at small batches runs split over k-slices whose partials
    meet in LDS reductions and a last-arriver sum (pgp_gantrain.hip; a missing
    barrier between two LDS reductions made round 5's first version race).
    Twenty launches on the same inputs, interleaved with launches on other
    batch sizes that reuse the same workspace, must give the same bits."""
    from preganplus_amd import train as TR
    w = W.synth_weights(H, seed=6)
    rng = np.random.Generator(np.random.PCG64(40 + H + B))
    emb = np.where(rng.uniform(size=(B, H, 1)) < 0.3, rng.uniform(size=(B, H, 2)), 0.0).astype(np.float32)
    sched = np.zeros((B, H, H), np.float32)
    sched[np.arange(B)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(B, H))] = 1.0
    other = np.zeros((2 * B + 5, H, H), np.float32)
    other[:, np.arange(H), 0] = 1.0
    tr = TR.Trainer(H, w, max_batch=2 * B + 5)
    e = torch.tensor(emb, device="cuda")
    s = torch.tensor(sched, device="cuda")
    eo = torch.zeros((2 * B + 5, H, 2), device="cuda")
    so = torch.tensor(other, device="cuda")
    first = None
    for i in range(20):
        ns, pr = tr.gan_forward(e, s)
        got = (ns.cpu().numpy().copy(), pr.cpu().numpy().copy())
        if first is None:
            first = got
        else:
            assert np.array_equal(got[0], first[0]) and np.array_equal(got[1], first[1]), i
        if i % 3 == 0:
            tr.gan_forward(eo, so)   # another batch through the same workspace in between
    torch.cuda.synchronize()


@pytest.mark.parametrize("H", [16, 50])
def test_smaller_batch_after_larger_is_unchanged(H):
    """The workspace regions move with B, so a batch smaller than the previous
    one lands on that batch's data (run_model's detect window after a tune
    step): its forward + backward equal a fresh trainer's bit for bit."""
    from preganplus_amd import train as TR
    Bbig, B = 300, 23
    w, xb, yb, mb, tb = _batched_case(H, Bbig, seed=11)
    _, x, y, mult, tgt = _batched_case(H, B, seed=12)
    a, b = TR.Trainer(H, w, max_batch=Bbig), TR.Trainer(H, w, max_batch=Bbig)
    a.tune_forward(torch.tensor(xb, dtype=torch.float32))
    a.tune_backward(Bbig, yb, mb, tb)
    out = []
    for tr in (a, b):
        lg, pr = tr.tune_forward(torch.tensor(x, dtype=torch.float32))
        tr.tune_backward(B, y, mult, tgt)
        out.append((lg.cpu().numpy().copy(), pr.cpu().numpy().copy(), tr.G.cpu().numpy().copy()))
    for u, v in zip(*out):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("H,B", [(8, 3), (16, 37), (50, 21), (64, 5), (16, 300)])
def test_batched_gan_step_matches_autograd(H, B):
    """GAN step over a ragged batch (pgp_gantrain.hip): new schedule and Disc
    probabilities within fp32 tolerance of the fp64 forward; Disc gradients of
    the summed BCE toward per-window targets, and Gen gradients of the summed
    BCE toward [0,1] through the (unchanged) Disc == autograd (PreGANPlus.py:60-74)."""
    from preganplus_amd import train as TR
    w = W.synth_weights(H, seed=4)
    rng = np.random.Generator(np.random.PCG64(21 + H + B))
    emb = np.where(rng.uniform(size=(B, H, 1)) < 0.3, rng.uniform(size=(B, H, 2)), 0.0)
    sched = np.zeros((B, H, H))
    sched[np.arange(B)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(B, H))] = 1.0
    lab = rng.uniform(size=B) < 0.5
    target = np.stack([1.0 - lab, lab], axis=1).astype(np.float64)
    tr = TR.Trainer(H, w, max_batch=B)
    ns, probs = tr.gan_forward(emb, sched)
    ns, probs = ns.cpu().numpy(), probs.cpu().numpy()
    tr.gan_disc_backward(target)
    tr.gan_gen_backward(B)
    g = tr.G.cpu().numpy()
    gw = TO.leaf_params(w["gen"])
    dw = TO.leaf_params(w["disc"])
    e_t, s_t = torch.tensor(emb), torch.tensor(sched)
    ns_r = TO.gen_t(gw, e_t, s_t)
    p_r = TO.disc_t(dw, s_t, ns_r.detach())
    close(ns, ns_r.detach().numpy(), rel=1e-4, abs_scale=1e-5, what="ns")
    close(probs, p_r.detach().numpy(), rel=1e-4, abs_scale=1e-5, what="probs")
    bce = torch.nn.functional.binary_cross_entropy
    torch.stack([bce(p_r[i], torch.tensor(target[i])) for i in range(B)]).sum().backward()
    for t in tr.tensors:
        if t["section"] == "disc":
            close(g[t["offset"]:t["offset"] + t["n"]], dw[t["name"]].grad.numpy().reshape(-1), rel=1e-3,
                  abs_scale=1e-4, what="disc " + t["name"])
    for p in dw.values():
        p.grad = None
    p2 = TO.disc_t(dw, s_t, ns_r)
    torch.stack([bce(p2[i], torch.tensor([0.0, 1.0], dtype=torch.float64)) for i in range(B)]).sum().backward()
    for t in tr.tensors:
        if t["section"] == "gen":
            close(g[t["offset"]:t["offset"] + t["n"]], gw[t["name"]].grad.numpy().reshape(-1), rel=1e-3,
                  abs_scale=1e-4, what="gen " + t["name"])


def test_dp_tune_step_single_rank():
    """dp_tune_step on one rank == its pieces run by hand:
    forward, loss_targets_dp on the step-start state, backward, AdamW, state
    update; parameters bit-identical, state updated (device bookkeeping,
    DPTuner, vs the numpy restatement)."""
    from preganplus_amd import train as TR
    H, B = 16, 12
    w = W.synth_weights(H, seed=6)
    rng = np.random.Generator(np.random.PCG64(5))
    wins = rng.uniform(0, 0.8, size=(B, 3, 3 * H)).astype(np.float32)
    anom = (rng.uniform(size=(B, H)) < 0.3).astype(np.int32)
    cls = rng.integers(0, 3, size=(B, H))
    p0 = np.array([[0.2, 0.3], [0.6, 0.1], [0.5, 0.9]])
    t1, s1 = TR.Trainer(H, w, max_batch=B), TR.TuneState(p0.copy())
    TR.dp_tune_step(t1, s1, wins, anom, cls)
    t2, s2 = TR.Trainer(H, w, max_batch=B), TR.TuneState(p0.copy())
    lg, pr = t2.tune_forward(torch.tensor(wins))
    mult, tgt, _, _, inc = TR.loss_targets_dp(lg.cpu().numpy(), pr.cpu().numpy(), anom, cls, s2)
    t2.tune_backward(B, anom, mult, tgt)
    t2.adam_step("transformer")
    TR.dp_state_update(s2, inc)
    torch.cuda.synchronize()
    assert torch.equal(t1.P, t2.P)
    # the device sums the batch's EMA deltas in a tree order, numpy sequentially
    np.testing.assert_allclose(s1.protos, s2.protos, rtol=1e-13, atol=1e-15)
    assert not np.array_equal(s1.protos, p0) and s1.num_ones > 1


def test_backprop_device_bookkeeping_matches_reference():
    """TR.backprop (custom_loss bookkeeping on the device, no host round trip
    between steps) against the same reference fixture as the host-loop test."""
    from preganplus_amd import train as TR
    w, extra = load16()
    z = np.load(f"{GOLD}/tune_h16.npz")
    tr = TR.Trainer(16, w, extra)
    st = TR.TuneState(z["protos0"], float(z["factor0"]))
    losses = TR.backprop(tr, st, z["windows"], z["anom"], z["cls"])
    np.testing.assert_allclose(np.array(losses), z["losses"], rtol=1e-4, atol=1e-5)
    pw = tr.weights_numpy()["transformer"]
    for k, v in pw.items():
        if k != "pos_encoder.pe":
            close_params(v, z[f"p10/{k}"], k, 10, rel=1e-4, abs_scale=2e-5, what="p10 " + k)
    np.testing.assert_allclose(st.protos, z["protos_steps"][-1], atol=1e-5)
    assert abs(st.factor - float(z["factor_end"])) < 1e-12
    assert st.num_zero == z["num_zero"] and st.num_ones == z["num_ones"]


@pytest.mark.parametrize("H", [16, 50])
def test_tune_targets_bit_exact_vs_host_bookkeeping(H):
    """pgp_tune_targets vs train.loss_targets (the numpy restatement of
    train.py:13-40) over 40 consecutive windows of random forward outputs:
    mult, tgt and the fp64 state (prototype EMA, factor, counters) bit-exact,
    loss values to fp64 rounding.  Anchors are drawn near the class prototypes
    so both outcomes of the EMA condition occur."""
    from preganplus_amd import train as TR
    rng = np.random.default_rng(7 + H)
    w = W.synth_weights(H, seed=3) if H != 16 else load16()[0]
    tr = TR.Trainer(H, w, None)
    protos0 = rng.uniform(0.1, 0.9, (H, 2))  # K = n_hosts prototypes (models.py:373)
    st_h = TR.TuneState(protos0, 0.2)
    st_d = TR.TuneState(protos0, 0.2)
    dev = tr.device
    state = st_d.to_device(dev)
    mult = torch.empty((1, H), dtype=torch.float32, device=dev)
    tgt = torch.empty((1, H, 2), dtype=torch.float32, device=dev)
    loss = torch.empty(2, dtype=torch.float64, device=dev)
    ema_hits = 0
    for it in range(40):
        y = (rng.random(H) < 0.4).astype(np.int32)
        c = rng.integers(0, 3, H).astype(np.int32)
        lg = rng.normal(0, 2, (H, 2)).astype(np.float32)
        pr = np.clip(protos0[c] + rng.normal(0, 0.15, (H, 2)), 0, 1).astype(np.float32)
        tr.logits[0].copy_(torch.from_numpy(lg))
        tr.protos[0].copy_(torch.from_numpy(pr))
        tr._fwd_batch = 1
        before = st_h.protos.copy()
        m_h, t_h, a_h, l_h = TR.loss_targets(lg, pr, y, c, st_h)
        ema_hits += int(np.any(before != st_h.protos))
        tr.tune_targets(torch.from_numpy(y).to(dev), torch.from_numpy(c).to(dev), state, mult, tgt, loss)
        np.testing.assert_array_equal(mult[0].cpu().numpy(), m_h.astype(np.float32))
        np.testing.assert_array_equal(tgt[0].cpu().numpy(), t_h.astype(np.float32))
        st_d.from_device(state)
        np.testing.assert_array_equal(st_d.protos, st_h.protos)
        assert st_d.factor == st_h.factor
        assert (st_d.num_zero, st_d.num_ones) == (st_h.num_zero, st_h.num_ones)
        np.testing.assert_allclose(loss.cpu().numpy(), [a_h, l_h], rtol=1e-12, atol=1e-12)
    assert ema_hits > 5


def _host_loop_backprop(tr, st, wins, anom, cls):
    """backprop as a plain host loop: numpy bookkeeping (loss_targets) and one
    adam_step launch per step, synchronising every step."""
    from preganplus_amd import train as TR
    st.num_zero, st.num_ones = 1, 1
    out = []
    for i in range(wins.shape[0]):
        logits, protos = tr.tune_forward(torch.as_tensor(wins[i:i + 1], dtype=torch.float32))
        mult, tgt, aloss, tloss = TR.loss_targets(logits[0].cpu().numpy(), protos[0].cpu().numpy(),
                                                  anom[i], cls[i], st)
        tr.tune_backward(1, anom[i][None], mult[None], tgt[None])
        inactive = () if np.any(anom[i] > 0) else ("prototype_decoder.0.weight", "prototype_decoder.0.bias")
        tr.adam_step("transformer", inactive)
        out.append((aloss, tloss))
    return out


def test_backprop_graph_bit_identical_to_host_loop():
    """The graph-replayed backprop (device bookkeeping, AdamW table; the
    per-kernel step, fused=False) produces the same bits as the host loop over
    three consecutive calls (capture, then two replays with new inputs),
    including a window with no anomaly (inactive prototype decoder) and a
    shorter call (a second cached graph).  The fused step is checked against
    this path and the reference in test_gpu_tune1.py."""
    from preganplus_amd import train as TR
    w, extra = load16()
    z = np.load(f"{GOLD}/tune_h16.npz")
    wins, anom, cls = z["windows"], z["anom"].copy(), z["cls"]
    anom[3] = 0
    a, b = TR.Trainer(16, w, extra), TR.Trainer(16, w, extra)
    sa, sb = TR.TuneState(z["protos0"], float(z["factor0"])), TR.TuneState(z["protos0"], float(z["factor0"]))
    rng = np.random.default_rng(0)
    for call, n in enumerate([10, 10, 6]):
        idx = rng.permutation(wins.shape[0])[:n] if call else np.arange(n)
        la = _host_loop_backprop(a, sa, wins[idx], anom[idx], cls[idx])
        lb = TR.backprop(b, sb, wins[idx], anom[idx], cls[idx], fused=False)
        np.testing.assert_array_equal(a.P.cpu().numpy(), b.P.cpu().numpy())
        np.testing.assert_array_equal(a.m.cpu().numpy(), b.m.cpu().numpy())
        np.testing.assert_array_equal(a.v.cpu().numpy(), b.v.cpu().numpy())
        np.testing.assert_array_equal(sa.protos, sb.protos)
        assert (sa.factor, sa.num_zero, sa.num_ones) == (sb.factor, sb.num_zero, sb.num_ones)
        assert [t["step"] for t in a.tensors] == [t["step"] for t in b.tensors]
        np.testing.assert_allclose(np.array(lb), np.array(la), rtol=1e-12, atol=1e-12)
    assert len(b._graphs) == 2


# ---------------------------------------------------------------------------
# H = 50 against the reference's own modules (tests/golden/make_golden_train50.py)
# ---------------------------------------------------------------------------
def _dclose(rel, abs_scale, H=50, steps=None):
    """close() on a digest part; full in_proj_bias parts get the key-bias
    treatment (identically-zero gradient, see key_bias_mask)."""
    def f(got, want, what):
        if steps is not None and what.endswith("self_attn.in_proj_bias/full"):
            kb = key_bias_mask("self_attn.in_proj_bias", want.size, d=H)
            close(got[~kb], want[~kb], rel=rel, abs_scale=abs_scale, what=what)
            assert np.all(np.abs(got[kb] - want[kb]) <= 2e-4 * steps), what + " (key bias)"
        else:
            close(got, want, rel=rel, abs_scale=abs_scale, what=what)
    return f


def _param_close(z, k, steps, rel, abs_scale, lr=1e-4, H=50):
    """Parameters after `steps` fresh-AdamW steps.  AdamW's first step moves
    every entry by ~lr * g / |g|, so an entry whose fp64 gradient is below the
    fp32 gradient's own absolute accuracy (1e-4 of the tensor's largest
    gradient, as the gradient check allows) takes a step whose sign is rounding
    noise on both sides: those entries (and the key bias, see key_bias_mask) are
    held to 2 lr per step; all others to rel / abs_scale."""
    from tests.golden import digest as D
    g = D.parts(z, f"g0/{k}")

    def cmp(got, want, what):
        part = what.rsplit("/", 1)[1]
        gr = g[part].reshape(-1)
        noise = np.abs(gr) <= 1e-4 * np.abs(gr).max()
        if part == "full" and k.endswith("self_attn.in_proj_bias"):
            noise |= key_bias_mask(k, want.size, d=H)
        got, want = got.reshape(-1), want.reshape(-1)
        close(got[~noise], want[~noise], rel=rel, abs_scale=abs_scale, what=what)
        assert np.all(np.abs(got[noise] - want[noise]) <= 2 * lr * steps), what + " (noise-level gradients)"
    return cmp


def test_tuning_step_matches_reference_h50():
    """backprop (train.py:42-57) at H=50 vs the reference's own modules: step-0
    gradients, parameters after steps 1 and 10, prototypes and counters."""
    from preganplus_amd import train as TR
    from tests.golden import digest as D
    H = 50
    w = W.synth_weights(H, 0)
    z = np.load(f"{GOLD}/tune_h50.npz")
    tr = TR.Trainer(H, w)
    st = TR.TuneState(w["prototypes"], float(z["factor0"]))
    wins, anom, cls = z["windows"], z["anom"], z["cls"]
    st.num_zero, st.num_ones = 1, 1
    losses = []
    for i in range(wins.shape[0]):
        logits, protos = tr.tune_forward(torch.tensor(wins[i:i + 1], dtype=torch.float32))
        mult, tgt, aloss, tloss = TR.loss_targets(logits[0].cpu().numpy(), protos[0].cpu().numpy(),
                                                  anom[i], cls[i], st)
        tr.tune_backward(1, anom[i][None], mult[None], tgt[None])
        if i == 0:
            g = tr.G.cpu().numpy()
            for t in tr.tensors:
                if t["section"] == "transformer" and t["trainable"]:
                    D.check(z, f"g0/{t['name']}", g[t["offset"]:t["offset"] + t["n"]].reshape(
                        w["transformer"][t["name"]].shape), _dclose(1e-3, 1e-4), sum_rel=1e-4, key=t["name"])
        inactive = () if np.any(anom[i] > 0) else ("prototype_decoder.0.weight", "prototype_decoder.0.bias")
        tr.adam_step("transformer", inactive)
        if i == 0:
            for k, v in tr.weights_numpy()["transformer"].items():
                if k != "pos_encoder.pe":
                    D.check(z, f"p1/{k}", v, _param_close(z, k, 1, 1e-5, 1e-6), key=k)
        losses.append((aloss, tloss))
    np.testing.assert_allclose(np.array(losses), z["losses"], rtol=1e-4, atol=1e-5)
    for k, v in tr.weights_numpy()["transformer"].items():
        if k != "pos_encoder.pe":
            D.check(z, f"p10/{k}", v, _param_close(z, k, 10, 1e-4, 2e-5), key=k)
    np.testing.assert_allclose(st.protos[:3], z["protos_steps"][-1], atol=1e-5)
    assert abs(st.factor - float(z["factor_end"])) < 1e-12
    assert st.num_zero == z["num_zero"] and st.num_ones == z["num_ones"]


@pytest.mark.parametrize("tag,scores", [("better", [1.0, 2.0]), ("worse", [3.0, 1.0])])
def test_gan_step_matches_reference_h50(tag, scores):
    from preganplus_amd import train as TR
    from tests.golden import digest as D
    w = W.synth_weights(50, 0)
    z = np.load(f"{GOLD}/gan_h50.npz")
    tr = TR.Trainer(50, w)
    it = iter(scores)
    ns, _, _, _, _ = TR.train_gan(tr, z["emb"], z["sched"], lambda s: next(it))
    np.testing.assert_allclose(ns, z[f"{tag}/sim_new"], rtol=1e-4, atol=1e-5)
    pw = tr.weights_numpy()
    for k, v in pw["gen"].items():
        D.check(z, f"{tag}/gen/{k}", v, _dclose(1e-5, 1e-6), sum_rel=1e-5, key=k)
    for k, v in pw["disc"].items():
        D.check(z, f"{tag}/disc/{k}", v, _dclose(1e-5, 1e-6), sum_rel=1e-5, key=k)


def test_dp_step_b1024_h50_matches_reference():
    """C3's local batch: the product's data-parallel step (train.dp_tune_step)
    on 1,024 windows at H=50 vs the reference modules under the DP loss
    (dp_h50_b1024.npz): per-window losses, every transformer gradient, and the
    state after the step (prototype EMA increments, counters, factor)."""
    from preganplus_amd import train as TR
    from tests.golden import digest as D
    from tests.test_train_oracle_golden import dp_inputs
    H = 50
    w = W.synth_weights(H, 0)
    z = np.load(f"{GOLD}/dp_h50_b1024.npz")
    x, y, c = dp_inputs(z), z["y"], z["c"]
    B = y.shape[0]
    tr = TR.Trainer(H, w, max_batch=B)
    st = TR.TuneState(w["prototypes"], float(z["factor"]))
    st.num_zero, st.num_ones = float(z["num_zero"]), float(z["num_ones"])
    p0 = st.protos.copy()
    aloss, tloss = TR.dp_tune_step(tr, st, x.astype(np.float32), y, c)
    np.testing.assert_allclose(np.stack([aloss, tloss], 1), z["losses"], rtol=1e-4, atol=2e-3)
    g = tr.G.cpu().numpy()
    for t in tr.tensors:
        if t["section"] == "transformer" and t["trainable"]:
            D.check(z, f"grad/{t['name']}", g[t["offset"]:t["offset"] + t["n"]].reshape(
                w["transformer"][t["name"]].shape), _dclose(1e-3, 1e-4), sum_rel=1e-4, key=t["name"])
    cnt = z["count"]
    want = p0.copy()
    want[:3] += z["delta"] / np.maximum(cnt, 1)[:, None]
    np.testing.assert_allclose(st.protos, want, atol=1e-5)
    assert st.num_zero == z["num_zero"] + B * H and st.num_ones == z["num_ones"] + y.sum()
    assert abs(st.factor - float(z["factor"]) * 0.995 ** B) < 1e-12


def test_gan_step_b1024_h50_matches_reference():
    """The batched GAN step at C3's local batch vs the reference Gen_50/Disc_50
    over the same 1,024 windows: new schedules, Disc gradients (per-window BCE
    targets) and Gen gradients (BCE toward [0, 1] through the Disc)."""
    from preganplus_amd import train as TR
    from tests.golden import digest as D
    H = 50
    w = W.synth_weights(H, 0)
    z = np.load(f"{GOLD}/dp_h50_b1024.npz")
    emb, sidx, target = z["gan/emb"], z["gan/sidx"], z["gan/target"]
    B = emb.shape[0]
    s = np.zeros((B, H, H), np.float32)
    s[np.arange(B)[:, None], np.arange(H)[None, :], sidx] = 1.0
    tr = TR.Trainer(H, w, max_batch=B)
    ns, _ = tr.gan_forward(emb, s)
    D.check(z, "gan/ns", ns.cpu().numpy(), _dclose(1e-4, 1e-5), sum_rel=1e-5)
    tr.gan_disc_backward(target)
    tr.gan_gen_backward(B)
    g = tr.G.cpu().numpy()
    for t in tr.tensors:
        sec = {"disc": "gan/dgrad", "gen": "gan/ggrad"}.get(t["section"])
        if sec:
            D.check(z, f"{sec}/{t['name']}", g[t["offset"]:t["offset"] + t["n"]].reshape(
                w[t["section"]][t["name"]].shape), _dclose(1e-3, 1e-4), sum_rel=1e-4, key=t["name"])


@pytest.mark.parametrize("H", [16, 50])
def test_reserved_cus_same_gradients(H):
    """pgp_tune_reserve_cus (the C3 bench leaves 8 CUs to the GAN stream): the
    fused launches then run on fewer workgroups, so units are dealt differently
    and the weight gradients are summed in other fp32 groupings; the gradients
    agree with the full-grid step to fp32 summation tolerance, and two reserved
    steps are bit-identical (still one fixed slab per workgroup)."""
    import ctypes
    from preganplus_amd import _native
    from preganplus_amd import train as TR
    B = 1030
    w, x, y, mult, tgt = _batched_case(H, B, seed=9)
    tr = TR.Trainer(H, w, max_batch=B)
    xs = torch.tensor(x, dtype=torch.float32)
    L = _native.lib()
    L.pgp_tune_reserve_cus.argtypes = [ctypes.c_int]

    def grads(n):
        _native.check(L.pgp_tune_reserve_cus(n), "pgp_tune_reserve_cus")
        tr.tune_forward(xs)
        tr.tune_backward(B, y, mult, tgt)
        return tr.G.cpu().numpy().copy()
    try:
        g0 = grads(0)
        g8, g8b = grads(8), grads(8)
        g128 = grads(200)      # clamped to half the CUs
    finally:
        _native.check(L.pgp_tune_reserve_cus(0), "pgp_tune_reserve_cus")
    assert np.array_equal(g8, g8b)
    for g in (g8, g128):
        for t in tr.tensors:
            if t["section"] == "transformer" and t["trainable"]:
                sl = slice(t["offset"], t["offset"] + t["n"])
                close(g[sl], g0[sl], rel=1e-4, abs_scale=1e-5, what=f"reserved {t['name']}")
