"""GPU parity of the fused batch-1 tuning step (pgp_tune1.hip, ``pgp_tune_step1``):
one launch doing the Transformer forward, custom_loss / triplet_loss
bookkeeping and the backward of ONE window (train.py:46-53).

* against autograd of the fp64 torch oracle (gradients of the window's loss
  with the mult / tgt the device bookkeeping chose, which the numpy
  restatement must reproduce bit for bit from the kernel's own outputs);
* against the per-kernel path (tune_forward / tune_targets / tune_backward)
  over whole backprop() calls, and the reference fixture (tune_h16.npz) via
  test_gpu_train.test_backprop_device_bookkeeping_matches_reference, which runs
  the fused step by default at 16 hosts.
"""
import numpy as np
import pytest
import torch

from oracle import pregan_train_oracle as TO
from preganplus_amd import weights as W
from tests.test_gpu_train import close, close_params, load16

pytestmark = pytest.mark.gpu
GOLD = "tests/golden"


def _window(rng, H):
    x = rng.uniform(0, 0.8, size=(3, 3 * H))
    spike = rng.uniform(size=x.shape) < 0.05
    return np.where(spike, rng.uniform(0.9, 1.3, size=x.shape), x)


@pytest.mark.parametrize("H,seed,pos", [(8, 1, 0.4), (16, 2, 0.4), (16, 3, 0.0), (16, 4, 1.0), (8, 5, 0.1)])
def test_fused_step_matches_autograd(H, seed, pos):
    from preganplus_amd import train as TR
    rng = np.random.default_rng(seed)
    w = load16()[0] if (H == 16 and seed == 2) else W.synth_weights(H, seed=seed)
    tr = TR.Trainer(H, w, max_batch=1)
    dev = tr.device
    x = _window(rng, H)
    y = (rng.random(H) < pos).astype(np.int32)
    c = rng.integers(0, 3, H).astype(np.int32)
    protos0 = rng.uniform(0.1, 0.9, (H, 2))
    st_h, st_d = TR.TuneState(protos0, 0.2), TR.TuneState(protos0, 0.2)
    st_h.num_zero, st_h.num_ones = st_d.num_zero, st_d.num_ones = 7, 3
    state = st_d.to_device(dev)
    loss = torch.zeros(2, dtype=torch.float64, device=dev)
    sentinel = torch.full((tr.P.numel() - tr.sec_end["transformer"],), 7.0, device=dev)
    tr.G[tr.sec_end["transformer"]:].copy_(sentinel)
    tr.G[:tr.sec_end["transformer"]].fill_(float("nan"))        # every transformer entry must be written
    win = torch.tensor(x, dtype=torch.float32, device=dev)
    tr.tune_step1(win, torch.from_numpy(y).to(dev), torch.from_numpy(c).to(dev), state, loss)
    torch.cuda.synchronize()
    lg, pr = tr.logits[0].cpu().numpy(), tr.protos[0].cpu().numpy()
    # the kernel's bookkeeping == the numpy restatement on the kernel's own outputs
    mult, tgt, a_h, l_h = TR.loss_targets(lg, pr, y, c, st_h)
    st_d.from_device(state)
    np.testing.assert_array_equal(st_d.protos, st_h.protos)
    assert (st_d.factor, st_d.num_zero, st_d.num_ones) == (st_h.factor, st_h.num_zero, st_h.num_ones)
    np.testing.assert_allclose(loss.cpu().numpy(), [a_h, l_h], rtol=1e-12, atol=1e-12)
    # forward and gradients vs autograd of the fp64 oracle with those targets
    tw = TO.leaf_params(w["transformer"])
    lat = TO.encode_t(tw, torch.tensor(x[None]))
    logits, protos = TO.decode_t(tw, lat)
    close(lg, logits.detach().numpy()[0], rel=1e-4, abs_scale=1e-5, what="logits")
    close(pr, protos.detach().numpy()[0], rel=1e-4, abs_scale=1e-5, what="protos")
    ce = torch.nn.functional.cross_entropy(logits.reshape(-1, 2), torch.tensor(y, dtype=torch.long),
                                           reduction="none")
    L = (ce * torch.tensor(np.asarray(mult, np.float32).astype(np.float64))).sum()
    L = L + (((protos[0] - torch.tensor(np.asarray(tgt, np.float32).astype(np.float64))) ** 2).mean(-1)
             * torch.tensor(y > 0)).sum()
    L.backward()
    g = tr.G.cpu().numpy()
    for t in tr.tensors:
        if t["section"] != "transformer":
            continue
        seg = g[t["offset"]:t["offset"] + t["n"]]
        if not t["trainable"]:
            assert np.all(seg == 0), t["name"]
            continue
        gr = tw[t["name"]].grad
        ref = np.zeros(t["n"]) if gr is None else gr.numpy().reshape(-1)
        close(seg, ref, rel=1e-3, abs_scale=1e-4, what=t["name"])
    assert torch.equal(tr.G[tr.sec_end["transformer"]:], sentinel)


def test_fused_backprop_matches_per_kernel_path():
    """Three backprop() calls on the reference fixture's windows: the fused
    graph (2 launches per step) vs the per-kernel graph — parameters within the
    fp32 tolerance the reference comparison uses, state and losses close."""
    from preganplus_amd import train as TR
    w, extra = load16()
    z = np.load(f"{GOLD}/tune_h16.npz")
    wins, anom, cls = z["windows"], z["anom"].copy(), z["cls"]
    anom[3] = 0
    a, b = TR.Trainer(16, w, extra), TR.Trainer(16, w, extra)
    sa, sb = TR.TuneState(z["protos0"], float(z["factor0"])), TR.TuneState(z["protos0"], float(z["factor0"]))
    rng = np.random.default_rng(1)
    steps = 0
    for call, n in enumerate([10, 10, 6]):
        idx = rng.permutation(wins.shape[0])[:n] if call else np.arange(n)
        la = TR.backprop(a, sa, wins[idx], anom[idx], cls[idx], fused=False)
        lb = TR.backprop(b, sb, wins[idx], anom[idx], cls[idx], fused=True)
        steps += n
        np.testing.assert_allclose(np.array(lb), np.array(la), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(sb.protos, sa.protos, atol=1e-5)
        assert (sa.num_zero, sa.num_ones) == (sb.num_zero, sb.num_ones)
        assert abs(sa.factor - sb.factor) < 1e-12
    pa, pb = a.weights_numpy()["transformer"], b.weights_numpy()["transformer"]
    for k in pa:
        if k != "pos_encoder.pe":
            close_params(pb[k], pa[k], k, steps, rel=1e-4, abs_scale=2e-5, what="fused vs per-kernel " + k)
    assert [t["step"] for t in a.tensors] == [t["step"] for t in b.tensors]
    assert len(b._graphs) == 2


def test_fused_step_is_deterministic():
    """One workgroup, every sum in a fixed order: two identical backprop calls
    give bit-identical parameters, moments and state."""
    from preganplus_amd import train as TR
    w, extra = load16()
    z = np.load(f"{GOLD}/tune_h16.npz")
    out = []
    for _ in range(2):
        tr = TR.Trainer(16, w, extra)
        st = TR.TuneState(z["protos0"], float(z["factor0"]))
        TR.backprop(tr, st, z["windows"], z["anom"], z["cls"], fused=True)
        out.append((tr.P.cpu().numpy(), tr.m.cpu().numpy(), tr.v.cpu().numpy(), st.protos.copy()))
    for u, v in zip(*out):
        assert np.array_equal(u, v)


def test_fused_step_rejects_unsupported_hosts():
    from preganplus_amd import _native
    from preganplus_amd import train as TR
    tr = TR.Trainer(50, W.synth_weights(50, seed=1), max_batch=1)
    dev = tr.device
    state = TR.TuneState(np.full((50, 2), 0.5)).to_device(dev)
    z = torch.zeros((3, 150), device=dev)
    yi = torch.zeros(50, dtype=torch.int32, device=dev)
    loss = torch.zeros(2, dtype=torch.float64, device=dev)
    with pytest.raises(_native.NativeError):
        tr.tune_step1(z, yi, yi, state, loss)


def test_backprop_score_equals_separate_accuracy():
    """backprop(score=True) — accuracy()'s forward inside the tuning graph —
    gives the same losses, parameters and (AScore, CScore) as backprop followed
    by a separate accuracy() call."""
    from preganplus_amd import train as TR
    w, extra = load16()
    z = np.load(f"{GOLD}/tune_h16.npz")
    a, b = TR.Trainer(16, w, extra), TR.Trainer(16, w, extra)
    sa, sb = TR.TuneState(z["protos0"], float(z["factor0"])), TR.TuneState(z["protos0"], float(z["factor0"]))
    for _ in range(2):
        la = TR.backprop(a, sa, z["windows"], z["anom"], z["cls"])
        acc_a = TR.accuracy(a, sa, z["windows"], z["anom"], z["cls"])
        lb, acc_b = TR.backprop(b, sb, z["windows"], z["anom"], z["cls"], score=True)
        assert la == lb and acc_a == acc_b
        assert torch.equal(a.P, b.P)
        np.testing.assert_array_equal(sa.protos, sb.protos)
