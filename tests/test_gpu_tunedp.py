"""GPU parity of the device-resident data-parallel tuning bookkeeping
(pgp_tunedp.hip through the C-ABI) against the host restatements that the CPU
tests pin to the reference: form_test_dataset / convert_to_windows /
normalize_test_time_data (utils.py:7-24, 94-95), train.loss_targets_dp and
train.dp_state_update (train.py:13-40 in the DP form of SURVEY §8e)."""
import math

import numpy as np
import pytest
import torch

from oracle import pregan_oracle as O
from preganplus_amd import weights as W

pytestmark = pytest.mark.gpu


def _series(rng, E, R, H, ties=True):
    scale = rng.uniform(10, 100, size=3 * H)
    s = rng.uniform(0.05, 0.6, size=(E, R, 3 * H)) * scale
    spike = rng.uniform(size=s.shape) < 0.05
    s = np.where(spike, rng.uniform(0.8, 1.0, size=s.shape) * scale, s)
    if ties:
        s[0] = s[0, :1]                               # constant rows: every percentile == the value
        if R >= 2:
            s[1, -1] = s[1, -2]                       # the two largest rows equal in every column
        s[2, :, ::3] = np.round(s[2, :, ::3] / 10) * 10  # many exact ties
    train = rng.uniform(0.1, 1.0, size=(40, 3 * H)) * scale
    return s, train


@pytest.mark.parametrize("H,E,R", [(16, 37, 10), (50, 9, 10), (8, 5, 3), (16, 4, 16), (16, 6, 1), (50, 6, 2)])
def test_tune_dataset_bit_exact(H, E, R):
    from preganplus_amd import train as TR
    rng = np.random.default_rng(H * 100 + R)
    series, train = _series(rng, E, R, H)
    tr = TR.Trainer(H, W.synth_weights(H, 1), max_batch=4)
    wins, y, cls, inf = TR.tune_dataset(tr, series, train.max(axis=0))
    wins, y, cls, inf = (a.cpu().numpy() for a in (wins, y, cls, inf))
    for e in range(E):
        td = TR.normalize_test_time_data(series[e], train)          # utils.py:94-95
        an, wh = TR.form_test_dataset(td)                            # utils.py:16-24
        np.testing.assert_array_equal(y[e * R:(e + 1) * R], an)
        np.testing.assert_array_equal(cls[e * R:(e + 1) * R], wh)
        np.testing.assert_array_equal(wins[e * R:(e + 1) * R], TR.convert_to_windows(td).astype(np.float32))
        np.testing.assert_array_equal(inf[e], O.inference_window(series[e], train).astype(np.float32))
    assert (y == 0).any() and (y.sum() > 0 or R < 3)   # one or two rows: nothing exceeds its own percentile


def _host_state(P, factor, nz, no):
    from preganplus_amd import train as TR
    st = TR.TuneState(P.copy(), factor)
    st.num_zero, st.num_ones = nz, no
    return st


@pytest.mark.parametrize("H,B", [(16, 300), (50, 1030), (8, 1)])
def test_tune_targets_dp_matches_host(H, B):
    """pgp_tune_targets_dp vs train.loss_targets_dp on random forward outputs:
    mult / tgt bit-identical, per-window losses and the increments to fp64
    rounding (the batch sum is tree-ordered), counts exact."""
    from preganplus_amd import train as TR
    rng = np.random.default_rng(B + H)
    tr = TR.Trainer(H, W.synth_weights(H, 2), max_batch=B)
    P = rng.uniform(0.1, 0.9, (H, 2))
    st = _host_state(P, 0.2, 311.0, 29.0)
    y = (rng.random((B, H)) < 0.35).astype(np.int32)
    c = rng.integers(0, 3, (B, H)).astype(np.int32)
    lg = rng.normal(0, 2, (B, H, 2)).astype(np.float32)
    pr = np.clip(P[c] + rng.normal(0, 0.15, (B, H, 2)), 0, 1).astype(np.float32)
    m_h, t_h, a_h, l_h, inc_h = TR.loss_targets_dp(lg, pr, y, c, st)
    tun = TR.DPTuner(tr, st, B)
    dev = tr.device
    tr.logits[:B].copy_(torch.from_numpy(lg))
    tr.protos[:B].copy_(torch.from_numpy(pr))
    L = tr._L
    from preganplus_amd import _native
    yd, cd = torch.from_numpy(y).to(dev), torch.from_numpy(c).to(dev)   # kept alive for the launch
    _native.check(L.pgp_tune_targets_dp(H, H, B, tr.logits.data_ptr(), tr.protos.data_ptr(),
                                        yd.data_ptr(), cd.data_ptr(),
                                        tun.state.data_ptr(), TR.PROTO_UPDATE_MIN, tun.mult.data_ptr(),
                                        tun.tgt.data_ptr(), tun.loss.data_ptr(), tun.inc.data_ptr(),
                                        tun.ws.data_ptr(), tr._stream()), "pgp_tune_targets_dp")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tun.mult[:B].cpu().numpy(), m_h.astype(np.float32))
    np.testing.assert_array_equal(tun.tgt[:B].cpu().numpy(), t_h.astype(np.float32))
    np.testing.assert_allclose(tun.loss[:B].cpu().numpy(), np.stack([a_h, l_h], 1), rtol=1e-12, atol=1e-12)
    inc = tun.inc.cpu().numpy()
    K = H
    np.testing.assert_allclose(inc[:2 * K], inc_h.delta.reshape(-1), rtol=1e-12, atol=1e-14)
    np.testing.assert_array_equal(inc[2 * K:3 * K], inc_h.count)
    assert (inc[3 * K], inc[3 * K + 1], inc[3 * K + 2]) == (inc_h.num_zero, inc_h.num_ones, inc_h.windows)
    assert inc_h.count.sum() > 0


@pytest.mark.parametrize("positives", [True, False])
def test_state_apply_matches_host(positives):
    """pgp_tune_state_apply vs train.dp_state_update, and the prototype
    decoder's AdamW rows vs the host formula (inactive without a positive
    label: torch skips a parameter with no gradient, its step count stays)."""
    from preganplus_amd import _native
    from preganplus_amd import train as TR
    H, B = 16, 64
    rng = np.random.default_rng(5 if positives else 6)
    tr = TR.Trainer(H, W.synth_weights(H, 2), max_batch=B)
    P = rng.uniform(0.1, 0.9, (H, 2))
    st = _host_state(P, 0.2, 11.0, 3.0)
    tun = TR.DPTuner(tr, st, B)
    inc = TR.TuneIncrements(H)
    inc.delta[:3] = rng.normal(0, 0.1, (3, 2))
    inc.count[:3] = [3, 0, 7]
    inc.num_zero, inc.num_ones, inc.windows = B * H, (37.0 if positives else 0.0), float(B)
    tun.inc.copy_(torch.from_numpy(inc.flat()))
    steps0 = tun.cond_steps.cpu().numpy().copy()
    tun._fill_table()
    row = tun.table[0]
    _native.check(tr._L.pgp_tune_state_apply(
        H, tun.state.data_ptr(), tun.inc.data_ptr(), TR.PROTO_FACTOR_DECAY, len(tun.cond), tun.cond_rows,
        tun.cond_steps.data_ptr(), row.data_ptr(), tr.lrs["transformer"], tr.b1, tr.b2, tr._stream()),
        "pgp_tune_state_apply")
    TR.dp_state_update(st, inc)
    dev = TR.TuneState(P.copy())
    dev.from_device(tun.state)
    np.testing.assert_array_equal(dev.protos, st.protos)
    assert (dev.num_zero, dev.num_ones) == (st.num_zero, st.num_ones)
    assert abs(dev.factor - st.factor) <= 1e-15 * st.factor
    steps = tun.cond_steps.cpu().numpy()
    r = row.cpu().numpy()
    lr = tr.lrs["transformer"]
    for i, k in enumerate(tun.cond):
        want_step = steps0[i] + (1 if positives else 0)
        assert steps[i] == want_step
        s = max(want_step, 1.0)
        want = np.array([1.0 if positives else 0.0, lr / (1 - tr.b1 ** s), math.sqrt(1 - tr.b2 ** s)], np.float32)
        np.testing.assert_array_equal(r[k], want)


def test_dp_tuner_steps_equal_host_pieces():
    """Three DPTuner steps == the same steps with host bookkeeping
    (loss_targets_dp + dp_state_update + adam_step): parameters and moments to
    fp32 equality, state to fp64 rounding, including a step without positive
    labels (prototype decoder skipped by AdamW)."""
    from preganplus_amd import train as TR
    H, B = 16, 40
    w = W.synth_weights(H, seed=6)
    rng = np.random.default_rng(9)
    P0 = np.array([[0.2, 0.3], [0.6, 0.1], [0.5, 0.9]] + [[0.5, 0.5]] * (H - 3))
    a, b = TR.Trainer(H, w, max_batch=B), TR.Trainer(H, w, max_batch=B)
    sa, sb = TR.TuneState(P0.copy()), TR.TuneState(P0.copy())
    tun = TR.DPTuner(b, sb, B)
    for it in range(3):
        wins = rng.uniform(0, 0.8, size=(B, 3, 3 * H)).astype(np.float32)
        y = (rng.uniform(size=(B, H)) < 0.3).astype(np.int32) * (0 if it == 1 else 1)
        c = rng.integers(0, 3, size=(B, H)).astype(np.int32)
        lg, pr = a.tune_forward(torch.tensor(wins))
        mult, tgt, al, tl, inc = TR.loss_targets_dp(lg.cpu().numpy(), pr.cpu().numpy(), y, c, sa)
        a.tune_backward(B, y, mult, tgt)
        tot = TR.dp_state_update(sa, inc)
        a.adam_step("transformer", () if tot.num_ones > 0 else TR.DPTuner.COND)
        loss = tun.step(torch.tensor(wins, device=b.device), torch.tensor(y, device=b.device),
                        torch.tensor(c, device=b.device)).cpu().numpy()
        np.testing.assert_allclose(loss, np.stack([al, tl], 1), rtol=1e-12, atol=1e-12)
        torch.cuda.synchronize()
        assert torch.equal(a.P, b.P) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v), it
    tun.sync(sb)
    np.testing.assert_allclose(sb.protos, sa.protos, rtol=1e-13, atol=1e-15)
    assert (sb.num_zero, sb.num_ones) == (sa.num_zero, sa.num_ones)
    assert abs(sb.factor - sa.factor) <= 1e-15
    assert [t["step"] for t in a.tensors] == [t["step"] for t in b.tensors]
