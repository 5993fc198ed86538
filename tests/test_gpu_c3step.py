"""The C3 step's composition (train.OnlineTrainStep): detect's windows share
the tuning forward (pgp_tune_backward_prefix differentiates only the tuning
windows), AdamW's scalars come from device rows, and the step replays as a
captured HIP graph with the same results as eager issue."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H", [16, 50])
def test_prefix_backward_equals_backward_of_the_prefix(H):
    """Forward over B + E windows, backward over the first B == forward and
    backward over the B windows alone (the forward's decoder split-K grouping
    depends on the batch: fp32 rounding apart)."""
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    rng = np.random.default_rng(3)
    B, E = 24, 7
    w = W.synth_weights(H, seed=1)
    wins = torch.tensor(rng.uniform(0, 1, size=(B + E, 3, 3 * H)), dtype=torch.float32, device="cuda")
    y = torch.tensor(rng.integers(0, 2, size=(B, H)), dtype=torch.int32, device="cuda")
    mult = torch.tensor(rng.uniform(0.5, 2, size=(B, H)), dtype=torch.float32, device="cuda")
    tgt = torch.tensor(rng.uniform(0, 1, size=(B, H, 2)), dtype=torch.float32, device="cuda")
    a = TR.Trainer(H, w, device="cuda", max_batch=B + E)
    lg_a, _ = a.tune_forward(wins)
    a.tune_backward(B, y, mult, tgt)
    b = TR.Trainer(H, w, device="cuda", max_batch=B)
    lg_b, _ = b.tune_forward(wins[:B].contiguous())
    b.tune_backward(B, y, mult, tgt)
    torch.cuda.synchronize()
    np.testing.assert_allclose(lg_a[:B].cpu().numpy(), lg_b.cpu().numpy(), rtol=1e-5, atol=1e-6)
    ga = a.G[a.sec_off["transformer"]:a.sec_end["transformer"]].cpu().numpy()
    gb = b.G[b.sec_off["transformer"]:b.sec_end["transformer"]].cpu().numpy()
    np.testing.assert_allclose(ga, gb, rtol=1e-4, atol=1e-5 * np.abs(gb).max())
    with pytest.raises(ValueError):
        a.tune_backward(B + E + 1, y, mult, tgt)


def _online(H, E, seed=5, native=False):
    from preganplus_amd import simulate as SIM
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    import bench
    w = W.synth_weights(H, seed=0)
    tr = TR.Trainer(H, w, device="cuda", max_batch=11 * E)
    st = TR.TuneState(w["prototypes"])
    series, tmax = bench.synth_series(E, H, seed, 10)
    rng = np.random.default_rng(seed)
    s = np.zeros((E, H, H), dtype=np.float32)
    s[np.arange(E)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(E, H))] = 1.0
    envs = SIM.synth_envs(E, H, seed=seed)
    side = torch.cuda.Stream()
    step = TR.OnlineTrainStep(tr, st, SIM.Simulation(H, device="cuda"), series, tmax, s, envs, side=side,
                              native=native)
    return tr, step


@pytest.mark.parametrize("H", [16, 50])
def test_online_step_graph_replay_equals_eager(H):
    """Three steps issued eagerly == one eager step + two replays of the
    captured step: every weight, AdamW moment, the tuning state and the GAN
    label outcome are identical (same kernels, same order)."""
    main = torch.cuda.Stream()
    with torch.cuda.stream(main):
        tr_a, sa = _online(H, 6)
        for _ in range(3):
            sa.run()
        tr_b, sb = _online(H, 6)
        sb.run()
        sb.capture()
        for _ in range(2):
            sb.run()
        torch.cuda.synchronize()
    for x, y in ((tr_a.P, tr_b.P), (tr_a.m, tr_b.m), (tr_a.v, tr_b.v), (sa.tun.state, sb.tun.state),
                 (sa.target, sb.target), (sa.sim_out, sb.sim_out)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    assert sa.tun.n == sb.tun.n == 3
    for t_a, t_b in zip(tr_a.tensors, tr_b.tensors):
        assert t_a["step"] == t_b["step"], t_a["name"]
    # the GAN sections stepped three times, as adam_step would have counted
    assert {t["step"] for t in tr_a.tensors if t["section"] in ("gen", "disc") and t["trainable"]} == {3.0}


@pytest.mark.parametrize("H", [16, 50])
def test_native_step_equals_python_composition(H):
    """pgp_online_step (the whole step issued from C++, AdamW's scalars from
    the library's step counts) == the step composed from the per-op C-ABI
    calls in Python (AdamW's scalars from the host tables), three steps each:
    every weight, AdamW moment, the tuning state, the GAN labels and scores,
    the per-window losses and the step counts identical."""
    main = torch.cuda.Stream()
    with torch.cuda.stream(main):
        tr_a, sa = _online(H, 6, native=False)
        tr_b, sb = _online(H, 6, native=True)
        for _ in range(3):
            sa.run()
            sb.run()
        torch.cuda.synchronize()
    for x, y in ((tr_a.P, tr_b.P), (tr_a.m, tr_b.m), (tr_a.v, tr_b.v), (sa.tun.state, sb.tun.state),
                 (sa.target, sb.target), (sa.sim_out, sb.sim_out), (sa.tun.loss, sb.tun.loss),
                 (sa.tun.cond_steps, sb.tun.cond_steps), (sa.emb, sb.emb)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    sa.tun.sync(__import__("preganplus_amd.train", fromlist=["x"]).TuneState(np.zeros((H, 2))))
    sb.sync()
    for t_a, t_b in zip(tr_a.tensors, tr_b.tensors):
        assert t_a["step"] == t_b["step"], t_a["name"]
    assert {t["step"] for t in tr_b.tensors if t["section"] in ("gen", "disc") and t["trainable"]} == {3.0}


@pytest.mark.parametrize("H", [16, 50])
def test_native_step_issue_worker_equals_one_thread(H):
    """pgp_online_issue_worker: the GAN stream's launches issued from the
    library's second host thread (the default at world size 1) == one thread
    issuing both streams, over five back-to-back steps (the worker spinning
    between them) and a step after an idle pause (the worker asleep): every
    weight, moment, the tuning state, the GAN labels and the step counts."""
    import time
    main = torch.cuda.Stream()
    with torch.cuda.stream(main):
        tr_a, sa = _online(H, 6, native=True)
        tr_b, sb = _online(H, 6, native=True)
        sb.issue_worker(False)
        for s in (sa, sb):
            for _ in range(5):
                s.run()
            torch.cuda.synchronize()
            time.sleep(0.05)
            s.run()
        torch.cuda.synchronize()
    for x, y in ((tr_a.P, tr_b.P), (tr_a.m, tr_b.m), (tr_a.v, tr_b.v), (sa.tun.state, sb.tun.state),
                 (sa.target, sb.target), (sa.sim_out, sb.sim_out), (sa.tun.loss, sb.tun.loss), (sa.emb, sb.emb)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    sa.sync()
    sb.sync()
    for t_a, t_b in zip(tr_a.tensors, tr_b.tensors):
        assert t_a["step"] == t_b["step"], t_a["name"]
    assert {t["step"] for t in tr_a.tensors if t["section"] in ("gen", "disc") and t["trainable"]} == {6.0}


def test_native_sync_updates_tune_state_and_dptuner():
    """after native steps, sync() writes the tuning state into the
    TuneState the step was built with and re-anchors the DPTuner's host step
    bookkeeping, so a following tun.sync(st) keeps the native counts (it used
    to reset them to base + 0) and the Python composition continues from them."""
    from preganplus_amd import train as TR
    main = torch.cuda.Stream()
    with torch.cuda.stream(main):
        tr, sb = _online(16, 4, native=True)
        for _ in range(3):
            sb.run()
        torch.cuda.synchronize()
        sb.sync()
    dev = TR.TuneState(np.zeros_like(sb.st.protos))
    dev.from_device(sb.tun.state)
    np.testing.assert_array_equal(sb.st.protos, dev.protos)
    assert sb.st.factor < TR.PROTO_UPDATE_FACTOR   # decayed on the device, now on the host
    steps = {t["name"] + t["section"]: t["step"] for t in tr.tensors}
    assert {t["step"] for t in sb.tun.sel if t["name"] not in TR.DPTuner.COND} == {3.0}
    sb.tun.sync(sb.st)
    assert {t["name"] + t["section"]: t["step"] for t in tr.tensors} == steps


def test_native_step_stage_timing():
    """pgp_online_timing / pgp_online_stage_ms: every span is non-negative and
    the main stream's span covers its stages."""
    from preganplus_amd import train as TR
    main = torch.cuda.Stream()
    with torch.cuda.stream(main):
        _, sb = _online(16, 4, native=True)
        sb.run()
        sb.timing(True)
        sb.run()
        ms = sb.stage_ms()
        sb.timing(False)
    assert set(ms) == set(TR.ONLINE_STAGES)
    assert all(v >= 0 for v in ms.values())
    assert ms["main"] + 1e-3 >= ms["dataset"] + ms["tune_model"] - 1e-2
    with pytest.raises(RuntimeError):
        sb.issue()


def test_section_rows_match_adam_step():
    """SectionRows' device rows drive AdamW to the same weights as adam_step."""
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    w = W.synth_weights(16, seed=2)
    a = TR.Trainer(16, w, device="cuda", max_batch=1)
    b = TR.Trainer(16, w, device="cuda", max_batch=1)
    g = torch.randn_like(a.G)
    rows = TR.SectionRows(b, "gen")
    row = rows.buffer()
    sel = [t for t in b.tensors if t["section"] == "gen" and t["trainable"]]
    for _ in range(3):
        a.G.copy_(g)
        b.G.copy_(g)
        a.adam_step("gen")
        rows.next_row(row)
        b.adam_step_table("gen", sel, row)
    torch.cuda.synchronize()
    np.testing.assert_allclose(a.P.cpu().numpy(), b.P.cpu().numpy(), rtol=1e-6, atol=1e-7)
    assert [t["step"] for t in a.tensors] == [t["step"] for t in b.tensors]
