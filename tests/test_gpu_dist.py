"""The product's data-parallel training step with two ranks on the one GPU of
the box (gloo process group: RCCL refuses two ranks on one device; the driver's
multi-GPU runs use RCCL with one rank per GPU).

Each rank runs train.dp_tune_step (device bookkeeping, gradient and state
all-reduces, the default group) and train.train_gan_batched(all_reduce=True)
with its all-reduces on the GAN's own group (train.dp_groups) on its half of the
windows / environments; the result must equal one process on the
concatenated batch (SURVEY §8e parity rule): gradients and parameters to fp32
reduction tolerance, prototypes / counters / factor to fp64 rounding."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, B, E = 16, 64, 24


def _inputs():
    rng = np.random.Generator(np.random.PCG64(77))
    x = rng.uniform(0, 0.8, size=(B, 3, 3 * H)).astype(np.float32)
    y = (rng.uniform(size=(B, H)) < 0.3).astype(np.int32)
    c = rng.integers(0, 3, size=(B, H)).astype(np.int32)
    emb = np.where(rng.uniform(size=(E, H, 1)) < 0.4, rng.uniform(size=(E, H, 2)), 0.0).astype(np.float32)
    s = np.zeros((E, H, H), np.float32)
    s[np.arange(E)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(E, H))] = 1.0
    return x, y, c, emb, s


def _state0():
    from preganplus_amd import train as TR
    st = TR.TuneState(np.array([[0.2, 0.3], [0.6, 0.1], [0.5, 0.9]] + [[0.5, 0.5]] * (H - 3)))
    st.num_zero, st.num_ones = 40, 9
    return st


def _run(sl_w, sl_e, group_init=None):
    """One DP tuning step + one batched GAN step on the given slices."""
    from preganplus_amd import simulate as SIM
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    w = W.synth_weights(H, seed=12)
    x, y, c, emb, s = _inputs()
    tr = TR.Trainer(H, w, max_batch=B)
    st = _state0()
    tune_group, gan_group = TR.dp_groups()   # the bench's two-communicator design
    TR.dp_tune_step(tr, st, x[sl_w], y[sl_w], c[sl_w], group=tune_group)
    envs = SIM.synth_envs(E, H, seed=3)[sl_e]
    sim = SIM.Simulation(H, device=tr.device)
    out, target = TR.train_gan_batched(tr, sim, envs, emb[sl_e], s[sl_e], all_reduce=True, group=gan_group)
    torch.cuda.synchronize()
    return (tr.G.cpu().numpy(), tr.P.cpu().numpy(), st.protos.copy(), st.num_zero, st.num_ones, st.factor,
            target.cpu().numpy())


def _rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        res = _run(slice(rank * B // world, (rank + 1) * B // world), slice(rank * E // world, (rank + 1) * E // world))
        gathered = [None] * world
        dist.all_gather_object(gathered, res[-1])
        if rank == 0:
            q.put(res[:-1] + (np.concatenate(gathered),))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_dp_steps_equal_full_batch():
    import torch.multiprocessing as mp
    from preganplus_amd import train as TR
    from tests.test_gpu_train import close
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        G2, P2, pr2, nz2, no2, f2, tg2 = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    G1, P1, pr1, nz1, no1, f1, tg1 = _run(slice(0, B), slice(0, E))
    np.testing.assert_array_equal(tg2, tg1)        # per-environment simulated GAN labels
    tr = TR.Trainer(H, __import__("preganplus_amd.weights", fromlist=["x"]).synth_weights(H, 12))
    for t in tr.tensors:
        if not t["trainable"]:
            continue
        sl = slice(t["offset"], t["offset"] + t["n"])
        close(G2[sl], G1[sl], rel=1e-4, abs_scale=1e-5, what="grad " + t["name"])
        # fresh AdamW's first step is ~lr * sign(g): entries with noise-level
        # gradients may move differently by up to 2 lr
        lr = tr.lrs[t["section"]]
        g = np.abs(G1[sl])
        noise = g <= 1e-4 * g.max()
        close(P2[sl][~noise], P1[sl][~noise], rel=1e-5, abs_scale=1e-6, what="param " + t["name"])
        assert np.all(np.abs(P2[sl][noise] - P1[sl][noise]) <= 2 * lr)
    np.testing.assert_allclose(pr2, pr1, rtol=1e-13, atol=1e-15)
    assert (nz2, no2) == (nz1, no1) and abs(f2 - f1) <= 1e-15


# ---------------------------------------------------------------------------
# The C3 step itself at world size 2: OnlineTrainStep (native: pgp_online_step
# with the collectives called back into torch.distributed), two streams per
# rank, the GAN stream shared as the tuning backward's side stream
# (pgp_tune_set_side_stream, as bench.py does at world > 1) and the two
# process groups (train.dp_groups).  H = 50 with 48 environments per rank: 72 k
# tokens, above the side stream's threshold, so the backward's side work
# really runs on the shared stream.  One step on each half == one process on
# the concatenated batch.
# ---------------------------------------------------------------------------
HS, ES = 50, 96


def _c3_inputs():
    import bench
    from preganplus_amd import simulate as SIM
    series, tmax = bench.synth_series(ES, HS, 21, 10)
    rng = np.random.default_rng(21)
    s = np.zeros((ES, HS, HS), np.float32)
    s[np.arange(ES)[:, None], np.arange(HS)[None, :], rng.integers(0, HS, size=(ES, HS))] = 1.0
    return series, tmax, s, SIM.synth_envs(ES, HS, seed=21)


def _c3_run(sl, world):
    from preganplus_amd import _native
    from preganplus_amd import simulate as SIM
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    import ctypes
    series, tmax, s, envs = _c3_inputs()
    w = W.synth_weights(HS, seed=4)
    E = len(range(ES)[sl])
    main = torch.cuda.Stream()
    side = torch.cuda.Stream()
    L = _native.lib()
    L.pgp_tune_set_side_stream.argtypes = [ctypes.c_void_p]
    if world > 1:
        _native.check(L.pgp_tune_set_side_stream(ctypes.c_void_p(side.cuda_stream)), "pgp_tune_set_side_stream")
    try:
        with torch.cuda.stream(main):
            tr = TR.Trainer(HS, w, max_batch=11 * E)
            st = TR.TuneState(w["prototypes"])
            step = TR.OnlineTrainStep(tr, st, SIM.Simulation(HS, device=tr.device), series[sl], tmax, s[sl], envs[sl],
                                      side=side, groups=TR.dp_groups())
            step.run()
            torch.cuda.synchronize()
            step.sync()
            # the tuning loss's per-(window, host) weights and targets (tune_targets_dp_kernel)
            lt = torch.cat([step.tun.mult[:step.B, :, None], step.tun.tgt[:step.B]], dim=2).cpu().numpy()
            return (tr.P.cpu().numpy(), step.tun.state.cpu().numpy(), step.target.cpu().numpy(),
                    step.sim_out.cpu().numpy(), [t["step"] for t in tr.tensors], tr.G.cpu().numpy(), lt)
    finally:
        L.pgp_tune_set_side_stream(None)


def _c3_rank(rank, world, port, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        per = ES // world
        P, state, target, sim_out, steps, G, lt = _c3_run(slice(rank * per, (rank + 1) * per), world)
        got = [None] * world
        dist.all_gather_object(got, (target, sim_out, lt))
        if rank == 0:
            q.put((P, state, np.concatenate([g[0] for g in got]), np.concatenate([g[1] for g in got]), steps, G,
                   np.concatenate([g[2] for g in got])))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_online_step_two_ranks_equal_full_batch():
    import torch.multiprocessing as mp
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    from tests.test_gpu_train import key_bias_mask
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + os.getpid() % 1000
    procs = [ctx.Process(target=_c3_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        P2, st2, tg2, so2, steps2, G2, lt2 = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    P1, st1, tg1, so1, steps1, G1, lt1 = _c3_run(slice(0, ES), 1)
    # the tuning loss's weights and targets: decisions on the forward's outputs,
    # whose fp32 rounding depends on the batch (decoder split-K grouping), so a
    # decision within rounding of a tie could flip between the two partitions
    # and move the gradients by a whole window's share; this dataset has none
    # (asserted first, so such a flip reads as what it is)
    flip = np.argwhere(np.any(lt1 != lt2, axis=2))
    assert flip.size == 0, ("tuning-target decisions differ at (row, host)", flip[:8].tolist(), lt1[tuple(flip[0])],
                            lt2[tuple(flip[0])])
    # the GAN labels and scores of every environment: the step-start GAN, per environment
    np.testing.assert_array_equal(tg2, tg1)
    np.testing.assert_array_equal(so2, so1)
    assert steps2 == steps1
    K = (st1.size - 3) // 2
    # prototypes: the deltas f (a - P) come from the forward's prototype outputs a, whose
    # decoder split-K grouping depends on the batch (fp32 rounding apart, as the gradients)
    np.testing.assert_allclose(st2[:2 * K], st1[:2 * K], rtol=1e-7, atol=1e-9)
    assert st2[2 * K + 1] == st1[2 * K + 1] and st2[2 * K + 2] == st1[2 * K + 2]      # num_zero, num_ones
    assert abs(st2[2 * K] - st1[2 * K]) <= 1e-15                                       # factor
    tr = TR.Trainer(HS, W.synth_weights(HS, seed=4))
    P0 = tr.P.cpu().numpy()
    eps, u = tr.eps, 2.0 ** -24
    for t in tr.tensors:
        if not t["trainable"]:
            continue
        sl = slice(t["offset"], t["offset"] + t["n"])
        lr = tr.lrs[t["section"]]
        # one AdamW step from zero moments (torch AdamW, step 1: m-hat = g, v-hat = g^2)
        # moves an entry by -lr wd p - lr g / (|g| + eps).  The decay term is the same
        # on both sides, so the two runs' parameters must differ by exactly what their
        # gradients (equal up to fp32 summation grouping) predict, every entry:
        #   P2 - P1 = -lr (f(g2) - f(g1)),  f(g) = g / (|g| + eps)
        # up to the fp32 rounding of the two updates: each side's AdamW evaluation
        # (m-hat, v-hat, sqrt, the division, the update) is within 8 ulps of |p| + lr
        # of the exact formula on ITS gradient, and the two errors are independent
        # where the gradients' bits differ, so their difference is within 16.
        if np.array_equal(P1[sl], P0[sl]):   # a tensor the step left alone (the prototype decoder's gate)
            assert np.array_equal(P2[sl], P0[sl]), t["name"]
            continue
        g1 = G1[sl].astype(np.float64)
        g2 = G2[sl].astype(np.float64)
        f = lambda g: g / (np.abs(g) + eps)
        pred = -lr * (f(g2) - f(g1))
        d = P2[sl].astype(np.float64) - P1[sl].astype(np.float64)
        # The attention key biases' gradient is identically zero in exact
        # arithmetic (key_bias_mask): both runs hold rounding noise there, which
        # AdamW's g / (|g| + eps) turns into O(lr) steps where the formula's own
        # rounding is not negligible against the noise; those entries are held
        # to the step bound |d| <= 2 lr (each side moves by at most lr + lr wd |p|)
        noise = key_bias_mask(t["name"], t["n"], HS)
        tol = 16 * u * (np.abs(P1[sl]).astype(np.float64) + lr)
        bad = (np.abs(d - pred) > tol) & ~noise
        assert not bad.any(), (t["name"], int(bad.sum()), float((np.abs(d - pred) / tol)[~noise].max()))
        assert np.all(np.abs(d[noise]) <= 2 * lr * (1 + 1e-6)), t["name"] + " (key bias)"
        # and the gradients themselves agree to fp32 grouping where they are not
        # rounding noise (exact zeros on both sides: key biases)
        scale = np.abs(g1).max() + 1e-30
        np.testing.assert_allclose(g2[~noise], g1[~noise], rtol=1e-3, atol=1e-5 * scale, err_msg=t["name"])
