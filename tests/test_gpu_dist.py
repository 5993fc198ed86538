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
