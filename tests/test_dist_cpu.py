"""Multi-process (gloo, world_size 2, CPU) checks of the data-parallel paths.

* Tuning: each rank computes the gradients of its shard of
  windows; Trainer.all_reduce_grads (the product's call: one flat all-reduce,
  RCCL on the GPU box, gloo here) over a Trainer whose buffer holds them
  equals the gradient of the concatenated batch.  Gradients come from the
  torch training oracle (no GPU here); tests/test_gpu_dist.py runs the whole
  product step (train.dp_tune_step) with two ranks on the GPU.
* Inference sharding: bench.py gives every rank its own independent windows;
  the per-rank seeds differ and no collective touches the data path.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pregan_train_oracle as TO
from preganplus_amd import weights as W

H, B = 8, 4


def _batch_grads(w, x, y, mult, tgt):
    tw = TO.leaf_params(w["transformer"])
    logits, protos = TO.decode_t(tw, TO.encode_t(tw, torch.tensor(x)))
    ce = torch.nn.functional.cross_entropy(logits.reshape(-1, 2), torch.tensor(y.reshape(-1), dtype=torch.long),
                                           reduction="none").reshape(x.shape[0], H)
    loss = (ce * torch.tensor(mult)).sum() + (((protos - torch.tensor(tgt)) ** 2).mean(-1)
                                              * torch.tensor(y > 0)).sum()
    loss.backward()
    return torch.cat([tw[k].grad.reshape(-1) for k in tw if tw[k].grad is not None])


def _inputs():
    rng = np.random.Generator(np.random.PCG64(3))
    x = rng.uniform(0, 0.8, size=(B, 3, 3 * H))
    y = (rng.uniform(size=(B, H)) < 0.4).astype(np.int64)
    mult = rng.uniform(0.5, 2, size=(B, H))
    tgt = rng.uniform(0, 1, size=(B, H, 2))
    return x, y, mult, tgt


def _stub_trainer(g):
    """A Trainer whose gradient buffer is `g` (the oracle's gradients; no GPU
    here), with a gen section after the transformer one that must stay local."""
    from preganplus_amd import train as TR
    tr = TR.Trainer.__new__(TR.Trainer)
    n = g.numel()
    tr.G = torch.cat([g, torch.full((5,), 7.0, dtype=g.dtype)])
    tr.sec_off, tr.sec_end = {"transformer": 0, "gen": n}, {"transformer": n, "gen": n + 5}
    return tr


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = W.synth_weights(H, seed=1)
    x, y, mult, tgt = _inputs()
    sl = slice(rank * B // world, (rank + 1) * B // world)
    g = _batch_grads(w, x[sl], y[sl], mult[sl], tgt[sl])
    tr = _stub_trainer(g)
    tr.all_reduce_grads("transformer")  # the product's call: one flat SUM all-reduce
    if rank == 0:
        q.put(tr.G.numpy())
    dist.destroy_process_group()


def test_dp_gradient_allreduce_equals_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    g_dp = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    w = W.synth_weights(H, seed=1)
    g_full = _batch_grads(w, *_inputs()).numpy()
    np.testing.assert_allclose(g_dp[:-5], g_full, rtol=1e-10, atol=1e-12)
    assert np.all(g_dp[-5:] == 7.0)  # only the named section is reduced


def test_trainer_allreduce_is_noop_without_process_group():
    """Single process: all_reduce_grads must not require torch.distributed."""
    from preganplus_amd import train as TR
    tr = TR.Trainer.__new__(TR.Trainer)
    tr.G = torch.arange(10, dtype=torch.float32)
    tr.sec_off, tr.sec_end = {"transformer": 0}, {"transformer": 10}
    tr.all_reduce_grads("transformer")
    assert tr.G.tolist() == list(range(10))


# ---- DP tuning host state (prototype EMA deltas, counters) ----
def _state_inputs(Bt=6, Hh=5):
    rng = np.random.Generator(np.random.PCG64(11))
    logits = rng.normal(size=(Bt, Hh, 2))
    protos = rng.uniform(size=(Bt, Hh, 2))
    y = (rng.uniform(size=(Bt, Hh)) < 0.5).astype(np.int64)
    c = rng.integers(0, 3, size=(Bt, Hh))
    return logits, protos, y, c


def _state_worker(rank, world, port, q):
    from preganplus_amd import train as TR
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lg, pr, y, c = _state_inputs()
    n = lg.shape[0]
    sl = slice(rank * n // world, (rank + 1) * n // world)
    st = TR.TuneState(np.array([[0.2, 0.3], [0.6, 0.1], [0.5, 0.9]]))
    st.num_zero, st.num_ones = 7, 3
    mult, tgt, _, _, inc = TR.loss_targets_dp(lg[sl], pr[sl], y[sl], c[sl], st)
    TR.dp_state_update(st, inc)
    if rank == 0:
        q.put((st.protos.copy(), st.num_zero, st.num_ones, st.factor, mult, tgt))
    dist.destroy_process_group()


def test_dp_tuning_state_equals_full_batch():
    """Prototype EMA / counters / factor after a 2-rank DP step == the same
    update computed on the concatenated batch in one process."""
    from preganplus_amd import train as TR
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_state_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    protos, nz, no, fac, mult0, tgt0 = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    lg, pr, y, c = _state_inputs()
    st = TR.TuneState(np.array([[0.2, 0.3], [0.6, 0.1], [0.5, 0.9]]))
    st.num_zero, st.num_ones = 7, 3
    mult, tgt, _, _, inc = TR.loss_targets_dp(lg, pr, y, c, st)
    TR.dp_state_update(st, inc)
    np.testing.assert_allclose(protos, st.protos, rtol=1e-13, atol=1e-15)
    assert (nz, no) == (st.num_zero, st.num_ones) and fac == pytest.approx(st.factor, rel=1e-15)
    np.testing.assert_array_equal(mult0, mult[:3])
    np.testing.assert_array_equal(tgt0, tgt[:3])


def test_dp_state_single_window_is_reference_update():
    """One window with one positive host on one rank: loss_targets_dp +
    dp_state_update == the reference-order loss_targets (train.py:27-40)
    exactly (with several positives the reference compounds within the window;
    the DP form scores them all against the step-start state)."""
    from preganplus_amd import train as TR
    lg, pr, y, c = _state_inputs(Bt=1, Hh=3)
    base = np.array([[0.2, 0.3], [0.6, 0.1], [0.5, 0.9]])
    y[0] = [0, 1, 0]
    c[0] = [0, 1, 2]
    pr[0, 1] = base[1] + [0.01, -0.02]  # closest to its own class: the EMA update fires
    st1, st2 = TR.TuneState(base.copy()), TR.TuneState(base.copy())
    m1, t1, a1, l1 = TR.loss_targets(lg[0], pr[0], y[0], c[0], st1)
    m2, t2, a2, l2, inc = TR.loss_targets_dp(lg, pr, y, c, st2)
    TR.dp_state_update(st2, inc)
    np.testing.assert_allclose(st2.protos, st1.protos, rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(m2[0], m1)
    np.testing.assert_allclose(t2[0], t1)
    assert not np.array_equal(st2.protos, base)
    assert a2[0] == pytest.approx(a1, rel=1e-14) and l2[0] == pytest.approx(l1, rel=1e-14, abs=1e-15)
    assert st2.factor == pytest.approx(st1.factor) and (st2.num_zero, st2.num_ones) == (st1.num_zero, st1.num_ones)


# ---- the C3 step's two communicators (tuning, GAN) ----
class _FakeGanTrainer:
    """Records the groups train_gan_batched hands to all_reduce_grads."""

    def __init__(self):
        self.calls = []
        self._gan_in = (None, None)

    def gan_forward(self, emb, sched):
        return torch.zeros((2, 1)), None

    def gan_disc_backward(self, target):
        pass

    def gan_gen_backward(self, B):
        pass

    def adam_step(self, section):
        pass

    def all_reduce_grads(self, section, group=None):
        self.calls.append((section, group))


class _FakeSim:
    def score(self, envs, ns, orig, out=None, target=None):
        return out, target


def _groups_worker(rank, world, port, q):
    from preganplus_amd import train as TR
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tune_g, gan_g = TR.dp_groups()
    # the GAN group is a communicator of its own over every rank
    own = gan_g is not None and gan_g is not dist.group.WORLD
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, group=gan_g)
    ranks = dist.get_process_group_ranks(gan_g)
    # train_gan_batched sends both of its all-reduces to that group
    fake = _FakeGanTrainer()
    TR.train_gan_batched(fake, _FakeSim(), None, None, None, all_reduce=True, group=gan_g)
    q.put((rank, own, tune_g is None, float(t.item()), ranks,
           [(s, g is gan_g) for s, g in fake.calls]))
    dist.destroy_process_group()


def test_gan_collectives_use_their_own_group():
    """at world size > 1 the C3 step's GAN
    all-reduces go to a second process group (communicator), so they do not
    queue behind the tuning step's gradient all-reduce on one communicator's
    stream; the tuning step keeps the default group."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_groups_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, own, tune_default, tsum, ranks, calls in res:
        assert own and tune_default
        assert tsum == 3.0 and ranks == [0, 1]
        assert calls == [("disc", True), ("gen", True)]


def test_dp_groups_single_process():
    from preganplus_amd import train as TR
    assert TR.dp_groups() == (None, None)
