"""GPU parity of the GAN-label simulation (csrc/pgp_sim.hip through the C-ABI,
SURVEY §8f row f4) against the reference's own runSimulation outputs
(tests/golden/sim_h*.npz, tests/golden/make_golden_sim.py) and the oracle
(oracle/sim_oracle.py): integer/fp64 bookkeeping, so bit-exact."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import sim_oracle as SO
from preganplus_amd import simulate as SIM

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H", [16, 50])
def test_simulate_matches_reference_fixtures(H):
    z = np.load(f"tests/golden/sim_h{H}.npz")
    out, target = SIM.Simulation(H).score(z["envs"], z["new"], z["orig"])
    out, target = out.cpu().numpy(), target.cpu().numpy()
    assert np.array_equal(out, z["ref"]), np.abs(out - z["ref"]).max()
    assert np.array_equal(target, z["target"])


def _sched(rng, E, H):
    s = rng.uniform(size=(E, H, H)).astype(np.float32)
    tie = rng.uniform(size=(E, H)) < 0.15
    s[tie] = np.float32(0.25)  # fully tied rows: first column
    e, r = np.nonzero(rng.uniform(size=(E, H)) < 0.15)
    s[e, r, rng.integers(0, H, len(e))] = s[e, r].max(axis=1)  # ties at the max
    return s


@pytest.mark.parametrize("H", [2, 8, 16, 50, 64])
def test_simulate_matches_oracle_synthetic(H):
    rng = np.random.Generator(np.random.PCG64(300 + H))
    E = 300
    envs = SIM.synth_envs(E, H, seed=H)
    new, orig = _sched(rng, E, H), _sched(rng, E, H)
    orig[::5] = new[::5]  # equal schedules: label [0, 1]
    out, target = SIM.Simulation(H).score(envs, new, orig)
    ref, rt = SO.simulate_batch(envs, new, orig, H)
    assert np.array_equal(out.cpu().numpy(), ref)
    assert np.array_equal(target.cpu().numpy(), rt)
    assert rt[:, 0].sum() > 0 and rt[:, 1].sum() > 0


def test_simulate_python_power_semantics():
    """Negative host IPS (apparent IPS of an overcommitted host can be < 0):
    PM.powerFromCPU indexes the power list from the end, as Python does; past
    the table the reference raises IndexError and the kernel reports NaN."""
    H = 8
    envs = SIM.synth_envs(3, H, seed=5)
    o = SIM.offsets(H)
    hs, ap = o["host"][0], o["app_ips"][0]
    for i, val in ((0, -300.0), (1, -4000.0), (2, -1e6)):
        envs[i, hs:hs + H] = -1
        envs[i, hs] = 0  # container 0 alone on host 0, stays there
        envs[i, ap] = val
    new = np.zeros((3, H, H), np.float32)
    new[:, :, 0] = 1.0
    out, _ = SIM.Simulation(H).score(envs, new, new)
    out = out.cpu().numpy()
    for i in (0, 1):
        ref, _ = SO.simulate_batch(envs[i:i + 1], new[i:i + 1], new[i:i + 1], H)
        assert np.array_equal(out[i], ref[0])
    with pytest.raises(IndexError):
        SO.simulate_batch(envs[2:3], new[2:3], new[2:3], H)
    assert np.isnan(out[2]).all()


def test_simulate_api_edges():
    from preganplus_amd import _native
    L = _native.lib()
    L.pgp_simulate.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 6
    assert L.pgp_simulate(65, 1, 1, 1, 1, 1, 1, None) == -2
    assert L.pgp_simulate(16, 0, None, None, None, None, None, None) == 0
    assert L.pgp_simulate(16, 1, None, None, None, None, None, None) == -1
    with pytest.raises(ValueError):
        SIM.Simulation(16).score(SIM.synth_envs(2, 16), np.zeros((2, 16, 15)), np.zeros((2, 16, 16)))


@pytest.mark.parametrize("H,B", [(16, 37), (50, 9)])
def test_gan_step_with_device_labels(H, B):
    """train_gan_batched (labels from pgp_simulate on the generator's output)
    == the same step with the oracle's labels computed on the host from that
    output: identical parameters after Disc and Gen AdamW steps."""
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    w = W.synth_weights(H, seed=8)
    rng = np.random.Generator(np.random.PCG64(H + B))
    emb = np.where(rng.uniform(size=(B, H, 1)) < 0.3, rng.uniform(size=(B, H, 2)), 0.0)
    sched = np.zeros((B, H, H))
    sched[np.arange(B)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(B, H))] = 1.0
    envs = SIM.synth_envs(B, H, seed=B)
    t1 = TR.Trainer(H, w, max_batch=B)
    out, target = TR.train_gan_batched(t1, SIM.Simulation(H), envs, emb, sched)
    t2 = TR.Trainer(H, w, max_batch=B)
    ns, _ = t2.gan_forward(emb, sched)
    ref, rt = SO.simulate_batch(envs, ns.cpu().numpy(), sched.astype(np.float32), H)
    assert np.array_equal(out.cpu().numpy(), ref) and np.array_equal(target.cpu().numpy(), rt)
    t2.gan_disc_backward(rt)
    t2.adam_step("disc")
    t2.gan_gen_backward(B)
    t2.adam_step("gen")
    torch.cuda.synchronize()
    assert torch.equal(t1.P, t2.P)
