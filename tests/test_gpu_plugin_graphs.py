"""The plugin's batch-1 latency plumbing against the eager path it replaces:
train_gan's two captured graphs (``_GanGraph``) vs ``train_gan_eager``
(individual launches, PreGANPlus.py:60-75), bit for bit, including the
post-training Disc gate recover_decision reads; the fused batch-1 GAN step
(pgp_gan_forward1 / pgp_gan_step1, one launch per graph) vs the same eager
path to fp32 / AdamW-step tolerance; and the packed single-copy detect outputs
vs the per-tensor outputs."""
import numpy as np
import pytest
import torch

from preganplus_amd import weights as W

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scores", [(1.0, 2.0), (3.0, 1.0)])
def test_gan_graph_equals_eager(scores):
    from preganplus_amd import train as TR
    w, extra = W.load_npz("preganplus_amd/data/simulator_16.npz")
    z = np.load("tests/golden/gan_h16.npz")
    a, b = TR.Trainer(16, w, extra), TR.Trainer(16, w, extra)
    for call in range(3):      # capture, then replays with new inputs
        emb = z["emb"] * (1 + 0.1 * call)
        sched = np.roll(z["sched"], call, axis=1)
        ia, ib = iter(scores), iter(scores)
        ra = TR.train_gan_eager(a, emb, sched, lambda s: next(ia))
        rb = TR.train_gan(b, emb, sched, lambda s: next(ib), fused=False)
        np.testing.assert_array_equal(ra[0], rb[0])
        assert ra[1:] == rb[1:]
        for t in ("P", "m", "v"):
            assert torch.equal(getattr(a, t), getattr(b, t)), t
        assert [t["step"] for t in a.tensors] == [t["step"] for t in b.tensors]
        _, probs = a.gan_forward(np.asarray(emb)[None], np.asarray(sched)[None])
        np.testing.assert_array_equal(probs[0].cpu().numpy(), b.gan_probs_after)


@pytest.mark.parametrize("scores", [(1.0, 2.0), (3.0, 1.0)])
def test_fused_gan_step_matches_eager(scores):
    """pgp_gan_forward1 + pgp_gan_step1 against the batched kernels at batch 1
    over 4 consecutive calls: schedules, losses and the gate to fp32 tolerance,
    parameters to within one AdamW step where a gradient element is rounding
    noise around zero (m / sqrt(v) is its sign on the first steps), moments
    and step counts."""
    from preganplus_amd import train as TR
    w, extra = W.load_npz("preganplus_amd/data/simulator_16.npz")
    z = np.load("tests/golden/gan_h16.npz")
    a, b = TR.Trainer(16, w, extra), TR.Trainer(16, w, extra)
    lr = max(a.lrs["gen"], a.lrs["disc"])
    for call in range(4):
        emb = z["emb"] * (1 + 0.1 * call)
        sched = np.roll(z["sched"], call, axis=1)
        ia, ib = iter(scores), iter(scores)
        ra = TR.train_gan_eager(a, emb, sched, lambda s: next(ia))
        rb = TR.train_gan(b, emb, sched, lambda s: next(ib), fused=True)
        np.testing.assert_allclose(rb[0], ra[0], rtol=1e-5, atol=1e-5)
        assert ra[1:3] == rb[1:3]                               # simulated scores
        np.testing.assert_allclose(rb[3:], ra[3:], rtol=1e-4, atol=1e-6)   # gen_loss, disc_loss
        pa, pb = a.P.cpu().numpy(), b.P.cpu().numpy()
        d = np.abs(pa - pb)
        assert (d <= 1e-5 * np.abs(pa) + 2.5 * lr * (call + 1)).all(), float(d.max())
        assert np.mean(d > 1e-5 * np.abs(pa) + 1e-7) < 1e-3    # step-sized differences are rare
        ma, mb = a.m.cpu().numpy(), b.m.cpu().numpy()
        np.testing.assert_allclose(mb, ma, rtol=1e-3, atol=1e-5 * float(np.abs(ma).max()))
        assert [t["step"] for t in a.tensors] == [t["step"] for t in b.tensors]
        _, probs = a.gan_forward(np.asarray(emb)[None], np.asarray(sched)[None])
        np.testing.assert_allclose(b.gan_probs_after, probs[0].cpu().numpy(), rtol=1e-4, atol=1e-6)


def test_fused_gan_step_h8_matches_eager():
    """The same at 8 hosts on seeded weights (one-hot schedules, as GOBI's)."""
    from preganplus_amd import train as TR
    H = 8
    w = W.synth_weights(H, seed=4)
    a, b = TR.Trainer(H, w), TR.Trainer(H, w)
    lr = max(a.lrs["gen"], a.lrs["disc"])
    rng = np.random.default_rng(8)
    for call in range(3):
        emb = rng.random(2 * H).astype(np.float32)
        sched = np.eye(H)[rng.integers(0, H, H)]
        scores = (1.0, 2.0) if call % 2 else (2.0, 1.0)
        ia, ib = iter(scores), iter(scores)
        ra = TR.train_gan_eager(a, emb, sched, lambda s: next(ia))
        rb = TR.train_gan(b, emb, sched, lambda s: next(ib), fused=True)
        np.testing.assert_allclose(rb[0], ra[0], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(rb[3:], ra[3:], rtol=1e-4, atol=1e-6)
        pa, pb = a.P.cpu().numpy(), b.P.cpu().numpy()
        assert (np.abs(pa - pb) <= 1e-5 * np.abs(pa) + 2.5 * lr * (call + 1)).all()
        _, probs = a.gan_forward(np.asarray(emb)[None], np.asarray(sched)[None])
        np.testing.assert_allclose(b.gan_probs_after, probs[0].cpu().numpy(), rtol=1e-4, atol=1e-6)


def test_fused_gan_step_rejects_unsupported_hosts():
    from preganplus_amd import _native
    from preganplus_amd import train as TR
    tr = TR.Trainer(50, W.synth_weights(50, seed=1))
    z = torch.zeros(2600, device="cuda")
    with pytest.raises(_native.NativeError):
        tr.gan_forward1(z[:100], z[100:2600], z[:2500], z[:2])


def test_packed_outputs_equal_plain():
    from preganplus_amd.model import DecisionModel, to_numpy
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    m = DecisionModel(16, w)
    rng = np.random.default_rng(1)
    x = torch.tensor(rng.uniform(0, 1, (3, 3, 48)), dtype=torch.float32, device=m.device)
    s = torch.tensor(rng.uniform(0, 1, (3, 16, 16)), dtype=torch.float32, device=m.device)
    a = to_numpy(m.forward(x, s))
    b = to_numpy(m.forward(x, s, out=m.alloc_outputs(3, packed=True)))
    assert a.keys() == b.keys()
    for k in a:
        assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), k
