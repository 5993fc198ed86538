"""GPU parity of ``pgp_tune_forward_many`` (csrc/pgp_tune1.hip fwd_many_kernel):
n independent batch-1 forwards from the master weights, the batched forward
accuracy() scores (train.py:94-109).  Against the token-major tuning forward
(pgp_tune_forward) on the same windows and weights — same fp32 model, a
different operation order, so to fp32 tolerance — and the argmax decisions
accuracy() counts are equal."""
import numpy as np
import pytest
import torch

from preganplus_amd import weights as W

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H", [8, 16])
def test_forward_many_matches_tune_forward(H):
    from preganplus_amd import train as TR
    n = 24
    w = W.synth_weights(H, seed=5 + H)
    tr = TR.Trainer(H, w, max_batch=n)
    rng = np.random.default_rng(H)
    wins = rng.random((n, 3, 3 * H)).astype(np.float32)
    wins[3] = 0.0
    wins[4] = 1.0
    x = torch.tensor(wins, device=tr.device)
    lg, pr = tr.tune_forward(x)
    lg, pr = lg[:n].cpu().numpy(), pr[:n].cpu().numpy()
    out = torch.zeros(4 * n * H, dtype=torch.float64, device=tr.device)
    tr.tune_forward_many(x, out[:2 * n * H], out[2 * n * H:])
    o = out.cpu().numpy()
    lg1, pr1 = o[:2 * n * H].reshape(n, H, 2), o[2 * n * H:].reshape(n, H, 2)
    np.testing.assert_allclose(lg1, lg, rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(pr1, pr, rtol=1e-4, atol=1e-6)
    gap = np.abs(lg[..., 1] - lg[..., 0])
    sure = gap > 1e-4
    assert np.array_equal((lg1[..., 1] > lg1[..., 0])[sure], (lg[..., 1] > lg[..., 0])[sure])
    # the widened fp32 values are exact fp32 numbers
    assert np.array_equal(lg1.astype(np.float32).astype(np.float64), lg1)


def test_forward_many_rejects_unsupported_hosts():
    from preganplus_amd import _native
    from preganplus_amd import train as TR
    tr = TR.Trainer(50, W.synth_weights(50, seed=1), max_batch=2)
    z = torch.zeros(2 * 9 * 50, device="cuda")
    o = torch.zeros(4 * 2 * 50, dtype=torch.float64, device="cuda")
    with pytest.raises(_native.NativeError):
        tr.tune_forward_many(z.view(2, 3, 150), o, o)
