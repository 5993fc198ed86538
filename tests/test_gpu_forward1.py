"""GPU parity of the plugin's batch-1 forward (``pgp_forward1``,
csrc/pgp_tune1.hip infer1_kernel): run_model's detect / diagnose / generate
for one window straight from the training master weights, one launch.  Held to
the same bar as the batched K1-K3 path: against the reference's own fixture
(every decision exact) and against the fp64 oracle on synthetic windows and
edge inputs (decision census with the per-decision fp32 bounds)."""
import numpy as np
import pytest
import torch

from oracle import pregan_oracle as O
from preganplus_amd import weights as W
from tests.parity_utils import assert_parity
from tests.test_gpu_parity import c2, fixture

pytestmark = pytest.mark.gpu


def run1(H, w, x, s):
    """forward1 per window; outputs stacked like DecisionModel's to_numpy."""
    from preganplus_amd import train as TR
    from preganplus_amd.model import DecisionModel, to_numpy
    tr = TR.Trainer(H, w, max_batch=1)
    dev = tr.device
    pd = torch.tensor(np.asarray(w["prototypes"], np.float64), device=dev)
    m = DecisionModel(H, w)
    out = m.alloc_outputs(1, packed=True)
    rows = []
    for i in range(x.shape[0]):
        win = torch.tensor(np.asarray(x[i], np.float32), device=dev).contiguous()
        sc = torch.tensor(np.asarray(s[i], np.float32), device=dev).contiguous()
        tr.forward1(win, sc, pd, out)
        rows.append(to_numpy(out))
    return {k: np.concatenate([r[k] for r in rows]) for k in rows[0]}


def test_forward1_reference_fixture_h16():
    w, ref = fixture(16)
    got = run1(16, w, ref["windows"], ref["sched"])
    assert_parity(got, ref, w, ref["sched"], check_latent=False, exact=True)
    for k in ("cls", "gen_target", "keep", "final_target", "any"):
        assert np.array_equal(got[k], ref[k]), k


@pytest.mark.parametrize("H", [8, 16])
def test_forward1_synthetic_vs_oracle(H):
    rng = np.random.Generator(np.random.PCG64(300 + H))
    w = W.synth_weights(H, seed=11)
    x, s = c2(rng, 48, H, dense=6)
    ref = O.forward(w, x, s)
    got = run1(H, w, x, s)
    assert_parity(got, ref, w, s, check_latent=False)


def test_forward1_matches_batched_path():
    """The batch-1 kernel and K1-K3 on the same windows: logits / probs to fp32
    tolerance, every decision equal (the shipped weights, recorded windows)."""
    from preganplus_amd.model import DecisionModel, to_numpy
    w, ref = fixture(16)
    x, s = ref["windows"][:64], ref["sched"][:64]
    got = run1(16, w, x, s)
    m = DecisionModel(16, w)
    b = to_numpy(m.forward(torch.tensor(x, dtype=torch.float32, device="cuda"),
                           torch.tensor(s, dtype=torch.float32, device="cuda")))
    np.testing.assert_allclose(got["logits"], b["logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(got["probs"], b["probs"], rtol=1e-4, atol=1e-6)
    for k in ("cls", "any", "keep", "final_target", "gen_target"):
        assert np.array_equal(got[k], b[k]), k


def test_forward1_edge_inputs_h16():
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    H = 16
    x = np.zeros((6, 3, 48))
    x[1] = 1.0
    x[2] = 50.0
    x[3, :, ::3] = 1.0
    x[4] = np.linspace(0, 2, 144).reshape(3, 48)
    x[5] = 1e-6
    s = np.zeros((6, H, H))
    s[1, :, 3] = s[1, :, 5] = 1.0
    s[2] = np.eye(H)
    s[3] = 0.5
    s[4:] = np.eye(H)[::-1]
    ref = O.forward(w, x, s)
    got = run1(H, w, x, s)
    assert_parity(got, ref, w, s, check_latent=False)
    assert got["final_target"][0].tolist() == [0] * H
    assert got["final_target"][1].tolist() == [3] * H


def test_forward1_rejects_unsupported_hosts():
    from preganplus_amd import _native
    from preganplus_amd import train as TR
    from preganplus_amd.model import DecisionModel
    w = W.synth_weights(50, seed=1)
    tr = TR.Trainer(50, w, max_batch=1)
    out = DecisionModel(50, w).alloc_outputs(1, packed=True)
    z = torch.zeros(50 * 50, device="cuda")
    with pytest.raises(_native.NativeError):
        tr.forward1(z, z, torch.zeros((50, 2), dtype=torch.float64, device="cuda"), out)
