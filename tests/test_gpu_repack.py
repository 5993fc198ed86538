"""Device repack (pgp_repack_master, pgp_repack.hip) vs the host packer
(pgp_load_weights_master): the packing code is shared (pgp_packcore.hpp, fp64,
no contraction), so the two must produce the same packed bits.  Checked through
the kernels: after perturbing the master weights and prototypes as an
optimizer step would, a model rebuilt on the device and one rebuilt on the host
give bit-identical forward outputs on a batch of windows, for every compiled
host count (tail mode H=50 included)."""
import numpy as np
import pytest
import torch

from preganplus_amd import weights as W

pytestmark = pytest.mark.gpu


def _outputs(model, x, s):
    out = model.forward(x, s)
    torch.cuda.synchronize()
    return {k: v.clone() for k, v in out.items() if v is not None}


@pytest.mark.parametrize("H", [8, 16, 32, 50, 64])
def test_device_repack_equals_host_pack(H):
    from preganplus_amd import train as TR
    from preganplus_amd.model import DecisionModel
    rng = np.random.default_rng(H)
    w = W.synth_weights(H, seed=H)
    tr = TR.Trainer(H, w, max_batch=1)
    # an "optimizer step": perturb every master weight and the prototypes
    tr.P.add_(torch.randn_like(tr.P) * 1e-2)
    protos = rng.uniform(0, 1, (H, 2))
    host, dev = DecisionModel(H, w), DecisionModel(H, w)
    host.load_master(tr.P, protos)
    pd = torch.tensor(protos, dtype=torch.float64, device=tr.device)
    dev.repack_master(tr.P, pd, protos)
    B = 48
    x = torch.tensor(rng.uniform(0, 1, (B, 3, 3 * H)), dtype=torch.float32, device=tr.device)
    s = torch.tensor(rng.uniform(0, 1, (B, H, H)), dtype=torch.float32, device=tr.device)
    a, b = _outputs(host, x, s), _outputs(dev, x, s)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    # and the repack really changed the model (outputs differ from the initial weights)
    base = _outputs(DecisionModel(H, w), x, s)
    assert not torch.equal(base["logits"], b["logits"])


@pytest.mark.parametrize("H", [16, 50])
def test_repack_sections_equal_full_repack(H):
    """pgp_repack_master_sections: the PreGAN+ part (1) then the GAN part (2),
    or the other way round, give the same packed model as one full repack
    (bit-identical forward outputs), and each part alone changes only its own
    outputs (the GAN part leaves the logits as they were)."""
    from preganplus_amd import train as TR
    from preganplus_amd.model import DecisionModel
    rng = np.random.default_rng(7 + H)
    w = W.synth_weights(H, seed=H + 1)
    tr = TR.Trainer(H, w, max_batch=1)
    tr.P.add_(torch.randn_like(tr.P) * 1e-2)
    protos = rng.uniform(0, 1, (H, 2))
    pd = torch.tensor(protos, dtype=torch.float64, device=tr.device)
    B = 40
    x = torch.tensor(rng.uniform(0, 1, (B, 3, 3 * H)), dtype=torch.float32, device=tr.device)
    s = torch.tensor(rng.uniform(0, 1, (B, H, H)), dtype=torch.float32, device=tr.device)
    full, a, b, gan_only = (DecisionModel(H, w) for _ in range(4))
    full.repack_master(tr.P, pd, protos)
    a.repack_master(tr.P, pd, protos, sections=1)
    a.repack_master(tr.P, pd, protos, sections=2)
    b.repack_master(tr.P, pd, protos, sections=2)
    b.repack_master(tr.P, pd, protos, sections=1)
    ref = _outputs(full, x, s)
    for m in (a, b):
        o = _outputs(m, x, s)
        for k in ref:
            assert torch.equal(ref[k], o[k]), k
    gan_only.repack_master(tr.P, pd, protos, sections=2)
    base, g = _outputs(DecisionModel(H, w), x, s), _outputs(gan_only, x, s)
    assert torch.equal(base["logits"], g["logits"])
    assert not torch.equal(base["probs"], g["probs"])


def test_plugin_sync_uses_device_state():
    """PreGANPlusRecovery.sync_inference_weights after tune_model rebuilds from
    the tuning graph's device state: same outputs as the host repack."""
    from preganplus_amd import train as TR
    from preganplus_amd.model import DecisionModel
    w, extra = W.load_npz("preganplus_amd/data/simulator_16.npz")
    z = np.load("tests/golden/tune_h16.npz")
    tr = TR.Trainer(16, w, extra)
    st = TR.TuneState(z["protos0"], float(z["factor0"]))
    TR.backprop(tr, st, z["windows"], z["anom"], z["cls"])
    host, dev = DecisionModel(16, w), DecisionModel(16, w)
    host.load_master(tr.P, st.protos)
    dev.repack_master(tr.P, tr.tune_state_dev[:32], st.protos)
    rng = np.random.default_rng(3)
    x = torch.tensor(rng.uniform(0, 1, (20, 3, 48)), dtype=torch.float32, device=tr.device)
    s = torch.tensor(rng.uniform(0, 1, (20, 16, 16)), dtype=torch.float32, device=tr.device)
    a, b = _outputs(host, x, s), _outputs(dev, x, s)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_repack_rejects_fpe_model():
    from preganplus_amd import _native
    from preganplus_amd.model import FPEDecisionModel
    w, _ = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    m = FPEDecisionModel(16, w)
    P = torch.zeros(16, device=m.device)
    pd = torch.zeros((3, 2), dtype=torch.float64, device=m.device)
    with pytest.raises((_native.NativeError, ValueError)):
        m.repack_master(P, pd)
