"""GPU parity of the PreGAN (FPE_16) variant — BASELINE config C4, SURVEY §8 a14:
K4 (pgp_fpe.hip) + K3 through pgp_forward_fpe vs the reference fixtures
(tests/golden/make_golden_fpe.py: FPE_16/Gen_16/Disc_16 from checkpoints/, GRU
h0 recorded) and the fp64 oracle.  Tolerance as the north star: scores and
probabilities rtol 1e-4 in fp32; decisions exact outside their derived fp32
error bound (tests/decision_bounds.py), and exact everywhere on the committed
fixtures."""
import numpy as np
import pytest
import torch

from oracle import pregan_oracle as O
from preganplus_amd import weights as W
from tests.parity_utils import assert_parity

pytestmark = pytest.mark.gpu

_models = {}


def model(key, w, H=16):
    from preganplus_amd.model import FPEDecisionModel
    if key not in _models:
        _models[key] = FPEDecisionModel(H, w)
    return _models[key]


def run(m, windows, h0, sched):
    from preganplus_amd.model import to_numpy
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.float32), device="cuda")
    out = m.forward(t(windows), t(h0), t(sched))
    torch.cuda.synchronize()
    return to_numpy(out)


def as_parity(got, ref):
    """Map FPE outputs onto assert_parity's keys: the anomaly softmax plays the
    role of the detect logits, the discriminator probs are 'probs'."""
    g = dict(got, logits=got["scores"])
    r = dict(ref, logits=ref["probs"], probs=ref["gprobs"])
    return g, r


def shipped():
    w, _ = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    return w


def test_fpe_reference_fixtures():
    z = np.load("tests/golden/fpe_h16.npz")
    ref = {k: z[k] for k in z.files}
    w = shipped()
    got = run(model("ship", w), ref["windows"], ref["h0"], ref["sched"])
    g, r = as_parity(got, ref)
    r["sched32"] = ref["sched"].astype(np.float32)
    assert_parity(g, r, w, ref["sched"], check_latent=False, exact=True)
    for k in ("cls", "any", "keep", "gen_target"):
        assert np.array_equal(got[k], ref[k]), k


@pytest.mark.parametrize("part", ["", "b/"])
def test_fpe50_reference_fixtures(part):
    """C4 at 50 hosts: the reference FPE_16 class instantiated at n_hosts=50
    with Gen_50/Disc_50 (tests/golden/make_golden_fpe50.py).  Set "b/" (anomaly
    bias shifted) holds windows without any flagged host; every decision must
    match the reference exactly."""
    from tests.test_oracle_golden import fpe50_weights
    z = np.load("tests/golden/fpe_h50.npz")
    ref = {k[len(part):]: z[k] for k in z.files if k.startswith(part) and (part or "/" not in k)}
    w = fpe50_weights(z, part)
    got = run(model("fix50" + part, w, 50), ref["windows"], ref["h0"], ref["sched"])
    g, r = as_parity(got, ref)
    assert_parity(g, r, w, ref["sched"], check_latent=False, exact=True)
    for k in ("cls", "any", "keep", "gen_target", "final_target"):
        assert np.array_equal(got[k], ref[k]), k
    if part:
        assert 0 < got["any"].sum() < got["any"].size


@pytest.mark.parametrize("H,B", [(16, 1), (16, 63), (16, 64), (16, 65), (16, 1000), (50, 1), (50, 65), (50, 700)])
def test_fpe_synthetic_vs_oracle(H, B):
    w = W.synth_fpe_weights(H, seed=11)
    rng = np.random.Generator(np.random.PCG64(B))
    x = rng.uniform(0, 1.2, size=(B, 3, 3 * H)).astype(np.float32)
    h0 = rng.standard_normal((B, 3)).astype(np.float32)
    sched = rng.uniform(0, 1, size=(B, H, H)).astype(np.float32)
    ref = O.forward_fpe(w, x.astype(np.float64), h0.astype(np.float64), sched.astype(np.float64))
    got = run(model(f"syn{H}", w, H), x, h0, sched)
    g, r = as_parity(got, ref)
    r["sched32"] = sched
    assert_parity(g, r, w, sched, check_latent=False)


def test_fpe_edge_inputs():
    """zeros, constant rows (all edge scores equal), large values (softmax
    saturation), negative h0 extremes."""
    w = shipped()
    B = 4
    x = np.zeros((B, 3, 48), np.float32)
    x[1] = 0.5
    x[2] = np.linspace(0, 40, 144).reshape(3, 48)
    x[3] = -np.linspace(0, 3, 144).reshape(3, 48)
    h0 = np.array([[0, 0, 0], [1, -1, 0.5], [5, 5, 5], [-5, 2, -3]], np.float32)
    sched = np.tile(np.eye(16, dtype=np.float32), (B, 1, 1))
    ref = O.forward_fpe(w, x.astype(np.float64), h0.astype(np.float64), sched.astype(np.float64))
    got = run(model("ship", w), x, h0, sched)
    g, r = as_parity(got, ref)
    r["sched32"] = sched
    assert_parity(g, r, w, sched, check_latent=False)


def test_fpe50_edge_inputs_and_batch_invariance():
    """H=50: zeros (every edge score equal), constant rows, large and negative
    loads; then a 4,099-window launch vs its ragged tail run alone."""
    w = W.synth_fpe_weights(50, seed=0)
    m = model("edge50", w, 50)
    B = 4
    x = np.zeros((B, 3, 150), np.float32)
    x[1] = 0.5
    x[2] = np.linspace(0, 40, 450).reshape(3, 150)
    x[3] = -np.linspace(0, 3, 450).reshape(3, 150)
    h0 = np.array([[0, 0, 0], [1, -1, 0.5], [5, 5, 5], [-5, 2, -3]], np.float32)
    sched = np.tile(np.eye(50, dtype=np.float32), (B, 1, 1))
    ref = O.forward_fpe(w, x.astype(np.float64), h0.astype(np.float64), sched.astype(np.float64))
    got = run(m, x, h0, sched)
    g, r = as_parity(got, ref)
    assert_parity(g, r, w, sched, check_latent=False)
    rng = np.random.Generator(np.random.PCG64(9))
    B = 4099
    x = rng.uniform(0, 1, size=(B, 3, 150)).astype(np.float32)
    h0 = rng.standard_normal((B, 3)).astype(np.float32)
    sched = rng.uniform(0, 1, size=(B, 50, 50)).astype(np.float32)
    big = run(m, x, h0, sched)
    small = run(m, x[-37:], h0[-37:], sched[-37:])
    for k in small:
        assert np.array_equal(big[k][-37:], small[k]), k


@pytest.mark.timeout(900)
@pytest.mark.parametrize("seed_off", [0, 970])
def test_fpe50_full_size_census(seed_off):
    """BASELINE C4 at its full size: 65,536 windows at 50 hosts through K4 + K3,
    every window compared with the fp64 FPE oracle (tests/census.py): scores /
    protos / probs within the north-star tolerance, every decision equal
    unless its fp64 margin lies inside its derived fp32 bound."""
    import json
    import os

    from preganplus_amd.model import to_numpy
    from tests import census as CE
    from tests import decision_bounds as DB
    from tests.test_gpu_parity import _c2_torch
    H, B = 50, 65536
    w = W.synth_fpe_weights(H, seed=0)
    m = model("census50", w, H)
    seed = 77 + seed_off
    x, s = _c2_torch(B, H, seed=seed)
    g = torch.Generator(device="cuda").manual_seed(seed + 1)
    h0 = torch.randn((B, 3), generator=g, device="cuda")
    full = to_numpy(m.forward(x, h0, s))
    torch.cuda.synchronize()
    for lo, hi in ((0, 64), (B // 2 - 7, B // 2 + 50), (B - 45, B)):
        part = to_numpy(m.forward(x[lo:hi].contiguous(), h0[lo:hi].contiguous(), s[lo:hi].contiguous()))
        torch.cuda.synchronize()
        for k in part:
            assert np.array_equal(full[k][lo:hi], part[k]), (k, lo, hi)
    got = dict(full, logits=full["scores"])
    anom = got["logits"][..., 1] > got["logits"][..., 0]
    assert np.array_equal(full["any"], anom.any(axis=1))
    assert np.array_equal(full["cls"] < 0, ~anom)
    x32, h32 = x.cpu().numpy(), h0.cpu().numpy()
    sidx = s.argmax(dim=-1).cpu().numpy()
    del x, s, h0
    st, worst = CE.run(w, x32, sidx, got, log=print, h0=h32)
    res = {"variant": "fpe", "H": H, "windows": B, "seed": seed, "census": st, "worst_error_over_tolerance": worst}
    print("CENSUS", json.dumps(res))
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/census_fpe_h{H}_b{B}_s{seed}.json", "w") as f:
        json.dump(res, f, indent=1)
    assert worst["logits"] <= 1.0 and worst["protos"] <= 1.0 and worst["probs"] <= 1.0, worst
    assert not DB.violations(st), st
    assert st["windows"] == B
    # the in-band share is a property of the data's margins, not of the kernel: the
    # seeded (untrained) Disc_50 puts its two probabilities within 1e-4 of each other
    # for ~0.15 % of the windows (101 of 65,536 at seed 77, all decided as the oracle)
    for kind, cap in (("anomaly", 1e-3), ("class", 1e-3), ("keep", 5e-3), ("gen", 1e-3)):
        assert st[kind]["in_band"] <= cap * max(st[kind]["n"], 1), (kind, st[kind])
    for kind in ("any", "class", "keep", "final"):
        assert st[kind]["mismatch"] == 0, (kind, st[kind])
    assert st["anomaly"]["mismatch"] <= 8 and st["gen"]["mismatch"] <= 8, st


def test_fpe_batch_invariance_and_errors():
    from preganplus_amd._native import NativeError
    w = shipped()
    m = model("ship", w)
    rng = np.random.Generator(np.random.PCG64(5))
    B = 8192
    x = rng.uniform(0, 1, size=(B, 3, 48)).astype(np.float32)
    h0 = rng.standard_normal((B, 3)).astype(np.float32)
    sched = rng.uniform(0, 1, size=(B, 16, 16)).astype(np.float32)
    big = run(m, x, h0, sched)
    small = run(m, x[-37:], h0[-37:], sched[-37:])
    for k in small:
        assert np.array_equal(big[k][-37:], small[k]), k
    t = lambda a: torch.tensor(a, device="cuda")
    with pytest.raises(ValueError):
        m.forward(t(x[:4]), t(h0[:3]), t(sched[:4]))
    out = m.alloc_outputs(0)
    m.forward(t(x[:0]), t(h0[:0]), t(sched[:0]), out=out)   # empty batch is a no-op
    # the PreGAN+ entry point refuses an FPE model
    from preganplus_amd import _native
    L = _native.lib()
    rc = L.pgp_forward(m._h, 1, *([None] * 11), None)
    assert rc == -4
    with pytest.raises(NativeError):
        _native.check(rc, "pgp_forward")


def test_pregan_plugin_run_model_matches_reference():
    """PreGANRecovery.run_model over the 4 recorded intervals (training on):
    same decisions as the reference plugin, GAN weights after the 4 Disc/Gen
    AdamW steps within fp32 tolerance.  torch.manual_seed(2000+step) before
    each call reproduces the reference's h0 draw."""
    from preganplus_amd.recovery import PreGANRecovery
    from tests.test_gpu_train import close
    from tests.test_train_oracle_golden import fake_env
    w, extra = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    z = np.load("tests/golden/pregan_plugin_h16.npz")
    rec = PreGANRecovery(16, "", training=True, weights=w, extra=extra)
    for step in range(4):
        env = fake_env(z, step, extra["train_time_data"], z["schedule_series"])
        rec.setEnvironment(env)
        torch.manual_seed(2000 + step)
        dec = rec.run_model(None, [tuple(x) for x in z[f"s{step}/decision_in"]])
        assert [tuple(map(int, d)) for d in dec] == [tuple(x) for x in z[f"s{step}/decision_out"].tolist()], step
    pw = rec.trainer.weights_numpy()
    for k, v in pw["gen"].items():
        close(v, z[f"end/g/{k}"], rel=1e-4, abs_scale=1e-5, what="g " + k)
    for k, v in pw["disc"].items():
        close(v, z[f"end/d/{k}"], rel=1e-4, abs_scale=1e-5, what="d " + k)
    np.testing.assert_allclose(np.array(rec.accuracy_list[-4:]), z["end/accuracy_list"], rtol=1e-4, atol=1e-6)
    assert rec.epoch == int(extra["meta/gen/epoch"]) + 4


def test_pregan_plugin_inference_only():
    """training=False: frozen GAN, the decision comes from the single
    pgp_forward_fpe call (K3's probs)."""
    from preganplus_amd.recovery import PreGANRecovery
    from tests.test_train_oracle_golden import fake_env
    w, extra = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    z = np.load("tests/golden/pregan_plugin_h16.npz")
    rec = PreGANRecovery(16, "", training=False, weights=w, extra=extra)
    env = fake_env(z, 0, extra["train_time_data"], z["schedule_series"])
    rec.setEnvironment(env)
    torch.manual_seed(2000)
    dec = rec.run_model(None, [tuple(x) for x in z["s0/decision_in"]])
    # oracle: same window / h0 / frozen weights
    torch.manual_seed(2000)
    h0 = torch.randn(1, 1, 3, dtype=torch.double).numpy().reshape(1, 3)
    win = O.inference_window(env.stats.time_series, extra["train_time_data"])
    ref = O.forward_fpe(w, win[None], h0, np.asarray(z["s0/sched"], np.float64)[None])
    if not ref["any"][0]:
        assert dec == [tuple(x) for x in z["s0/decision_in"]]
    assert rec.classes == ref["cls"][0].tolist()
