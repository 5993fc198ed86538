"""GPU parity: the HIP path (through the C-ABI) vs the reference fixtures and
the fp64 oracle.  Marked gpu: runs on the MI355X box only."""
import numpy as np
import pytest
import torch

from oracle import pregan_oracle as O
from preganplus_amd import weights as W
from tests.parity_utils import assert_parity

pytestmark = pytest.mark.gpu

GOLD = "tests/golden"
_models = {}


def get_model(H, w, key):
    from preganplus_amd.model import DecisionModel
    if key not in _models:
        _models[key] = DecisionModel(H, w)
    return _models[key]


def run(model, windows, sched, latent=False, stage_split=False):
    from preganplus_amd.model import to_numpy
    wt = torch.tensor(np.asarray(windows, dtype=np.float32), device="cuda")
    st = torch.tensor(np.asarray(sched, dtype=np.float32), device="cuda")
    if stage_split:
        out = model.alloc_outputs(wt.shape[0], latent)
        for s in (0, 1, 2, 3):
            model.forward(wt, st, out=out, stage=s)
    else:
        out = model.forward(wt, st, latent=latent)
    torch.cuda.synchronize()
    return to_numpy(out)


def fixture(H):
    z = np.load(f"{GOLD}/fwd_h{H}.npz")
    if H == 16:
        w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    else:
        w = W.synth_weights(H, int(z["weights_seed"]))
    ref = {k: z[k] for k in z.files}
    ref["sched32"] = z["sched"].astype(np.float32)
    return w, ref


@pytest.mark.parametrize("H", [16, 50])
def test_reference_fixtures(H):
    """HIP vs outputs of the reference's own modules (fp64, eval)."""
    w, ref = fixture(H)
    m = get_model(H, w, f"fix{H}")
    got = run(m, ref["windows"], ref["sched"], latent=True)
    # on the committed fixtures every decision must match exactly
    assert_parity(got, ref, w, ref["sched"], exact=True)
    assert np.array_equal(got["cls"], ref["cls"])
    assert np.array_equal(got["gen_target"], ref["gen_target"])
    assert np.array_equal(got["keep"], ref["keep"])


def test_reference_fixture_both_branches_h16():
    """H=16 windows on both sides of run_model's gates (no flagged host / some;
    discriminator keeps / overrides; make_golden_branches16.py): every decision
    exactly the reference's."""
    from tests.test_oracle_golden import branches16_weights
    z = np.load(f"{GOLD}/fwd_h16_branches.npz")
    w = branches16_weights(z)
    ref = {k: z[k] for k in z.files}
    ref["sched32"] = z["sched"].astype(np.float32)
    m = get_model(16, w, "branches16")
    got = run(m, ref["windows"], ref["sched"], latent=True)
    assert_parity(got, ref, w, ref["sched"], exact=True)
    for k in ("any", "keep", "cls", "gen_target", "final_target"):
        assert np.array_equal(got[k], ref[k]), k
    assert 0 < got["any"].sum() < got["any"].size and 0 < got["keep"].sum() < got["keep"].size


@pytest.mark.parametrize("H", [16, 50])
def test_stage_split_equals_fused_call(H):
    w, ref = fixture(H)
    m = get_model(H, w, f"fix{H}")
    a = run(m, ref["windows"][:40], ref["sched"][:40])
    b = run(m, ref["windows"][:40], ref["sched"][:40], stage_split=True)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def c2(rng, n, H, dense=0):
    x = rng.uniform(0, 0.6, size=(n, 3, 3 * H))
    spike = rng.uniform(0, 1, size=x.shape) < 0.02
    x[spike] = rng.uniform(0.9, 1.3, size=int(spike.sum()))
    s = np.zeros((n, H, H))
    s[np.arange(n)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(n, H))] = 1.0
    if dense:
        s[-dense:] = rng.uniform(0, 1, size=(dense, H, H))
    return x, s


@pytest.mark.parametrize("H", [8, 16, 32, 50, 64])
def test_synthetic_vs_oracle_ragged_batch(H):
    """Every compiled H, seeded weights, a batch that is not a multiple of 16."""
    rng = np.random.Generator(np.random.PCG64(100 + H))
    w = W.synth_weights(H, seed=7)
    x, s = c2(rng, 37, H, dense=5)
    ref = O.forward(w, x, s)
    ref["sched32"] = s.astype(np.float32)
    m = get_model(H, w, f"syn{H}")
    got = run(m, x, s, latent=True)
    assert_parity(got, ref, w, s)


@pytest.mark.parametrize("H", [32, 50])
def test_split_bf16_decoder_vs_fp32_decoder(H):
    """K2b's split-bf16 form (the default at H = 32, 50: six bf16 MFMAs per fp32
    product, pgp_decoder.hip) and its fp32-MFMA form on the same latent: both
    within the north-star tolerance of the fp64 oracle, their logits within a
    few fp32 ulps of the contraction's magnitude of each other, and every
    decision equal (on these inputs no decision sits in band)."""
    rng = np.random.Generator(np.random.PCG64(300 + H))
    w = W.synth_weights(H, seed=3)
    x, s = c2(rng, 517, H, dense=9)
    ref = O.forward(w, x, s)
    ref["sched32"] = s.astype(np.float32)
    m = get_model(H, w, f"dsplit{H}")
    m.decoder_split(True)
    a = run(m, x, s)
    m.decoder_split(False)
    b = run(m, x, s)
    m.decoder_split(True)
    assert_parity(a, ref, w, s)
    assert_parity(b, ref, w, s)
    # the split form is no less accurate than the fp32 MFMA (tools/micro/bf16_split.hip:
    # the same error level): its worst logit / proto error against the fp64 oracle
    # within twice the fp32 form's (both far inside the north-star tolerance)
    for k in ("logits", "protos"):
        ea = np.abs(a[k].astype(np.float64) - ref[k]).max()
        eb = np.abs(b[k].astype(np.float64) - ref[k]).max()
        assert ea <= 2 * eb + 1e-7, (k, ea, eb)
    for k in ("cls", "any", "keep", "final_target", "gen_target"):
        assert np.array_equal(a[k], b[k]), k
    assert not np.array_equal(a["logits"], b["logits"])   # the two forms really ran


@pytest.mark.parametrize("dense", [0, 40])
def test_split_bf16_gan_vs_fp32_gan(dense):
    """K3's split-bf16 form (the default at H = 50, pgp_gansplit.hip; one-hot
    schedule blocks in three products, dense ones in six) and its fp32-MFMA
    form: both within tolerance of the fp64 oracle, probabilities within fp32
    rounding of each other, every decision equal, and the one-hot shortcut
    bitwise equal to the six-product form (its other products add exact zeros:
    here checked by a batch whose dense windows take the six-product path in
    the same launch)."""
    H = 50
    rng = np.random.Generator(np.random.PCG64(77 + dense))
    w = W.synth_weights(H, seed=5)
    x, s = c2(rng, 300, H, dense=dense)
    ref = O.forward(w, x, s)
    ref["sched32"] = s.astype(np.float32)
    m = get_model(H, w, "gsplit50")
    m.gan_split(True)
    a = run(m, x, s)
    m.gan_split(False)
    b = run(m, x, s)
    m.gan_split(True)
    assert_parity(a, ref, w, s)
    assert_parity(b, ref, w, s)
    ea = np.abs(a["probs"].astype(np.float64) - ref["probs"]).max()
    eb = np.abs(b["probs"].astype(np.float64) - ref["probs"]).max()
    assert ea <= 2 * eb + 1e-7, (ea, eb)
    for k in ("keep", "final_target", "gen_target", "any", "cls"):
        assert np.array_equal(a[k], b[k]), k
    # a window's outputs do not depend on the other windows of its wave (the
    # one-hot shortcut is chosen per wave): the first 16 alone give the same bits
    c = run(m, x[:16], s[:16])
    for k in a:
        assert np.array_equal(a[k][:16], c[k]), k


def test_edge_inputs_h16():
    """Constant / zero / extreme windows; all-zero and tied schedules."""
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    H = 16
    x = np.zeros((8, 3, 48))
    x[1] = 1.0                      # constant rows
    x[2] = 50.0                     # far outside the training range
    x[3, :, ::3] = 1.0              # cpu saturated everywhere
    x[4] = np.linspace(0, 2, 144).reshape(3, 48)
    x[5, 2] = 1.3
    x[6] = 1e-6
    x[7, 0] = 0.9
    s = np.zeros((8, H, H))         # all-zero rows -> argmax 0
    s[1, :, 3] = s[1, :, 5] = 1.0   # ties -> first index
    s[2] = np.eye(H)
    s[3] = 0.5
    s[4:] = np.eye(H)[::-1]
    ref = O.forward(w, x, s)
    ref["sched32"] = s.astype(np.float32)
    m = get_model(H, w, "fix16b")
    got = run(m, x, s)
    assert_parity(got, ref, w, s)
    assert got["final_target"][0].tolist() == [0] * H
    assert got["final_target"][1].tolist() == [3] * H
    assert np.isfinite(got["logits"]).all() and np.isfinite(got["probs"]).all()


def test_large_batch_properties_h50():
    """BASELINE config 2 shape (H=50), 8192 windows: per-window results do not
    depend on the batch (bitwise), and a random subset matches the oracle."""
    H = 50
    rng = np.random.Generator(np.random.PCG64(5))
    w = W.synth_weights(H, seed=0)
    x, s = c2(rng, 8192, H)
    m = get_model(H, w, "syn50L")
    full = run(m, x, s)
    part = run(m, x[1000:1100], s[1000:1100])
    for k in part:
        assert np.array_equal(full[k][1000:1100], part[k]), k
    idx = rng.choice(8192, size=128, replace=False)
    ref = O.forward(w, x[idx], s[idx])
    ref["sched32"] = s[idx].astype(np.float32)
    sub = {k: v[idx] for k, v in full.items()}
    assert_parity(sub, ref, w, s[idx], check_latent=False)
    assert np.array_equal(full["final_target"], O.first_argmax_rows(s.astype(np.float32)))


def _c2_torch(n, H, seed, device="cuda"):
    """The C2 input distribution generated on the device (full sizes would take
    minutes to build and copy from numpy)."""
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.rand((n, 3, 3 * H), generator=g, device=device) * 0.6
    spike = torch.rand(x.shape, generator=g, device=device) < 0.02
    x = torch.where(spike, 0.9 + 0.4 * torch.rand(x.shape, generator=g, device=device), x)
    s = torch.zeros((n, H, H), device=device)
    s.scatter_(2, torch.randint(0, H, (n, H, 1), generator=g, device=device), 1.0)
    return x.contiguous(), s


@pytest.mark.timeout(900)
@pytest.mark.parametrize("seed_off", [0, 970])
@pytest.mark.parametrize("H,B", [(50, 65536), (16, 262144)])
def test_full_size_census(H, B, seed_off):
    """BASELINE sizes: C2 (H=50, 65,536 windows) and one whole C5 launch (H=16,
    262,144 cell-windows), every window compared with the fp64 oracle
    (tests/census.py over a CPU worker pool).

    - continuous outputs within the north-star tolerance for every window
      (logits / protos rtol 1e-4; probs wherever the anomaly flags agree);
    - every decision (anomaly flag, any, class, keep, final target, generator
      target) equal to the oracle's unless its fp64 margin lies inside its
      derived fp32 error bound (tests/decision_bounds.py): mismatches outside
      the bound must be 0; in-band counts and mismatches are printed and written
      to gpurun_out/census_h{H}_b{B}.json;
    - windows at the start, middle and ragged tail give bitwise the same results
      when run alone; keep / any / class consistent with probs and logits."""
    import json
    import os

    from preganplus_amd.model import to_numpy
    from tests import census as CE
    from tests import decision_bounds as DB
    if H == 16:
        w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    else:
        w = W.synth_weights(H, seed=0)
    m = get_model(H, w, f"full{H}")
    # two input draws per size in the suite (seed_off); PGP_CENSUS_SEED overrides
    # the first for one-off runs over other draws
    seed = int(os.environ.get("PGP_CENSUS_SEED", 31 + H)) + seed_off
    x, s = _c2_torch(B, H, seed=seed)
    full = to_numpy(m.forward(x, s))
    torch.cuda.synchronize()
    for lo, hi in ((0, 64), (B // 2 - 7, B // 2 + 50), (B - 45, B)):
        part = to_numpy(m.forward(x[lo:hi].contiguous(), s[lo:hi].contiguous()))
        torch.cuda.synchronize()
        for k in part:
            assert np.array_equal(full[k][lo:hi], part[k]), (k, lo, hi)
    assert np.isfinite(full["logits"]).all() and np.isfinite(full["probs"]).all()
    np.testing.assert_allclose(full["probs"].sum(axis=1), 1.0, rtol=0, atol=2e-6)
    anom = full["logits"][..., 1] > full["logits"][..., 0]
    assert np.array_equal(full["any"], anom.any(axis=1))
    assert np.array_equal(full["cls"] < 0, ~anom)  # a class exactly where a host is flagged
    x32 = x.cpu().numpy()
    sidx = s.argmax(dim=-1).cpu().numpy()
    del x, s
    st, worst = CE.run(w, x32, sidx, full, log=print)
    res = {"H": H, "windows": B, "seed": seed, "census": st, "worst_error_over_tolerance": worst}
    print("CENSUS", json.dumps(res))
    os.makedirs("gpurun_out", exist_ok=True)
    tag = "" if "PGP_CENSUS_SEED" not in os.environ and seed_off == 0 else f"_s{seed}"
    with open(f"gpurun_out/census_h{H}_b{B}{tag}.json", "w") as f:
        json.dump(res, f, indent=1)
    assert worst["logits"] <= 1.0 and worst["protos"] <= 1.0 and worst["probs"] <= 1.0, worst
    assert not DB.violations(st), st
    assert st["windows"] == B
    # the rigorous bounds leave a small unverifiable fraction: keep it < 0.1 %
    for kind in ("anomaly", "class", "keep", "gen"):
        assert st[kind]["in_band"] <= 1e-3 * max(st[kind]["n"], 1), (kind, st[kind])
    # observed mismatch counts, asserted (PreGANPlus.py:87,99, Stats.py:164-166): every
    # census launch so far has had 0-2 generator-target near-ties (fp64 margin below
    # what fp32 resolves, inside the bound) and no other differing decision
    for kind in ("anomaly", "any", "class", "keep", "final"):
        assert st[kind]["mismatch"] == 0, (kind, st[kind])
    assert st["gen"]["mismatch"] <= 8, st["gen"]
