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


def test_split_bf16_encoder_vs_fp32_encoder():
    """K2's split-bf16 feed-forward (the default at H = 50: both layers' linear1
    / linear2 as six bf16 MFMAs per fp32 product, pgp_encoder.hip EncS) and its
    fp32-MFMA form: both within the north-star tolerance of the fp64 oracle
    (latent included), the split form no less accurate (worst latent / logit /
    proto error within twice the fp32 form's), every decision equal, and the
    two forms really ran (different bits).  (A repack of the master re-derives
    the split image: tests/test_gpu_repack.py, device repack == host pack at
    H = 50.)"""
    H = 50
    rng = np.random.Generator(np.random.PCG64(350))
    w = W.synth_weights(H, seed=4)
    x, s = c2(rng, 517, H, dense=9)
    ref = O.forward(w, x, s)
    ref["sched32"] = s.astype(np.float32)
    m = get_model(H, w, "esplit50")
    m.encoder_split(True)
    a = run(m, x, s, latent=True)
    m.encoder_split(False)
    b = run(m, x, s, latent=True)
    m.encoder_split(True)
    assert_parity(a, ref, w, s)
    assert_parity(b, ref, w, s)
    for k in ("latent", "logits", "protos"):
        n = ref[k].shape[0]
        ea = np.abs(a[k][:n].astype(np.float64) - ref[k]).max()
        eb = np.abs(b[k][:n].astype(np.float64) - ref[k]).max()
        assert ea <= 2 * eb + 1e-7, (k, ea, eb)
    for k in ("cls", "any", "keep", "final_target", "gen_target"):
        assert np.array_equal(a[k], b[k]), k
    assert not np.array_equal(a["latent"], b["latent"])


@pytest.mark.parametrize("H,dense", [(50, 0), (50, 3000), (16, 0), (16, 3000)])
def test_split_bf16_gan_vs_fp32_gan(H, dense):
    """K3's split-bf16 form (pgp_gansplit.hip; the default at H = 16 and 50 at
    every batch; one-hot schedule blocks in three products, dense ones in six)
    against its fp32-MFMA form on one 65,536-window launch: the first 2,048
    windows (and the dense tail) within tolerance of the fp64 oracle for both
    forms, the split form no less accurate, every decision of the whole launch
    equal except generator targets at fp32 near-ties (in band for both forms),
    and a window's outputs independent of the batch and of its wave's other
    windows (the one-hot shortcut is taken per wave: 16 windows alone and a
    300-window batch on 4-wave workgroups give the same bits)."""
    from preganplus_amd.model import to_numpy
    B = 65536
    w = W.synth_weights(H, seed=5) if H == 50 else W.load_npz("preganplus_amd/data/simulator_16.npz")[0]
    x, s = _c2_torch(B, H, seed=77 + H + dense)
    if dense:
        g = torch.Generator(device="cuda").manual_seed(5)
        s[-dense:] = torch.rand((dense, H, H), generator=g, device="cuda")
    m = get_model(H, w, f"gsplit{H}")
    m.gan_split(True)
    a = to_numpy(m.forward(x, s))
    m.gan_split(False)
    b = to_numpy(m.forward(x, s))
    m.gan_split(True)
    torch.cuda.synchronize()
    for k in ("keep", "final_target", "any", "cls"):
        assert np.array_equal(a[k], b[k]), k
    # generator targets: a container whose two largest new-schedule values tie
    # to within fp32 rounding (4 tanh(.) saturating at 1.0 in fp32 for two
    # hosts, frequent with the shipped H = 16 weights) may break the tie either
    # way in either form; every window where the forms differ must be in band
    # against the fp64 oracle for BOTH forms (assert_parity below), and few
    dw = np.nonzero((a["gen_target"] != b["gen_target"]).any(axis=1))[0]
    assert dw.size <= 16, dw.size
    idx = np.r_[0:2048, B - 256:B]
    idx = np.unique(np.r_[idx, dw])
    xs, ss = x[idx].cpu().numpy().astype(np.float64), s[idx].cpu().numpy().astype(np.float64)
    ref = O.forward(w, xs, ss)
    ref["sched32"] = ss.astype(np.float32)
    sa = {k: v[idx] for k, v in a.items()}
    sb = {k: v[idx] for k, v in b.items()}
    sta = assert_parity(sa, ref, w, ss)
    stb = assert_parity(sb, ref, w, ss)
    assert sta["gen"]["mismatch"] <= dw.size and stb["gen"]["mismatch"] <= dw.size, (sta["gen"], stb["gen"])
    ea = np.abs(sa["probs"].astype(np.float64) - ref["probs"]).max()
    eb = np.abs(sb["probs"].astype(np.float64) - ref["probs"]).max()
    assert ea <= 2 * eb + 1e-7, (ea, eb)
    # the split form runs at every batch (4-wave workgroups below 64 K
    # windows): a window's outputs do not depend on the batch it arrives in
    for lo, hi in ((0, 16), (B // 2 - 5, B // 2 + 300)):
        c = to_numpy(m.forward(x[lo:hi].contiguous(), s[lo:hi].contiguous()))
        for k in ("keep", "final_target", "gen_target", "probs"):
            assert np.array_equal(a[k][lo:hi], c[k]), (k, lo, hi)


@pytest.mark.parametrize("H", [16, 50])
def test_k3_onehot_rebuild_guard(H):
    """K3's split form rebuilds a wave's schedule rows from the 1.0 positions it
    recorded in phase 2 (pgp_gansplit.hip) only when every window of the wave
    has exactly C nonzero values, all 1.0, and every row holds one.  Near-one-hot
    schedules that break one condition each (a row holding two 1.0s next to an
    empty row: the counts still match; a 0.5; a 1.0 + 2^-7; a stray -1.0), each
    in a wave of its own, must take the row reads; legitimate one-hot rows whose
    1.0s sit at the row ends (a lane's values spanning two rows) take the
    rebuild.  Decisions equal to the fp32 form's and within tolerance of the
    oracle on every window of those waves."""
    from preganplus_amd.model import to_numpy
    B = 65536
    w = W.synth_weights(H, seed=5) if H == 50 else W.load_npz("preganplus_amd/data/simulator_16.npz")[0]
    x, s = _c2_torch(B, H, seed=913 + H)
    eye_end = torch.zeros((H, H), device="cuda")
    for r in range(H):
        eye_end[r, H - 1 if r % 2 == 0 else 0] = 1.0
    cases = []
    k = 16 * 37 + 5
    s[k, 3].zero_(); s[k, 3, 0] = s[k, 3, 5] = 1.0; s[k, 7].zero_()      # two in a row, an empty row
    cases.append(k)
    k = 16 * 911 + 0
    s[k, 2] *= 0.5                                                      # a 0.5 (bf16, not 1.0)
    cases.append(k)
    k = 16 * 1500 + 15
    s[k, H - 1] *= 1.0 + 2.0 ** -7                                      # bf16, not 1.0
    cases.append(k)
    k = 16 * 2047 + 9
    s[k, 1, (int(s[k, 1].argmax()) + 1) % H] = -1.0                     # a stray nonzero
    cases.append(k)
    k = 16 * 3000 + 3
    s[k] = eye_end                                                      # 1.0s at row ends
    cases.append(k)
    m = get_model(H, w, f"goh{H}")
    m.gan_split(True)
    a = to_numpy(m.forward(x, s))
    m.gan_split(False)
    b = to_numpy(m.forward(x, s))
    m.gan_split(True)
    torch.cuda.synchronize()
    for key in ("keep", "final_target", "any", "cls"):
        assert np.array_equal(a[key], b[key]), key
    # generator targets may differ only at fp32 near-ties (in band for both
    # forms against the oracle: checked below on those windows)
    dw = np.nonzero((a["gen_target"] != b["gen_target"]).any(axis=1))[0]
    assert dw.size <= 16, dw.size
    idx = np.concatenate([np.arange(16 * (c // 16), 16 * (c // 16) + 16) for c in cases] + [dw])
    xs, ss = x[idx].cpu().numpy().astype(np.float64), s[idx].cpu().numpy().astype(np.float64)
    ref = O.forward(w, xs, ss)
    ref["sched32"] = ss.astype(np.float32)
    assert_parity({key: v[idx] for key, v in a.items()}, ref, w, ss)
    assert_parity({key: v[idx] for key, v in b.items()}, ref, w, ss)


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
