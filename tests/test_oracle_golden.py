"""Pin the numpy oracle against fixtures produced by the reference itself
(tests/golden/make_golden.py: reference modules, eval mode, fp64)."""
import numpy as np
import pytest

from oracle import pregan_oracle as O
from preganplus_amd import weights as W

GOLD = "tests/golden"


def _weights(H, z):
    if H == 16:
        w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    else:
        w = W.synth_weights(H, int(z["weights_seed"]))
        assert W.weights_checksum(w) == float(z["weights_checksum"])
    return w


@pytest.mark.parametrize("H", [16, 50])
def test_oracle_fp64_matches_reference(H):
    z = np.load(f"{GOLD}/fwd_h{H}.npz")
    w = _weights(H, z)
    out = O.forward(w, z["windows"], z["sched"])
    n = z["latent"].shape[0]
    np.testing.assert_allclose(out["latent"][:n], z["latent"], rtol=0, atol=1e-12)
    for k in ["logits", "protos", "emb", "new_sched", "probs"]:
        np.testing.assert_allclose(out[k], z[k], rtol=0, atol=1e-12, err_msg=k)
    for k in ["cls", "any", "keep", "final_target", "gen_target"]:
        np.testing.assert_array_equal(out[k], z[k], err_msg=k)


@pytest.mark.parametrize("H", [16, 50])
def test_oracle_fp32_within_north_star_tolerance(H):
    """fp32 restatement vs the fp64 reference: logits within rtol 1e-4 (+ a small
    atol for logits near 0) and identical decisions on these fixtures."""
    z = np.load(f"{GOLD}/fwd_h{H}.npz")
    w = _weights(H, z)
    out = O.forward(w, z["windows"], z["sched"], dtype=np.float32)
    np.testing.assert_allclose(out["logits"], z["logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["protos"], z["protos"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(out["probs"], z["probs"], rtol=1e-4, atol=1e-6)
    for k in ["cls", "any", "keep", "final_target", "gen_target"]:
        np.testing.assert_array_equal(out[k], z[k], err_msg=k)


def test_inference_window_drops_newest_row():
    """PreGANPlus.py:107-112: window = rows [t-2, t-2, t-1] of the normalised series."""
    ts = np.arange(5 * 6, dtype=np.float64).reshape(5, 6) + 1.0
    train = np.ones((3, 6)) * 100.0
    win = O.inference_window(ts, train)
    norm = ts / (100.0 + 1e-8)
    np.testing.assert_allclose(win, np.stack([norm[2], norm[2], norm[3]]))


def test_real_fixture_windows_follow_run_encoder():
    z = np.load(f"{GOLD}/fwd_h16.npz")
    _, extra = W.load_npz("preganplus_amd/data/simulator_16.npz")
    series = extra["train_time_data"]
    for i in (0, 10, 198):
        tt = i + 3
        np.testing.assert_allclose(z["windows"][i], O.inference_window(series[:tt], series),
                                   rtol=0, atol=0)


def test_ties_break_to_first_index():
    logits = np.array([[[1.0, 1.0], [0.0, 2.0]]])
    protos = np.array([[[0.5, 0.5], [0.25, 0.75]]])
    P = np.array([[0.25, 0.75], [0.25, 0.75], [0.0, 0.0]])
    anom, emb, cls, anyb = O.classify(logits, protos, P)
    assert anom.tolist() == [[False, True]]
    assert cls.tolist() == [[-1, 0]]
    assert anyb.tolist() == [True]
    s = np.array([[[0.5, 0.5, 0.1]]])
    assert O.first_argmax_rows(s).tolist() == [[0]]


def test_fpe_oracle_matches_reference():
    """PreGAN's FPE_16 path (config C4) vs the reference modules (make_golden_fpe.py),
    shipped checkpoints/ weights, GRU h0 injected from the recorded draw."""
    z = np.load(f"{GOLD}/fpe_h16.npz")
    w, _ = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    assert "fpe" in w and w["prototypes"].shape == (W.FPE_PROTOS, 2)
    out = O.forward_fpe(w, z["windows"], z["h0"], z["sched"])
    for k in ["probs", "protos", "emb", "new_sched", "gprobs"]:
        np.testing.assert_allclose(out[k], z[k], rtol=0, atol=1e-12, err_msg=k)
    for k in ["cls", "any", "keep", "final_target", "gen_target"]:
        np.testing.assert_array_equal(out[k], z[k], err_msg=k)
    out32 = O.forward_fpe(w, z["windows"], z["h0"], z["sched"], dtype=np.float32)
    np.testing.assert_allclose(out32["probs"], z["probs"], rtol=1e-4, atol=1e-6)
    np.testing.assert_array_equal(out32["cls"], z["cls"])


def test_fpe_blob_layout():
    w, _ = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    blob = W.pack_blob(w, 16)
    assert blob.size == sum(int(np.prod(s)) for _, _, s in W.fpe_blob_layout(16))
    ws = W.synth_fpe_weights(16, 1)
    assert W.pack_blob(ws, 16).size == blob.size


def fpe50_weights(z, part=""):
    """Weights of tests/golden/fpe_h50.npz (make_golden_fpe50.py): seeded
    synth_fpe_weights(50), set "b/" with the anomaly bias moved by +-shift."""
    w = W.synth_fpe_weights(50, int(z["weights_seed"]))
    if part:
        sh = float(z[f"{part}bias_shift"])
        w["fpe"]["anomaly_decoder.0.bias"] = w["fpe"]["anomaly_decoder.0.bias"] + np.array([sh, -sh])
    return w


@pytest.mark.parametrize("part", ["", "b/"])
def test_fpe50_oracle_matches_reference(part):
    """C4 at 50 hosts: the reference FPE_16 class instantiated at n_hosts=50
    (make_golden_fpe50.py; FPE_50 itself raises in the reference) with
    Gen_50/Disc_50.  Set "b/" holds windows without any flagged host."""
    z = np.load(f"{GOLD}/fpe_h50.npz")
    w = fpe50_weights(z, part)
    out = O.forward_fpe(w, z[f"{part}windows"], z[f"{part}h0"], z[f"{part}sched"])
    for k in ["probs", "protos", "emb", "new_sched", "gprobs"]:
        np.testing.assert_allclose(out[k], z[f"{part}{k}"], rtol=0, atol=1e-12, err_msg=k)
    for k in ["cls", "any", "keep", "final_target", "gen_target"]:
        np.testing.assert_array_equal(out[k], z[f"{part}{k}"], err_msg=k)
    out32 = O.forward_fpe(w, z[f"{part}windows"], z[f"{part}h0"], z[f"{part}sched"], dtype=np.float32)
    np.testing.assert_allclose(out32["probs"], z[f"{part}probs"], rtol=1e-4, atol=1e-6)
    np.testing.assert_array_equal(out32["cls"], z[f"{part}cls"])
    if part:
        assert 0 < z["b/any"].sum() < z["b/any"].size   # both run_model branches (PreGAN.py:112-113)


def branches16_weights(z):
    """tests/golden/fwd_h16_branches.npz's weights: the shipped H=16 checkpoints
    with the stored anomaly-decoder and discriminator bias offsets."""
    import copy
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    w = copy.deepcopy(w)
    b = np.array(w["transformer"]["anomaly_decoder.0.bias"], dtype=np.float64)
    b[1::2] -= z["anomaly_bias_shift"]
    w["transformer"]["anomaly_decoder.0.bias"] = b
    db = np.array(w["disc"]["probs.2.bias"], dtype=np.float64)
    db[0] += float(z["disc_bias_shift"])
    w["disc"]["probs.2.bias"] = db
    return w


def test_oracle_matches_reference_both_branches_h16():
    """Both gates of run_model at H=16 (make_golden_branches16.py): windows that
    flag no host (the early return, PreGANPlus.py:125-127) and windows whose
    discriminator keeps the original decision (:87-88), from the reference's
    own modules on the shipped weights with stored bias offsets."""
    z = np.load(f"{GOLD}/fwd_h16_branches.npz")
    w = branches16_weights(z)
    assert 0 < z["any"].sum() < z["any"].size and 0 < z["keep"].sum() < z["keep"].size
    out = O.forward(w, z["windows"], z["sched"])
    for k in ["logits", "protos", "emb", "new_sched", "probs"]:
        np.testing.assert_allclose(out[k], z[k], rtol=0, atol=1e-12, err_msg=k)
    for k in ["cls", "any", "keep", "final_target", "gen_target"]:
        np.testing.assert_array_equal(out[k], z[k], err_msg=k)
