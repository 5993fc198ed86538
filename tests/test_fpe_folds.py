"""The algebraic folds K4 (pgp_fpe.hip) and its packer (pgp_pack.cpp pack_fpe_t)
rely on, restated in fp64 numpy and checked against the FPE oracle on CPU:
  * GAT node mean through the per-branch factorised edge softmax, as the
    kernel evaluates it: E1 sum_pos A + E2 (sum C - sum_pos C),
  * the node mean is rank 3 (Wfc / H times the r-weighted raw features), so
    each MHA token is c_w = P u_w with u_w = [GRU state; g_w],
  * MHA scores as u_s^T M6 u_t + beta6.u_t (s-only terms cancel),
  * V / out_proj / encoder / decoders folded into one [4H x 18] affine map.
The GPU parity test then checks the fp32 kernel itself (tests/test_gpu_fpe.py)."""
import numpy as np

from oracle import pregan_oracle as O
from preganplus_amd import weights as W

LOG2E = 1.4426950408889634


def _fold(fw, H=16):
    E, L = H + 3, 10
    fc = fw["gat.layer1.heads.0.fc.weight"]
    P = np.zeros((E, 6))
    P[:3, :3] = np.eye(3)
    P[3:, 3:] = fc / H
    Wq, Wk, Wv = np.split(fw["mha.in_proj_weight"], 3)
    bq, bk, bv = np.split(fw["mha.in_proj_bias"], 3)
    sc = LOG2E / np.sqrt(E)
    M6 = P.T @ (Wq.T @ Wk) @ P * sc
    beta6 = P.T @ (Wk.T @ bq) * sc
    A = fw["mha.out_proj.weight"] @ Wv @ P                                   # [E,6]
    a0 = fw["mha.out_proj.weight"] @ bv + fw["mha.out_proj.bias"]
    We = fw["encoder.0.weight"].reshape(H * L, 3, E)
    WA = np.einsum("rsf,fk->rsk", We, A).reshape(H, L, 18)
    bA = (fw["encoder.0.bias"] + np.einsum("rsf,f->r", We, a0)).reshape(H, L)
    D = np.concatenate([fw["anomaly_decoder.0.weight"], fw["prototype_decoder.0.weight"]])   # [4,L]
    bd = np.concatenate([fw["anomaly_decoder.0.bias"], fw["prototype_decoder.0.bias"]])
    W6 = np.einsum("ql,hlk->hqk", D, WA).reshape(4 * H, 18)
    b2 = (np.einsum("ql,hl->hq", D, bA) + bd).reshape(4 * H)
    att = fw["gat.layer1.heads.0.attn_fc.weight"][0]
    u, v = fc.T @ att[:H] * LOG2E, fc.T @ att[H:] * LOG2E
    return M6, beta6, W6, b2, u, v


def _kernel_restated(fw, x, h0, H=16):
    M6, beta6, W6, b2, u, v = _fold(fw, H)
    B = x.shape[0]
    h = h0.copy()
    us = []
    for w in range(3):
        xw = x[:, w]
        gi = xw @ fw["gru.weight_ih_l0"].T
        gh = h @ fw["gru.weight_hh_l0"].T
        bi, bh = fw["gru.bias_ih_l0"], fw["gru.bias_hh_l0"]
        r = 1 / (1 + np.exp(-(gi[:, :3] + gh[:, :3] + bi[:3] + bh[:3])))
        z = 1 / (1 + np.exp(-(gi[:, 3:6] + gh[:, 3:6] + bi[3:6] + bh[3:6])))
        n = np.tanh(gi[:, 6:] + bi[6:] + r * (gh[:, 6:] + bh[6:]))
        h = (1 - z) * n + z * h
        xn = xw.reshape(B, H, 3)
        s, t = xn @ u, xn @ v
        smax, tmax = s.max(1, keepdims=True), t.max(1, keepdims=True)
        mraw = smax + tmax
        m = np.maximum(mraw, 0.01 * mraw)
        k1, k2 = 2 ** (mraw - m), 2 ** (0.01 * mraw - m)
        Aj, Cj = 2 ** (t - tmax), 2 ** (0.01 * (t - tmax))
        pos = (s[:, :, None] + t[:, None, :]) > 0                             # [B,i,j]
        sa = (pos * Aj[:, None, :]).sum(-1)
        sc_pos = (pos * Cj[:, None, :]).sum(-1)
        rr = 2 ** (s - smax) * k1 * sa + 2 ** (0.01 * (s - smax)) * k2 * (Cj.sum(1, keepdims=True) - sc_pos)
        g = np.einsum("bi,bid->bd", rr, xn) / rr.sum(1, keepdims=True)
        us.append(np.concatenate([h, g], 1))
    uu = np.stack(us, 1)                                                       # [B,3,6]
    sc = np.einsum("bse,ef,btf->bst", uu, M6, uu) + (uu @ beta6)[:, None, :]
    p = 2 ** (sc - sc.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    ub = np.einsum("bst,bte->bse", p, uu).reshape(B, -1)
    o = (ub @ W6.T + b2).reshape(B, H, 4)
    a = np.exp(o[..., :2] - o[..., :2].max(-1, keepdims=True))
    return a / a.sum(-1, keepdims=True), 1 / (1 + np.exp(-o[..., 2:]))


def test_fpe_folds_match_oracle_shipped_weights():
    z = np.load("tests/golden/fpe_h16.npz")
    w, _ = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    probs, protos = _kernel_restated(w["fpe"], z["windows"], z["h0"])
    np.testing.assert_allclose(probs, z["probs"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(protos, z["protos"], rtol=0, atol=1e-12)


def test_fpe_folds_match_oracle_synthetic():
    w = W.synth_fpe_weights(16, seed=7)
    rng = np.random.Generator(np.random.PCG64(8))
    x = rng.uniform(-1, 2, size=(64, 3, 48))
    h0 = rng.standard_normal((64, 3))
    probs, protos = _kernel_restated(w["fpe"], x, h0)
    ref_p, ref_q = O.fpe_forward(w["fpe"], x, h0)
    np.testing.assert_allclose(probs, ref_p, rtol=0, atol=1e-12)
    np.testing.assert_allclose(protos, ref_q, rtol=0, atol=1e-12)


def test_fpe_folds_match_reference_h50():
    """The same folds at 50 hosts against the reference-generated fixture
    (FPE_16 code at n_hosts=50, tests/golden/make_golden_fpe50.py)."""
    from tests.test_oracle_golden import fpe50_weights
    z = np.load("tests/golden/fpe_h50.npz")
    for part in ("", "b/"):
        w = fpe50_weights(z, part)
        probs, protos = _kernel_restated(w["fpe"], z[f"{part}windows"], z[f"{part}h0"], H=50)
        np.testing.assert_allclose(probs, z[f"{part}probs"], rtol=0, atol=1e-12)
        np.testing.assert_allclose(protos, z[f"{part}protos"], rtol=0, atol=1e-12)
