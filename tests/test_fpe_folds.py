"""The algebraic folds K4 (pgp_fpe.hip) and its packer (pgp_pack.cpp pack_fpe_t)
rely on, restated in fp64 numpy and checked against the FPE oracle on CPU:
  * GAT node mean through the per-branch factorised edge softmax,
  * MHA scores as c_s^T M c_t + beta.c_t (s-only terms cancel),
  * V / out_proj / encoder / decoders folded into one [4H x 3E] affine map.
The GPU parity test then checks the fp32 kernel itself (tests/test_gpu_fpe.py)."""
import numpy as np

from oracle import pregan_oracle as O
from preganplus_amd import weights as W

LOG2E = 1.4426950408889634


def _fold(fw, H=16):
    E, L = H + 3, 10
    Wq, Wk, Wv = np.split(fw["mha.in_proj_weight"], 3)
    bq, bk, bv = np.split(fw["mha.in_proj_bias"], 3)
    sc = LOG2E / np.sqrt(E)
    M = Wq.T @ Wk * sc
    beta = Wk.T @ bq * sc
    A = fw["mha.out_proj.weight"] @ Wv
    a0 = fw["mha.out_proj.weight"] @ bv + fw["mha.out_proj.bias"]
    We = fw["encoder.0.weight"].reshape(H * L, 3, E)
    WA = np.einsum("rsf,fe->rse", We, A).reshape(H, L, 3 * E)
    bA = (fw["encoder.0.bias"] + np.einsum("rsf,f->r", We, a0)).reshape(H, L)
    D = np.concatenate([fw["anomaly_decoder.0.weight"], fw["prototype_decoder.0.weight"]])   # [4,L]
    bd = np.concatenate([fw["anomaly_decoder.0.bias"], fw["prototype_decoder.0.bias"]])
    W2 = np.einsum("ql,hlk->hqk", D, WA).reshape(4 * H, 3 * E)
    b2 = (np.einsum("ql,hl->hq", D, bA) + bd).reshape(4 * H)
    fc = fw["gat.layer1.heads.0.fc.weight"]
    att = fw["gat.layer1.heads.0.attn_fc.weight"][0]
    u, v = fc.T @ att[:H] * LOG2E, fc.T @ att[H:] * LOG2E
    return M, beta, W2, b2, u, v, fc / H


def _kernel_restated(fw, x, h0, H=16):
    M, beta, W2, b2, u, v, fcH = _fold(fw, H)
    B = x.shape[0]
    h = h0.copy()
    cs = []
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
        pos = t[:, None, :] > -s[:, :, None]                                   # [B,i,j]
        sa = (pos * Aj[:, None, :]).sum(-1)
        scn = (~pos * Cj[:, None, :]).sum(-1)
        rr = 2 ** (s - smax) * k1 * sa + 2 ** (0.01 * (s - smax)) * k2 * scn
        agg = np.einsum("bi,bid->bd", rr, xn) / rr.sum(1, keepdims=True)
        cs.append(np.concatenate([h, agg @ fcH.T], 1))
    c = np.stack(cs, 1)                                                        # [B,3,E]
    sc = np.einsum("bse,ef,btf->bst", c, M, c) + (c @ beta)[:, None, :]
    p = 2 ** (sc - sc.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    ch = np.einsum("bst,bte->bse", p, c).reshape(B, -1)
    o = (ch @ W2.T + b2).reshape(B, H, 4)
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
