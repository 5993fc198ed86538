"""Per-decision fp32 error bounds for decision parity — TEST INFRASTRUCTURE.

The HIP path computes in fp32, the reference (and the oracle) in fp64.  The
north star asks for bit-exact decisions; a decision can only differ where the
fp64 margin of that decision lies within what fp32 rounding can move it.  Each
bound here is derived per decision from the magnitudes of its own operands
(first-order forward error analysis, Higham, "Accuracy and Stability of
Numerical Algorithms" §3.1: |fl(sum_i w_i x_i) - sum_i w_i x_i| <=
gamma_n sum_i |w_i x_i|, gamma_n = n u / (1 - n u), u = 2^-24; an addition with
an exactly-zero operand is exact, so n counts the nonzero terms in any
summation order, MFMA blocking included).  Decision kinds (reference lines):

anomaly  ``PreGANPlus.py:120-122``: l1 > l0 on the kernel's OUTPUT logits.  The
         logits are asserted within the north-star tolerance, so a flip needs
         |l1 - l0|_ref <= env(l0) + env(l1), env(v) = ATOL + RTOL |v|.
keep     ``PreGANPlus.py:87``: p0 > p1 on the kernel's output probabilities:
         the same envelope rule on |p0 - p1|_ref.
class    ``utils.py:107-108``: first-argmin_k mean((emb - P_k)^2) on the
         kernel's output embedding.  The distance error is bounded from the
         OBSERVED |emb_gpu - emb_ref|, the fp32 rounding of the prototypes and
         the 3 roundings of the distance itself (gamma_4).
gen      ``Stats.py:164-166``: first-argmax of ns = s + 4 tanh(W2 (W1 [emb; s]
         + b1) + b2).  ns is not a kernel output, so its error is propagated
         through the Gen MLP: the observed emb error and the schedule's fp32
         rounding through |W1|, gamma_(nnz+2) per hidden unit (nnz nonzero
         input terms + bias, +1 product rounding, +1 weight rounding), then
         |W2| and gamma_66 (64 terms + bias + weight rounding), tanh_fast's
         absolute error EPS_TANH, and the final rounding of s + 4 t.
final    ``PreGANPlus.py:99``: first-argmax of the fp32 input schedule: exact.

``compare`` returns the census: per kind the number of decisions, how many
sit inside their bound ("in band"), how many differ, and how many differ
OUTSIDE their bound (must be 0), plus the smallest slack among in-band
mismatches.  Windows whose anomaly flags differ (necessarily in band) are
excluded from the downstream kinds, whose inputs they change.
"""
from __future__ import annotations

import numpy as np

RTOL = 1e-4          # north star: logits within rtol 1e-4 in fp32
ATOL_LOGIT = 1e-5    # for logits that are ~0 (relative error undefined)
ATOL_PROB = 1e-6
U = 2.0 ** -24       # fp32 unit roundoff
# tanh_fast = 1 - 2 rcp(exp2(2 x log2 e) + 1) on v_exp_f32 / v_rcp_f32
# (pgp_device.hpp): argument rounding <= 0.45u after the sech^2 damping, exp2 and
# rcp ~1 ulp each (x 0.5 and x 2 through the formula), e + 1 and 1 - 2r one
# rounding each: ~7u absolute; 16u is taken.
EPS_TANH = 16 * U
REF_EPS = 1e-12      # the fp64 reference's own rounding, absolute (negligible)


def gamma(n):
    n = np.asarray(n, dtype=np.float64)
    return n * U / (1.0 - n * U)


def envelope(v, atol):
    return atol + RTOL * np.abs(v)


def _first_argext_slack(v, bound, largest):
    """v [..., n] fp64 reference values, bound [..., n] per-entry error bounds.
    Returns (first arg-extremum index, slack) where slack = min over k != k* of
    (|v_k* - v_k| - bound_k* - bound_k): <= 0 means some other entry can overtake
    the reference's choice under the bounds (the decision is in band)."""
    k = np.argmax(v, axis=-1) if largest else np.argmin(v, axis=-1)
    vk = np.take_along_axis(v, k[..., None], axis=-1)
    bk = np.take_along_axis(bound, k[..., None], axis=-1)
    gap = (vk - v) if largest else (v - vk)
    slack = gap - bound - bk - REF_EPS
    np.put_along_axis(slack, k[..., None], np.inf, axis=-1)
    return k, slack.min(axis=-1)


def gen_ns_bound(gw, emb_ref, emb_gpu, sched):
    """Bound on |ns_gpu - ns_ref| per entry [B,C,H] (Gen_*: models.py:118-133,
    258-273; K3 pgp_gan.hip phases 1-3).  emb_* [B,H,2], sched [B,C,H] fp64 (the
    GPU reads its fp32 rounding)."""
    W1 = np.asarray(gw["delta.0.weight"], np.float64)
    b1 = np.asarray(gw["delta.0.bias"], np.float64)
    W2 = np.asarray(gw["delta.2.weight"], np.float64)
    b2 = np.asarray(gw["delta.2.bias"], np.float64)
    B, C, H = sched.shape
    s64 = np.asarray(sched, np.float64)
    s32 = s64.astype(np.float32).astype(np.float64)
    x = np.concatenate([emb_ref.reshape(B, -1), s64.reshape(B, -1)], axis=1)
    dx = np.concatenate([np.abs(emb_gpu.astype(np.float64) - emb_ref).reshape(B, -1),
                         np.abs(s32 - s64).reshape(B, -1)], axis=1)
    aW1, aW2 = np.abs(W1), np.abs(W2)
    nnz = np.count_nonzero(x, axis=1) + 1                      # + bias
    h = x @ W1.T + b1
    dh = dx @ aW1.T + gamma(nnz + 2)[:, None] * (np.abs(x) @ aW1.T + np.abs(b1))
    g = h @ W2.T + b2
    dg = dh @ aW2.T + gamma(W2.shape[1] + 2) * (np.abs(h) @ aW2.T + np.abs(b2))
    ns = s64.reshape(B, -1) + 4.0 * np.tanh(g)
    # tanh is 1-Lipschitz; 4 t is an exact scaling; s + 4t rounds once
    dns = 4.0 * (dg + EPS_TANH) + U * np.abs(ns) + np.abs(s32 - s64).reshape(B, -1)
    return dns.reshape(B, C, H)


def class_dist_bound(emb_ref, emb_gpu, prototypes):
    """Reference distances [B,H,K] (utils.py:107: torch.mean((emb - P_k)^2)) and
    a bound on the GPU's fp32 distance error per entry (pgp_decoder.hip
    epilogue: (d0 d0 + d1 d1) * 0.5 with d = e - P32)."""
    P = np.asarray(prototypes, np.float64)
    P32 = P.astype(np.float32).astype(np.float64)
    d = emb_ref[:, :, None, :] - P[None, None]                    # [B,H,K,2]
    dist = (d ** 2).mean(-1)
    de = np.abs(emb_gpu.astype(np.float64) - emb_ref)[:, :, None, :] + np.abs(P32 - P)[None, None]
    ddist = (2.0 * np.abs(d) * de + de ** 2).mean(-1) + gamma(4) * dist
    return dist, ddist


def compare(got, ref, weights, sched, prototypes=None):
    """Decision census of HIP outputs ``got`` against fp64 ``ref`` (numpy).

    got: logits/protos [B,H,2], probs [B,2], cls [B,H], any/keep [B],
    final_target/gen_target [B,C]; ref: the same keys from the reference or
    the oracle plus 'new_sched' [B,C,H].  weights: dict with 'gen' (and
    'prototypes' unless ``prototypes`` is given).  sched [B,C,H] fp64."""
    P = np.asarray(weights["prototypes"] if prototypes is None else prototypes, np.float64)
    st = {}
    lr, lg = np.asarray(ref["logits"], np.float64), got["logits"]
    # ---- anomaly flags (per host) ----
    ref_an, got_an = lr[..., 1] > lr[..., 0], lg[..., 1] > lg[..., 0]
    band = np.abs(lr[..., 1] - lr[..., 0]) <= envelope(lr[..., 0], ATOL_LOGIT) + envelope(lr[..., 1], ATOL_LOGIT)
    mis = got_an != ref_an
    st["anomaly"] = _kind(mis, band)
    win_ok = ~mis.any(axis=1)
    st["windows"] = int(lr.shape[0])
    st["windows_excluded"] = int((~win_ok).sum())
    st["any"] = _kind(got["any"][win_ok] != ref["any"][win_ok], np.zeros(int(win_ok.sum()), bool))
    # ---- classes: hosts flagged on both sides ----
    emb_ref = np.where(ref_an[..., None], np.asarray(ref["protos"], np.float64), 0.0)
    emb_gpu = np.where(got_an[..., None], got["protos"].astype(np.float64), 0.0)
    sel = win_ok[:, None] & ref_an
    dist, ddist = class_dist_bound(emb_ref[sel][None], emb_gpu[sel][None], P)
    k_ref, slack = _first_argext_slack(dist[0], ddist[0], largest=False)
    zero = np.all(emb_ref[sel] == 0, axis=-1)
    k_ref = np.where(zero, -1, k_ref)
    st["class"] = _kind(got["cls"][sel] != k_ref, slack <= 0, slack)
    _record_cases(st["class"], got["cls"][sel], k_ref, dist[0], ddist[0], largest=False)
    st["class_ref_consistent"] = bool(np.array_equal(k_ref, np.asarray(ref["cls"])[sel]))
    nsel = win_ok[:, None] & ~ref_an
    st["class_unflagged"] = _kind(got["cls"][nsel] != -1, np.zeros(int(nsel.sum()), bool))
    # ---- discriminator gate ----
    pr = np.asarray(ref["probs"], np.float64)[win_ok]
    kband = np.abs(pr[:, 0] - pr[:, 1]) <= envelope(pr[:, 0], ATOL_PROB) + envelope(pr[:, 1], ATOL_PROB)
    st["keep"] = _kind(got["keep"][win_ok] != ref["keep"][win_ok], kband)
    st["keep_consistent"] = bool(np.array_equal(got["keep"], got["probs"][:, 0] > got["probs"][:, 1]))
    # ---- final targets: exact ----
    s32 = np.asarray(sched, np.float64).astype(np.float32)
    st["final"] = _kind(got["final_target"] != np.argmax(s32, axis=-1), np.zeros(got["final_target"].shape, bool))
    # ---- generator proposal ----
    sw = np.asarray(sched, np.float64)[win_ok]
    dns = gen_ns_bound(weights["gen"], emb_ref[win_ok], emb_gpu[win_ok], sw)
    ns = np.asarray(ref["new_sched"], np.float64)[win_ok]
    g_ref, gslack = _first_argext_slack(ns, dns, largest=True)
    st["gen_ref_consistent"] = bool(np.array_equal(g_ref, np.asarray(ref["gen_target"])[win_ok]))
    st["gen"] = _kind(got["gen_target"][win_ok] != g_ref, gslack <= 0, gslack)
    _record_cases(st["gen"], got["gen_target"][win_ok], g_ref, ns, dns, largest=True)
    st["gen"]["bound_median"] = float(np.median(dns)) if dns.size else 0.0
    return st


def _kind(mis, band, slack=None):
    mis, band = np.asarray(mis, bool), np.asarray(band, bool)
    d = {"n": int(mis.size), "in_band": int(band.sum()), "mismatch": int(mis.sum()),
         "mismatch_outside_band": int((mis & ~band).sum())}
    if slack is not None and (mis & band).any():
        d["in_band_mismatch_min_slack"] = float(np.asarray(slack)[mis & band].min())
    return d


def _record_cases(d, got_k, ref_k, v, bound, largest, limit=16):
    """For decisions that differ: the fp64 margin between the reference's choice
    and the GPU's, and the bound of the two entries (first ``limit`` cases)."""
    idx = np.argwhere((got_k != ref_k) & (got_k >= 0) & (ref_k >= 0))[:limit]
    cases = []
    for ix in idx:
        ix = tuple(ix)
        a, b = int(ref_k[ix]), int(got_k[ix])
        gap = (v[ix + (a,)] - v[ix + (b,)]) * (1 if largest else -1)
        cases.append({"margin": float(gap), "bound": float(bound[ix + (a,)] + bound[ix + (b,)])})
    if cases:
        d["cases"] = cases


def violations(st):
    """Decisions that differ outside their bound, plus internal inconsistencies."""
    bad = {k: v["mismatch_outside_band"] for k, v in st.items()
           if isinstance(v, dict) and v.get("mismatch_outside_band", 0)}
    for k in ("class_ref_consistent", "gen_ref_consistent", "keep_consistent"):
        if k in st and not st[k]:
            bad[k] = 1
    return bad


def merge(stats):
    """Sum census dicts over chunks."""
    out = {}
    for st in stats:
        for k, v in st.items():
            if isinstance(v, dict):
                o = out.setdefault(k, {})
                for kk, vv in v.items():
                    if kk.endswith("min_slack"):
                        o[kk] = min(o.get(kk, np.inf), vv)
                    elif kk == "cases":
                        o[kk] = (o.get(kk, []) + vv)[:64]
                    elif kk == "bound_median":
                        o["bound_median_max"] = max(o.get("bound_median_max", 0.0), vv)
                    else:
                        o[kk] = o.get(kk, 0) + vv
            elif isinstance(v, bool):
                out[k] = out.get(k, True) and v
            else:
                out[k] = out.get(k, 0) + v
    return out
