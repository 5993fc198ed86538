"""Shared parity helpers: tolerances and margin-aware decision checks.

Tolerance (BASELINE.json north_star): logits within rtol 1e-4 in fp32; decisions
bit-exact.  The reference computes in fp64, the HIP path in fp32, so a decision
may only differ where the fp64 reference itself sits in a near-tie band; every
such case is counted and the band is asserted tiny (SURVEY.md §7 hard parts).
"""
import numpy as np

from oracle import pregan_oracle as O

RTOL = 1e-4
ATOL_LOGIT = 1e-5     # for logits that are ~0 (relative error undefined)
ATOL_PROB = 1e-6
BAND = 2e-5           # near-tie band on decision margins (fp32 vs fp64 noise ~1e-6)


def _top2_gap(m):
    s = np.sort(m, axis=-1)
    return s[..., -1] - s[..., -2]


def assert_parity(got, ref, prototypes, check_latent=True, band=BAND):
    """got: HIP outputs (numpy); ref: fp64 reference/oracle outputs."""
    n = ref["latent"].shape[0] if (check_latent and "latent" in ref and got.get("latent") is not None) else 0
    if n:
        np.testing.assert_allclose(got["latent"][:n], ref["latent"][:n], rtol=RTOL, atol=1e-4,
                                   err_msg="latent")
    np.testing.assert_allclose(got["logits"], ref["logits"], rtol=RTOL, atol=ATOL_LOGIT, err_msg="logits")
    np.testing.assert_allclose(got["protos"], ref["protos"], rtol=RTOL, atol=ATOL_PROB, err_msg="protos")
    np.testing.assert_allclose(got["probs"], ref["probs"], rtol=RTOL, atol=ATOL_PROB, err_msg="probs")

    stats = {}
    # anomaly flags per host -> any
    l = ref["logits"]
    ref_anom = l[..., 1] > l[..., 0]
    got_anom = got["logits"][..., 1] > got["logits"][..., 0]
    am = np.abs(l[..., 1] - l[..., 0])
    bad = (got_anom != ref_anom) & (am >= band)
    assert not bad.any(), f"anomaly flags differ outside the near-tie band: {bad.sum()}"
    stats["anom_mismatch_in_band"] = int((got_anom != ref_anom).sum())
    host_ok = got_anom == ref_anom
    win_ok = host_ok.all(axis=1)
    assert np.array_equal(got["any"][win_ok], ref["any"][win_ok]), "any_anom differs"
    # classes where the anomaly flag agrees
    cm = O.class_margin(np.where(ref_anom[..., None], ref["protos"], 0.0), prototypes)
    cbad = (got["cls"] != ref["cls"]) & host_ok & (cm >= band)
    assert not cbad.any(), f"classes differ outside the band: {cbad.sum()}"
    stats["cls_mismatch_in_band"] = int(((got["cls"] != ref["cls"]) & host_ok).sum())
    # discriminator gate: only meaningful where the embeddings agree
    pm = np.abs(ref["probs"][:, 0] - ref["probs"][:, 1])
    kbad = (got["keep"] != ref["keep"]) & win_ok & (pm >= band)
    assert not kbad.any(), f"keep_orig differs outside the band: {kbad.sum()}"
    stats["keep_mismatch_in_band"] = int(((got["keep"] != ref["keep"]) & win_ok).sum())
    # final target: argmax of the (fp32-rounded) input schedule
    sched32 = ref["sched32"] if "sched32" in ref else None
    if sched32 is not None:
        assert np.array_equal(got["final_target"], O.first_argmax_rows(sched32)), "final_target"
    else:
        assert np.array_equal(got["final_target"], ref["final_target"]), "final_target"
    # generator proposal
    gm = _top2_gap(ref["new_sched"])
    gbad = (got["gen_target"] != ref["gen_target"]) & win_ok[:, None] & (gm >= band)
    assert not gbad.any(), f"gen_target differs outside the band: {gbad.sum()}"
    stats["gen_mismatch_in_band"] = int(((got["gen_target"] != ref["gen_target"]) & win_ok[:, None]).sum())
    return stats
