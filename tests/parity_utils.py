"""Shared parity helpers: tolerances and bound-aware decision checks.

Tolerance (BASELINE.json north_star): logits within rtol 1e-4 in fp32; decisions
bit-exact.  The reference computes in fp64, the HIP path in fp32, so a decision
may only differ where its fp64 margin lies inside a per-decision fp32 error
bound derived from the magnitudes involved (tests/decision_bounds.py); every
such case is counted, and any difference outside its bound fails.
"""
import numpy as np

from tests import decision_bounds as DB
from tests.decision_bounds import ATOL_LOGIT, ATOL_PROB, RTOL  # noqa: F401  (re-exported)


def assert_parity(got, ref, weights, sched, check_latent=True, exact=False):
    """got: HIP outputs (numpy); ref: fp64 reference/oracle outputs (with
    'new_sched'); weights: dict with 'gen' and 'prototypes'; sched [B,C,H] the
    schedule the reference saw (fp64).  exact=True: every decision must match
    (the committed reference fixtures).  Returns the decision census."""
    n = ref["latent"].shape[0] if (check_latent and "latent" in ref and got.get("latent") is not None) else 0
    if n:
        np.testing.assert_allclose(got["latent"][:n], ref["latent"][:n], rtol=RTOL, atol=1e-4,
                                   err_msg="latent")
    st = DB.compare(got, ref, weights, np.asarray(sched, np.float64))
    ok = np.ones(got["logits"].shape[0], bool)
    if st["windows_excluded"]:   # an in-band anomaly flip changes that window's GAN inputs
        lr = ref["logits"]
        ok = ((got["logits"][..., 1] > got["logits"][..., 0]) == (lr[..., 1] > lr[..., 0])).all(axis=1)
    np.testing.assert_allclose(got["logits"], ref["logits"], rtol=RTOL, atol=ATOL_LOGIT, err_msg="logits")
    np.testing.assert_allclose(got["protos"], ref["protos"], rtol=RTOL, atol=ATOL_PROB, err_msg="protos")
    np.testing.assert_allclose(got["probs"][ok], ref["probs"][ok], rtol=RTOL, atol=ATOL_PROB, err_msg="probs")
    bad = DB.violations(st)
    assert not bad, f"decisions differ outside their fp32 bound: {bad}\n{st}"
    if exact:
        mism = {k: v["mismatch"] for k, v in st.items() if isinstance(v, dict) and v["mismatch"]}
        assert not mism, f"decisions differ on the reference fixtures: {mism}"
    return st
