"""CPU checks of the decision census (tests/decision_bounds.py): an independent
fp32 implementation (the oracle in fp32) stays inside every derived bound, and
a decision flipped outside its bound is caught."""
import numpy as np
import pytest

from oracle import pregan_oracle as O
from preganplus_amd import weights as W
from tests import decision_bounds as DB


def _inputs(H, B, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 0.6, (B, 3, 3 * H))
    sp = rng.uniform(size=x.shape) < 0.02
    x[sp] = rng.uniform(0.9, 1.3, int(sp.sum()))
    s = np.zeros((B, H, H))
    s[np.arange(B)[:, None], np.arange(H)[None], rng.integers(0, H, (B, H))] = 1.0
    return x, s


def _weights(H):
    return W.load_npz("preganplus_amd/data/simulator_16.npz")[0] if H == 16 else W.synth_weights(H, 0)


@pytest.mark.parametrize("H,B", [(16, 1024), (50, 256)])
def test_fp32_oracle_inside_bounds(H, B):
    w = _weights(H)
    x, s = _inputs(H, B, H)
    ref = O.forward(w, x, s)
    got = {k: np.asarray(v) for k, v in O.forward(w, x.astype(np.float32), s.astype(np.float32),
                                                   dtype=np.float32).items()}
    st = DB.compare(got, ref, w, s)
    assert not DB.violations(st), st
    assert st["gen"]["n"] == B * H and st["final"]["mismatch"] == 0
    assert st["gen_ref_consistent"] and st["class_ref_consistent"]


def test_flips_outside_bound_are_caught():
    H, B = 50, 64
    w = _weights(H)
    x, s = _inputs(H, B, 3)
    ref = O.forward(w, x, s)
    got = {k: np.array(v) for k, v in ref.items()}
    st = DB.compare(got, ref, w, s)
    assert not DB.violations(st) and all(v["mismatch"] == 0 for v in st.values() if isinstance(v, dict))
    # a generator target moved to the row's smallest entry: far outside any bound
    bad = {k: v.copy() for k, v in got.items()}
    bad["gen_target"][5, 7] = int(np.argmin(ref["new_sched"][5, 7]))
    assert DB.violations(DB.compare(bad, ref, w, s)) == {"gen": 1}
    # a class moved to the farthest prototype
    b, h = np.argwhere(ref["cls"] >= 0)[0]
    P = np.asarray(w["prototypes"])
    far = int(np.argmax(((ref["emb"][b, h][None] - P) ** 2).mean(-1)))
    bad = {k: v.copy() for k, v in got.items()}
    bad["cls"][b, h] = far
    assert DB.violations(DB.compare(bad, ref, w, s)) == {"class": 1}
    # a keep flip on a window with a clear discriminator margin
    i = int(np.argmax(np.abs(ref["probs"][:, 0] - ref["probs"][:, 1])))
    bad = {k: v.copy() for k, v in got.items()}
    bad["keep"][i] = ~bad["keep"][i]
    v = DB.violations(DB.compare(bad, ref, w, s))
    assert v.get("keep") == 1 and v.get("keep_consistent") == 1
