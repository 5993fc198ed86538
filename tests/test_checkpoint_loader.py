"""The checkpoint loader restores what load_model / load_gan restore
(utils.py:60-84): weights, the AdamW state per parameter, the epochs and the
Gen checkpoint's accuracy_list (PreGANPlus.py:32-34).  Checked on the
reference's shipped checkpoints (skipped where /root/reference is absent, e.g.
on the GPU box) against the packaged data files made from the same checkpoints
by the fixture generators (tests/golden/make_golden_train.py, make_golden_fpe.py)."""
import os

import numpy as np
import pytest

from preganplus_amd import weights as W

REF = "/root/reference/recovery/PreGANSrc"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkpoints not present")
@pytest.mark.parametrize("folder,encoder,packaged", [("checkpointsplus", "Transformer", "simulator_16.npz"),
                                                     ("checkpoints", "FPE", "pregan_simulator_16.npz")])
def test_loader_restores_training_state(folder, encoder, packaged):
    w, extra = W.load_reference_checkpoints(os.path.join(REF, folder), "simulator", 16, encoder=encoder,
                                            with_state=True)
    pw, pe = W.load_npz(os.path.join("preganplus_amd", "data", packaged))
    opt = [k for k in pe if k.startswith("opt/")]
    assert opt and all(np.array_equal(extra[k], pe[k]) for k in opt)
    assert int(extra["meta/gen/epoch"]) == int(pe["meta/gen/epoch"]) == 199
    acc = W.accuracy_list_from_arrays(extra, "meta/gen/accuracy_list")
    assert acc == W.accuracy_list_from_arrays(pe, "meta/gen/accuracy_list") and len(acc) >= 200
    sec = "fpe" if encoder == "FPE" else "transformer"
    for k, v in pw[sec].items():
        assert np.array_equal(w[sec][k], v), k


def test_accuracy_list_arrays_round_trip():
    acc = [(0.5, 0.25), (26.4, 0.2, 0.117, 0.744), (1.0, 2.0)]
    back = W.accuracy_list_from_arrays(W.accuracy_list_to_arrays(acc, "k"), "k")
    assert back == acc and W.accuracy_list_from_arrays({}, "k") == []
