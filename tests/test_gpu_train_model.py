"""Offline training (PreGANPlus.py:39-49, train_model): epochs of backprop +
accuracy over load_dataset's whole series (utils.py:36-42), the Transformer's
accuracy_list and checkpoint after each epoch, and the new-model fallback of
load_models when no checkpoint exists (PreGANPlus.py:26-28).  The step itself
is the pinned backprop() path (test_gpu_train.py holds it to the reference's
fixtures); here: the loop's bookkeeping, the dataset and the checkpoint."""
import os

import numpy as np
import pytest
import torch

from preganplus_amd import recovery as RC
from preganplus_amd import train as TR
from preganplus_amd import weights as W


def _series(rows=40, seed=3):
    z = np.load(os.path.join(RC._DATA, "simulator_16.npz"))
    return np.asarray(z["train_time_data"])[:rows]


@pytest.mark.gpu
def test_train_model_epochs_match_backprop_loop(tmp_path):
    series = _series()
    a = RC.PreGANPlusRecovery(16, "", model_folder=str(tmp_path / "in"), save_folder=str(tmp_path))
    b = RC.PreGANPlusRecovery(16, "", model_folder=str(tmp_path / "in"), save_folder=None)
    e0 = a.model_epoch
    a.train_model(num_epochs=2, time_data=series)
    # the same two epochs by hand on an identical plugin
    wins, anom, cls = TR.load_dataset(series)
    ref = []
    for _ in range(2):
        losses, (asc, csc) = TR.backprop(b.trainer, b.tune_state, wins, anom, cls, score=True)
        loss = float(np.mean([x for x, _ in losses]) + np.mean([t for _, t in losses]))
        ref.append((loss, b.tune_state.factor + TR.PROTO_UPDATE_MIN, asc, csc))
    assert a.model_epoch == e0 + 2
    assert a.model_accuracy_list[-2:] == ref
    torch.testing.assert_close(a.trainer.P, b.trainer.P, rtol=0, atol=0)
    # the Transformer checkpoint of the last epoch, in the reference's format
    ck = W._safe_load(os.path.join(str(tmp_path), "simulator_Transformer_16.ckpt"))
    assert int(ck["epoch"]) == e0 + 2 and len(ck["accuracy_list"]) == len(a.model_accuracy_list)
    np.testing.assert_array_equal(np.stack([p.numpy() for p in ck["model_prototypes"]]), a.tune_state.protos)


def test_load_dataset_matches_utils_restatement():
    series = _series(60)
    wins, anom, cls = TR.load_dataset(series)
    td = series / (series.max(axis=0) + 1e-8)                     # utils.py:91-92
    np.testing.assert_array_equal(wins[5], td[2:5])                 # utils.py:7-14
    np.testing.assert_array_equal(wins[0], np.repeat(td[:1], 3, 0))
    thr = np.percentile(td, 98, axis=0)                             # utils.py:16-24
    exp_any = (td > thr).reshape(60, 16, 3).any(axis=2) + 0
    np.testing.assert_array_equal(anom, exp_any)
    np.testing.assert_array_equal(cls, np.argmax(td.reshape(60, 16, 3), axis=2))


@pytest.mark.gpu
def test_new_model_trains_offline_without_checkpoint(tmp_path, monkeypatch):
    """No checkpoint and no packaged weights (H = 8): a new model, trained for
    num_epochs on recovery/PreGANSrc/data/<env>/time_series.npy (here 2 epochs
    of a synthetic 8-host series)."""
    rng = np.random.default_rng(0)
    d = tmp_path / "recovery" / "PreGANSrc" / "data" / "simulator"
    d.mkdir(parents=True)
    np.save(d / "time_series.npy", rng.random((24, 24)) + np.eye(24)[:24] * 3)
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(RC, "NUM_EPOCHS", 2)
    rec = RC.PreGANPlusRecovery(8, "", model_folder=str(tmp_path / "ck"), save_folder=str(tmp_path / "ck"))
    assert rec.model_epoch == 1 and len(rec.model_accuracy_list) == 2
    assert os.path.exists(tmp_path / "ck" / "simulator_Transformer_8.ckpt")
