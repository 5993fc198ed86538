"""Checkpoint round trip: recovery.save_checkpoints
writes the reference's checkpoint dict (utils.py:49-58) from the device master
weights and AdamW moments; weights.load_reference_checkpoints reads it back with
the safe loader (torch.load weights_only=True), and torch's AdamW accepts the
optimizer state exactly as the reference's load_model does (utils.py:60-79)."""
import os

import numpy as np
import pytest
import torch

from preganplus_amd import simulate as SIM
from preganplus_amd import train as TR
from preganplus_amd import weights as W
from preganplus_amd.recovery import save_checkpoints

pytestmark = pytest.mark.gpu


def test_checkpoint_round_trip(tmp_path):
    H, B = 16, 8
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    tr = TR.Trainer(H, w, max_batch=B)
    rng = np.random.Generator(np.random.PCG64(2))
    emb = np.where(rng.uniform(size=(B, H, 1)) < 0.3, rng.uniform(size=(B, H, 2)), 0.0)
    sched = np.zeros((B, H, H))
    sched[np.arange(B)[:, None], np.arange(H)[None, :], rng.integers(0, H, (B, H))] = 1.0
    TR.train_gan_batched(tr, SIM.Simulation(H), SIM.synth_envs(B, H), emb, sched)  # moments != 0
    protos = np.asarray(w["prototypes"])
    save_checkpoints(tr, str(tmp_path), "simulator", 7, [(0.5, 0.25)],
                     [("transformer", f"Transformer_{H}", protos), ("gen", f"Gen_{H}", None),
                      ("disc", f"Disc_{H}", None)])
    for name in ("Transformer", "Gen", "Disc"):
        assert os.path.exists(tmp_path / f"simulator_{name}_{H}.ckpt")
    back = W.load_reference_checkpoints(str(tmp_path), "simulator", H)
    cur = tr.weights_numpy()
    for sec in ("transformer", "gen", "disc"):
        for k, v in cur[sec].items():
            assert np.array_equal(back[sec][k], v), (sec, k)
    assert np.array_equal(back["prototypes"], protos)
    assert back["meta"]["epoch"] == 7

    # the optimizer state loads into torch.optim.AdamW over the same parameters
    ck = torch.load(tmp_path / f"simulator_Gen_{H}.ckpt", weights_only=True)
    names = [t["name"] for t in tr.tensors if t["section"] == "gen" and t["trainable"]]
    params = [torch.nn.Parameter(torch.tensor(cur["gen"][n])) for n in names]
    opt = torch.optim.AdamW(params, lr=tr.lrs["gen"], weight_decay=tr.wd)
    opt.load_state_dict(ck["optimizer_state_dict"])
    m = tr.m.cpu().numpy()
    for p, t in zip(params, [t for t in tr.tensors if t["section"] == "gen" and t["trainable"]]):
        st = opt.state[p]
        assert float(st["step"]) == t["step"] == 1.0
        want = m[t["offset"]:t["offset"] + t["n"]].reshape(p.shape)
        assert np.array_equal(st["exp_avg"].numpy(), want.astype(np.float64))


def test_plugin_checkpoint_resume(tmp_path):
    """A plugin that ran two intervals saves its checkpoints; a new plugin
    constructed on that folder (the checkpoint path of load_models) resumes
    with the same weights, AdamW moments and step counts, epoch and
    accuracy_list (the checkpoint path used to drop them)."""
    from preganplus_amd.recovery import PreGANPlusRecovery
    from tests.test_train_oracle_golden import fake_env
    w, extra = W.load_npz("preganplus_amd/data/simulator_16.npz")
    z = np.load("tests/golden/plugin_h16.npz")
    a = PreGANPlusRecovery(16, "", training=True, weights=w, extra=extra)
    for step in range(2):
        a.setEnvironment(fake_env(z, step, extra["train_time_data"], z["schedule_series"]))
        a.run_model(None, [tuple(x) for x in z[f"s{step}/decision_in"]])
    a.save_checkpoints(str(tmp_path))
    b = PreGANPlusRecovery(16, "", training=True, model_folder=str(tmp_path),
                           extra={"train_time_data": extra["train_time_data"]})
    assert b.epoch == a.epoch and b.accuracy_list == a.accuracy_list
    torch.cuda.synchronize()
    assert torch.equal(a.trainer.P, b.trainer.P)
    assert torch.equal(a.trainer.m, b.trainer.m) and torch.equal(a.trainer.v, b.trainer.v)
    assert [t["step"] for t in a.trainer.tensors] == [t["step"] for t in b.trainer.tensors]
    np.testing.assert_array_equal(b.prototypes, a.tune_state.protos)
    # the Disc checkpoint carries epoch 0 and an empty accuracy_list (utils.py:86-88)
    ck = torch.load(tmp_path / "simulator_Disc_16.ckpt", weights_only=True)
    assert ck["epoch"] == 0 and ck["accuracy_list"] == []


def test_plugin_save_gan_every_call_resumes(tmp_path):
    """save_gan is on by default (PreGANPlus.py:21, 76-81): a plugin built the
    drop-in way (no injected weights) rewrites the Gen / Disc checkpoints in
    its model folder after every train_gan, on a writer thread; a second plugin
    on the same folder resumes the first's GAN weights, AdamW moments and step
    counts, epoch and accuracy_list as of its last train_gan (the reference
    saves inside train_gan, before tune_model appends its entry)."""
    from preganplus_amd.recovery import PreGANPlusRecovery
    from tests.test_train_oracle_golden import fake_env
    _, extra = W.load_npz("preganplus_amd/data/simulator_16.npz")
    z = np.load("tests/golden/plugin_h16.npz")
    a = PreGANPlusRecovery(16, "", training=True, model_folder=str(tmp_path))
    assert a.save_gan and a.save_folder == str(tmp_path)
    for step in range(3):
        a.setEnvironment(fake_env(z, step, extra["train_time_data"], z["schedule_series"]))
        a.run_model(None, [tuple(x) for x in z[f"s{step}/decision_in"]])
    a.flush_checkpoints()
    for name in ("Gen", "Disc"):
        assert os.path.exists(tmp_path / f"simulator_{name}_16.ckpt")
    assert not os.path.exists(tmp_path / "simulator_Transformer_16.ckpt")   # never rewritten per call
    b = PreGANPlusRecovery(16, "", training=True, model_folder=str(tmp_path))
    assert b.epoch == a.epoch
    assert b.accuracy_list == a.accuracy_list[:-1]          # up to the last train_gan's entry
    tr_a, tr_b = a.trainer, b.trainer
    lo, hi = tr_a.sec_off["gen"], tr_a.sec_end["disc"]
    torch.cuda.synchronize()
    assert torch.equal(tr_a.P[lo:hi], tr_b.P[lo:hi])
    assert torch.equal(tr_a.m[lo:hi], tr_b.m[lo:hi]) and torch.equal(tr_a.v[lo:hi], tr_b.v[lo:hi])
    ga = [t["step"] for t in tr_a.tensors if t["section"] in ("gen", "disc")]
    assert ga == [t["step"] for t in tr_b.tensors if t["section"] in ("gen", "disc")] and min(ga) >= 3
    # the transformer comes from the packaged weights, untouched by save_gan
    t0 = tr_b.sec_off["transformer"]
    fresh = PreGANPlusRecovery(16, "", training=True, weights=W.load_npz("preganplus_amd/data/simulator_16.npz")[0],
                               extra=extra)
    assert torch.equal(tr_b.P[t0:lo], fresh.trainer.P[t0:lo])
    ck = torch.load(tmp_path / "simulator_Disc_16.ckpt", weights_only=True)
    assert ck["epoch"] == 0 and ck["accuracy_list"] == []


def test_pregan_save_gan_every_call_resumes(tmp_path):
    """PreGANRecovery rewrites the Gen / Disc checkpoints after every GAN step
    as the reference's train_gan does (PreGAN.py:66-71, save_gan utils.py:86-88),
    by default into the folder it loaded from; a second plugin on that folder
    (packaged FPE_16 weights, no FPE checkpoint there) resumes the first's GAN
    weights, AdamW moments and step counts, epoch and accuracy_list."""
    from preganplus_amd.recovery import PreGANRecovery
    from tests.test_train_oracle_golden import fake_env
    _, extra = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    z = np.load("tests/golden/pregan_plugin_h16.npz")
    a = PreGANRecovery(16, "", training=True, model_folder=str(tmp_path))
    assert a.save_gan and a.save_folder == str(tmp_path)
    e0 = a.epoch
    for step in range(3):
        a.setEnvironment(fake_env(z, step, extra["train_time_data"], z["schedule_series"]))
        torch.manual_seed(2000 + step)
        a.run_model(None, [tuple(x) for x in z[f"s{step}/decision_in"]])
    assert a.epoch == e0 + 3
    a.flush_checkpoints()
    for name in ("Gen", "Disc"):
        assert os.path.exists(tmp_path / f"simulator_{name}_16.ckpt")
    assert not os.path.exists(tmp_path / "simulator_FPE_16.ckpt")    # the encoder is frozen, never saved
    b = PreGANRecovery(16, "", training=True, model_folder=str(tmp_path))
    assert b.epoch == a.epoch and b.accuracy_list == a.accuracy_list
    lo, hi = a.trainer.sec_off["gen"], a.trainer.sec_end["disc"]
    torch.cuda.synchronize()
    assert torch.equal(a.trainer.P[lo:hi], b.trainer.P[lo:hi])
    assert torch.equal(a.trainer.m[lo:hi], b.trainer.m[lo:hi]) and torch.equal(a.trainer.v[lo:hi], b.trainer.v[lo:hi])
    sa = [t["step"] for t in a.trainer.tensors if t["section"] in ("gen", "disc")]
    assert sa == [t["step"] for t in b.trainer.tensors if t["section"] in ("gen", "disc")]
    ck = torch.load(tmp_path / "simulator_Disc_16.ckpt", weights_only=True)
    assert ck["epoch"] == 0 and ck["accuracy_list"] == []
    # injected weights (tests, benches): no save unless a folder is given
    w, ex = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    assert not PreGANRecovery(16, "", training=True, weights=w, extra=ex).save_gan
    a.close()
    b.close()
    assert a._writer is None


def test_writer_snapshots_are_never_torn(tmp_path):
    """posting as fast as possible (no pause between writes) must
    never hand the writer a buffer that a later post() is refilling: every
    snapshot it writes holds one post's weights and moments throughout."""
    from preganplus_amd import recovery as RC
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    tr = TR.Trainer(16, w, max_batch=1)
    lo, hi = tr.sec_off["gen"], tr.sec_end["disc"]
    seen = []

    class Checking(RC._GanCheckpointWriter):
        def _write(self, host, folder, env_name, epoch, acc, steps):
            p, m, v = host
            seen.append(epoch)
            assert p.min() == p.max() == m.min() == m.max() == v.min() == v.max() == float(epoch), epoch

    wr = Checking(tr, "Gen_16", "Disc_16", min_interval=0.0)
    try:
        for k in range(200):
            wr.fence()
            tr.P[lo:hi].fill_(float(k))
            tr.m[lo:hi].fill_(float(k))
            tr.v[lo:hi].fill_(float(k))
            wr.post(str(tmp_path), "simulator", k, [])
        wr.flush()
    finally:
        wr.close()
    assert wr.error is None, wr.error
    assert seen and seen[-1] == 199 and seen == sorted(seen)
    assert not wr.thread.is_alive()


def test_checkpoint_folder_without_gan_files_starts_a_new_gan(tmp_path):
    """load_gan creates a new Gen / Disc when their files are absent
    (utils.py:76-78, 81-84): a folder holding only the encoder checkpoint (an
    offline-trained model before its first train_gan) loads the encoder and a
    fresh GAN (Gen epoch -1, no optimizer state) instead of failing."""
    from preganplus_amd.recovery import PreGANPlusRecovery
    H, B = 16, 4
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    tr = TR.Trainer(H, w, max_batch=B)
    protos = np.asarray(w["prototypes"])
    save_checkpoints(tr, str(tmp_path), "simulator", 3, [], [("transformer", f"Transformer_{H}", protos)])
    assert not os.path.exists(tmp_path / f"simulator_Gen_{H}.ckpt")
    with pytest.raises(Exception):
        W.load_reference_checkpoints(str(tmp_path), "simulator", H)   # no fallback given: an absent file raises
    fresh = W.torch_default_weights(H, seed=5)
    back, extra = W.load_reference_checkpoints(str(tmp_path), "simulator", H, with_state=True,
                                               gan_fresh=lambda: fresh)
    cur = tr.weights_numpy()
    for k, v in cur["transformer"].items():
        assert np.array_equal(back["transformer"][k], v), k
    for sec in ("gen", "disc"):
        for k, v in fresh[sec].items():
            assert np.array_equal(np.asarray(back[sec][k]), np.asarray(v)), (sec, k)
    assert back["meta"]["gan_epoch"] == -1
    assert not any(k.startswith("opt/gen/") or k.startswith("opt/disc/") for k in extra)
    # the plugin's checkpoint branch takes the same path (init_seed seeds the new GAN)
    _, extra0 = W.load_npz("preganplus_amd/data/simulator_16.npz")
    plug = PreGANPlusRecovery(H, "", model_folder=str(tmp_path), save_folder=None, init_seed=5,
                              extra={"train_time_data": extra0["train_time_data"]})
    got = plug.trainer.weights_numpy()
    for k, v in cur["transformer"].items():
        assert np.array_equal(got["transformer"][k], v), k
    for k, v in fresh["gen"].items():
        assert np.array_equal(got["gen"][k], np.asarray(v, dtype=np.float32)), k


def test_writer_close_on_its_own_thread_returns(tmp_path):
    """close() called on the writer thread itself (a plugin collected by a GC
    pass that runs there) must not wait for that very thread: it returns, and
    the thread ends after the write in progress."""
    import threading
    from preganplus_amd.recovery import _GanCheckpointWriter
    H = 16
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    tr = TR.Trainer(H, w, max_batch=4)
    wr = _GanCheckpointWriter(tr, f"Gen_{H}", f"Disc_{H}", min_interval=0.0)
    done = threading.Event()
    real_write = wr._write

    def write_then_close(*a):
        real_write(*a)
        wr.close()            # on the writer thread
        done.set()

    wr._write = write_then_close
    wr.post(str(tmp_path), "simulator", 1, [])
    assert done.wait(60), "close() on the writer thread did not return"
    wr.thread.join(60)
    assert not wr.thread.is_alive()
    assert os.path.exists(tmp_path / f"simulator_Gen_{H}.ckpt")
