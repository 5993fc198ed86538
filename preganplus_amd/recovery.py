"""Drop-in ``PreGANPlusRecovery`` (and PreGAN's ``PreGANRecovery``) for the
COSCO framework/simulator on MI355X.

Same constructor and ``run_model(time_series, original_decision)`` contract as
``recovery/PreGANPlus.py:11-136`` (plugin base ``recovery/Recovery.py:3-14``):
``setEnvironment(env)`` then one ``run_model`` per scheduling interval
(``main.py:157``), reading ``env.stats.time_series`` / ``schedule_series`` /
``runSimulation``, ``env.scheduler.result_cache``, ``env.hostlist`` and
``env.containerlist`` by reference, returning a new decision list.

Per call, as the reference:
  1. detect + diagnose on the newest window (at 8 / 16 hosts one launch from
     the training master, ``pgp_forward1``; otherwise the HIP inference
     kernels K1-K3 on the packed copy, rebuilt on the device after training);
     no anomaly -> the original decision (PreGANPlus.py:119-127);
  2. ``train_gan`` (PreGANPlus.py:60-81): Gen/Disc forward, two simulator
     scores, Disc step then Gen step (HIP training kernels + AdamW);
  3. ``tune_model`` (PreGANPlus.py:51-58): 10 sequential tuning steps on the
     latest window set (HIP);
  4. ``recover_decision`` (PreGANPlus.py:83-105) with the updated GAN.
The Gen / Disc checkpoints are rewritten after every ``train_gan`` as the
reference's ``save_gan`` does (PreGANPlus.py:76-81, utils.py:86-88), into the
folder the models were loaded from (default ``recovery/PreGANSrc/checkpointsplus``,
constants.py:3), off the critical path: a device-to-host copy on a side
stream and ``torch.save`` on a writer thread (``_GanCheckpointWriter``).
Deliberate deviations: dropout is off (the reference runs its
modules in train mode with p=0.1, so its own decisions are stochastic); no
plotting; a plugin built from injected ``weights=`` (tests, benches) writes
only when ``save_folder`` is given.

``PreGANRecovery`` (``recovery/PreGAN.py:11-126``, BASELINE config C4): frozen
FPE_16 encoder + K = 3 prototypes (HIP kernel K4), PreGAN's own Gen/Disc (K3),
GAN-only online training when ``training``.  The GRU state is drawn exactly as
the reference draws it (``torch.randn(1, 1, 3, dtype=double)`` on the CPU
generator, ``models.py:70``), so a seeded run reproduces the reference's h0.
"""
from __future__ import annotations

import atexit
import os
import threading
import warnings
import weakref

import numpy as np
import torch

from . import train as TR
from . import weights as W
from .model import DecisionModel, FPEDecisionModel, assemble_decision, migrations, to_numpy

COEFF_ENERGY, COEFF_LATENCY = 0.8, 0.2  # constants.py:19-20
NUM_EPOCHS = 50                          # constants.py:10 (offline training, train_model)
MODEL_PLUS_FOLDER = "recovery/PreGANSrc/checkpointsplus"   # constants.py:3
_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
_AUTO = object()   # save_folder default: where load_models read the checkpoints


class Recovery:
    """recovery/Recovery.py:3-14."""

    def __init__(self):
        self.env = None
        self.env_name = ""
        self.model = None
        self.latent = None

    def setEnvironment(self, env):
        self.env = env

    def run_model(self, time_series, original_decision):
        return original_decision


class _SaveGan:
    """save_gan after every train_gan (utils.py:86-88) through one
    _GanCheckpointWriter per plugin, created on first use; the plugin's
    finalizer (or ``close()``) ends the writer's thread."""

    _writer = None

    def _post_gan_checkpoint(self):
        if self._writer is None:
            self._writer = _GanCheckpointWriter(self.trainer, self.gen_name, self.disc_name)
            self._writer_fin = weakref.finalize(self, _close_writer, self._writer)
        self._writer.post(self.save_folder, self.env_name, self.epoch, self.accuracy_list)

    def flush_checkpoints(self):
        """Wait until the last posted Gen / Disc checkpoint is on disk."""
        if self._writer is not None:
            self._writer.flush()

    def close(self):
        """Write the queued checkpoint and end the writer thread."""
        if self._writer is not None:
            self._writer_fin()
            self._writer = None


class PreGANPlusRecovery(_SaveGan, Recovery):
    def __init__(self, hosts, env, training=False, device=None, model_folder=None, save_folder=_AUTO,
                 weights=None, extra=None, init_seed=0):
        super().__init__()
        self.init_seed = int(init_seed)   # seeds a fresh model's initialisation (no checkpoint, no packaged weights)
        self.model_name = f"Transformer_{hosts}"
        self.gen_name = f"Gen_{hosts}"
        self.disc_name = f"Disc_{hosts}"
        self.hosts = hosts
        self.env_name = "simulator" if env == "" else "framework"
        self.training = training
        if save_folder is _AUTO:   # the reference's save_gan = True, into model_plus_folder (PreGANPlus.py:21)
            save_folder = None if weights is not None else (model_folder or MODEL_PLUS_FOLDER)
        self.save_gan = save_folder is not None
        self.save_folder = save_folder
        self.device = torch.device(device or "cuda")
        self._writer = None
        self.load_models(model_folder, weights, extra)

    # -- PreGANPlus.py:23-37 --
    def load_models(self, model_folder=None, weights=None, extra=None):
        if weights is None:
            folder = model_folder or "recovery/PreGANSrc/checkpointsplus"
            ck = os.path.join(folder, f"{self.env_name}_{self.model_name}.ckpt")
            if os.path.exists(ck):   # load_model + load_gan (utils.py:60-84): weights AND training state
                fresh = lambda: W.torch_default_weights(self.hosts, seed=self.init_seed)
                weights, state = W.load_reference_checkpoints(folder, self.env_name, self.hosts, with_state=True,
                                                              gan_fresh=fresh)
                extra = dict(state, **(extra or {}))
            else:
                packaged = os.path.join(_DATA, f"{self.env_name}_{self.hosts}.npz")
                if not os.path.exists(packaged):
                    # no checkpoint at all: a new model trained offline, as the
                    # reference's load_models does (PreGANPlus.py:26-28, 39-49)
                    self._load_new_model(folder)
                    return
                weights, extra = W.load_npz(packaged)
                # the GAN checkpoints save_gan keeps rewriting (load_gan, PreGANPlus.py:32-34)
                gan = W.load_gan_checkpoints(folder, self.env_name, self.hosts)
                if gan is not None:
                    weights = dict(weights, **gan[0])
                    extra = {k: v for k, v in extra.items()
                             if not k.startswith(("opt/gen/", "opt/disc/", "meta/gen/", "meta/disc/"))}
                    extra.update(gan[1])
        self.extra = extra or {}
        self.prototypes = np.asarray(weights["prototypes"], dtype=np.float64)
        self._infer = DecisionModel(self.hosts, weights, device=self.device)
        self._infer_stale = False
        self.trainer = TR.Trainer(self.hosts, weights, self.extra, device=self.device)
        self.tune_state = TR.TuneState(self.prototypes)
        # load_gan's epoch and accuracy_list are the ones the plugin keeps (PreGANPlus.py:32-34);
        # the encoder checkpoint's own are kept for an explicit full save
        self.epoch = int(self.extra.get("meta/gen/epoch", 0))
        self.accuracy_list = W.accuracy_list_from_arrays(self.extra, "meta/gen/accuracy_list")
        self.model_epoch = int(self.extra.get("meta/transformer/epoch", self.epoch))
        self.model_accuracy_list = W.accuracy_list_from_arrays(self.extra, "meta/transformer/accuracy_list")
        if "train_time_data" in self.extra:
            self.train_time_data = np.asarray(self.extra["train_time_data"], dtype=np.float64)
        else:
            self.train_time_data = np.load(os.path.join("recovery/PreGANSrc/data", self.env_name, "time_series.npy"))

    def _load_new_model(self, folder):
        """load_model without a checkpoint (utils.py:76-78: epoch -1, fresh
        parameters drawn from the distributions torch's module constructors use,
        ``weights.torch_default_weights``, ``init_seed`` seeds it) and the GAN's
        (load_gan: its checkpoints, else new as well, Gen epoch -1), then
        train_model for num_epochs on the reference's data/<env>/time_series.npy."""
        data = os.path.join("recovery/PreGANSrc/data", self.env_name, "time_series.npy")
        if not os.path.exists(data):
            raise FileNotFoundError(f"no checkpoint for {self.model_name} in {folder}, no packaged weights, and "
                                    f"no training data {data} (utils.py:27-31)")
        weights = W.torch_default_weights(self.hosts, seed=self.init_seed)
        extra = {"meta/transformer/epoch": np.array(-1), "meta/gen/epoch": np.array(-1),
                 "train_time_data": np.load(data)}
        gan = W.load_gan_checkpoints(folder, self.env_name, self.hosts)
        if gan is not None:
            weights = dict(weights, **gan[0])
            extra.update(gan[1])
        self.load_models(weights=weights, extra=extra)
        self.model_accuracy_list = []
        self.train_model(NUM_EPOCHS)

    # -- PreGANPlus.py:39-49 (offline training; the plotter is out of scope) --
    def train_model(self, num_epochs=None, time_data=None):
        """num_epochs epochs of backprop + accuracy over the whole training
        series (load_dataset, utils.py:36-42), each appending (loss, factor,
        AScore, CScore) to the Transformer's accuracy_list and, with a save
        folder, rewriting its checkpoint (save_model, utils.py:49-58).  One
        epoch is one backprop() graph of sequential batch-1 steps, the same
        device path tune_model takes."""
        wins, anom, cls = TR.load_dataset(self.train_time_data if time_data is None else time_data)
        for _ in range(NUM_EPOCHS if num_epochs is None else num_epochs):
            self.model_epoch += 1
            losses, (anomaly_score, class_score) = TR.backprop(self.trainer, self.tune_state, wins, anom, cls,
                                                               score=True)
            loss = float(np.mean([a for a, _ in losses]) + np.mean([t for _, t in losses]))   # train.py:56-57
            factor = self.tune_state.factor + TR.PROTO_UPDATE_MIN
            self.model_accuracy_list.append((loss, factor, anomaly_score, class_score))
            if self.save_folder is not None:
                self.flush_checkpoints()
                save_checkpoints(self.trainer, self.save_folder, self.env_name, self.model_epoch,
                                 self.model_accuracy_list,
                                 [("transformer", self.model_name, self.tune_state.protos)])
        self.sync_inference_weights()

    # -- PreGANPlus.py:107-113 --
    def input_window(self):
        td = TR.normalize_test_time_data(self.env.stats.time_series, self.train_time_data)
        if td.shape[0] >= 3:
            td = td[-3:]
        return TR.convert_to_windows(td)[-1]

    def _score(self, schedule):
        e, r = self.env.stats.runSimulation(torch.tensor(schedule))  # utils.py:97-100
        return COEFF_ENERGY * e + COEFF_LATENCY * r

    # -- PreGANPlus.py:60-81 --
    def train_gan(self, embedding, schedule_data):
        if self._writer is not None:
            self._writer.fence()   # the previous call's snapshot copy precedes this update
        ns, new_score, orig_score, gen_loss, disc_loss = TR.train_gan(self.trainer, embedding, schedule_data,
                                                                      self._score)
        # the reference's save_gan is always on: epoch += 1, (gen_loss, disc_loss)
        # appended, Gen / Disc checkpoints rewritten (PreGANPlus.py:76-81)
        self.epoch += 1
        self.accuracy_list.append((gen_loss, disc_loss))
        if self.save_gan:
            self._post_gan_checkpoint()
        return ns

    # -- PreGANPlus.py:51-58 --
    def tune_model(self):
        return self._tune_finish(self._tune_launch())

    def _tune_launch(self):
        """tune_model up to its device work: the on-the-fly dataset, then
        backprop + accuracy (PreGANPlus.py:55-56) as one device graph launched
        on the plugin's tuning stream, ordered after everything already issued
        on the current stream (the detect forward read the weights it updates)."""
        wins, _, anom, cls = TR.on_the_fly_dataset(self.env.stats.time_series, self.env.stats.schedule_series,
                                                   self.train_time_data)
        cur = torch.cuda.current_stream(self.trainer.device)
        if getattr(self, "_tune_stream", None) is None:
            self._tune_stream = torch.cuda.Stream(self.trainer.device)
        self._tune_stream.wait_stream(cur)
        return TR.backprop(self.trainer, self.tune_state, wins, anom, cls, score=True, stream=self._tune_stream,
                           defer=True)

    def _tune_finish(self, finish):
        # later work on the current stream (weight sync, repack, the next detect) follows the graph
        torch.cuda.current_stream(self.trainer.device).wait_stream(self._tune_stream)
        losses, (anomaly_score, class_score) = finish()
        loss = float(np.mean([a for a, _ in losses]) + np.mean([t for _, t in losses]))   # train.py:56-57
        factor = self.tune_state.factor + TR.PROTO_UPDATE_MIN
        self.accuracy_list.append((loss, factor, anomaly_score, class_score))                  # :58
        return losses

    @property
    def infer(self):
        """The packed inference model (K1-K3), rebuilt from the trained master on
        first use after an optimizer step (the packed weights are a cache of the
        master; the 8 / 16-host plugin path reads the master directly)."""
        if self._infer_stale:
            self._repack()
        return self._infer

    def _repack(self):
        """pgp_repack_master: P and the prototypes of the tuning state never
        leave the GPU."""
        self._infer.repack_master(self.trainer.P, self._protos_dev(), self.tune_state.protos)
        self._infer_stale = False

    def sync_inference_weights(self):
        """After training: the inference model follows the updated master
        (utils.py:64-65 updates the reference's modules in place).  The packed
        copy is rebuilt on the device when it is next used (``infer``); the
        device prototypes the detect path and the repack read are refreshed
        here, from the tuning graph's device state when the last backprop left
        one, else from the host TuneState (DPTuner.sync, a reload, ...)."""
        self._infer_stale = True
        self.prototypes = self.tune_state.protos.copy()
        K = self.tune_state.protos.shape[0]
        if getattr(self, "_protos_buf", None) is None or self._protos_buf.numel() != 2 * K:
            self._protos_buf = torch.zeros(2 * K, dtype=torch.float64, device=self.trainer.device)
        st = self.trainer.__dict__.pop("tune_state_dev", None)
        if st is not None:
            self._protos_buf.copy_(st[:2 * K])
        else:
            self._protos_buf.copy_(torch.from_numpy(np.ascontiguousarray(self.tune_state.protos.reshape(-1))))

    # -- PreGANPlus.py:83-105 --
    def recover_decision(self, embedding, schedule_data, original_decision):
        # the updated GAN's gate on (embedding, schedule_data): computed at the end of
        # train_gan's graph (tr.gan_probs_after, same kernels and inputs), else here
        p = self.trainer.__dict__.pop("gan_probs_after", None)
        if p is None:
            _, probs = self.trainer.gan_forward(np.asarray(embedding)[None], np.asarray(schedule_data)[None])
            p = probs[0].cpu().numpy()
        res, hf = _recover(self.env, self.hosts, schedule_data, original_decision, bool(p[0] > p[1]),
                           self.device_, getattr(self, "_final_target", None), io=self._recover_io())
        if hf is not None:
            self.hosts_from = hf
        return res

    @property
    def device_(self):
        return self._infer.device

    def _recover_io(self):
        if getattr(self, "_rio", None) is None:
            self._rio = _RecoverIO(self.hosts, self.device_)
        return self._rio

    def _detect(self, win, schedule_data):
        """The batch-1 forward of run_model (K1-K3) from pinned staging buffers:
        one host-to-device copy in, one device-to-host copy out (to_numpy)."""
        H, dev = self.hosts, self.device_
        if getattr(self, "_io", None) is None:
            nin = 9 * H + H * H
            self._io = (torch.zeros(nin, dtype=torch.float32).pin_memory(),
                        torch.zeros(nin, dtype=torch.float32, device=dev),
                        self._infer.alloc_outputs(1, packed=True))
        hin, din, out = self._io
        h = hin.numpy()
        h[:9 * H] = np.asarray(win, dtype=np.float32).reshape(-1)
        h[9 * H:] = np.asarray(schedule_data, dtype=np.float32).reshape(-1)
        din.copy_(hin, non_blocking=True)
        if H in TR.FUSED_STEP_HOSTS:
            # one launch from the master weights and the tuning state's prototypes (pgp_forward1):
            # the same model the packed copy holds after sync_inference_weights
            return self.trainer.forward1(din[:9 * H], din[9 * H:], self._protos_dev(), out)
        return self.infer.forward(din[:9 * H].view(1, 3, 3 * H), din[9 * H:].view(1, H, H), out=out)

    def _protos_dev(self):
        """The prototypes of the inference model on the device: the plugin's own
        buffer, refreshed by sync_inference_weights after every change."""
        if getattr(self, "_protos_buf", None) is None:
            self.sync_inference_weights()
            self._infer_stale = False   # nothing was trained yet: the packed copy is current
        return self._protos_buf

    # -- PreGANPlus.py:115-136 --
    def run_model(self, time_series, original_decision):
        schedule_data = np.asarray(self.env.scheduler.result_cache, dtype=np.float64)
        win = self.input_window()
        out = to_numpy(self._detect(win, schedule_data))
        if not out["any"][0]:
            return original_decision
        anom = out["logits"][0, :, 1] > out["logits"][0, :, 0]
        embedding = np.where(anom[:, None], out["protos"][0], 0.0)
        self.classes = out["cls"][0].tolist()
        self._final_target = out["final_target"][0].tolist()
        # train_gan then tune_model (PreGANPlus.py:133-134).  They share no data
        # (the GAN step reads the embedding and writes the GAN; the tuning step
        # reads the time series and writes the Transformer and prototypes), so
        # the tuning graph is launched first on its own stream and runs while
        # train_gan waits for the host simulator; its host bookkeeping and
        # accuracy_list entry still come after train_gan's, in the reference's
        # order.  (If train_gan raises, the already launched tuning step is still
        # completed and recorded, where the reference would not have run it.)
        pending = launch_err = first = None
        try:
            try:
                pending = self._tune_launch()
            except Exception as e:   # raised after train_gan, in the reference's order
                launch_err = e
            self.train_gan(embedding, schedule_data)
            if launch_err is not None:
                raise launch_err
            fin, pending = pending, None
            self._tune_finish(fin)
        except BaseException as e:
            first = e
            raise
        finally:
            if pending is not None:
                try:
                    self._tune_finish(pending)
                except Exception as e2:
                    if first is None:
                        raise
                    # train_gan's error propagates; the launched tuning step's own is reported beside it
                    warnings.warn(f"tune_model after a failed train_gan also failed: {e2!r}", RuntimeWarning)
            # the master moved even if tune_model raised (accuracy() divides by zero
            # without a positive label, as the reference's does): K1-K3 follow it
            self.sync_inference_weights()
        return self.recover_decision(embedding, schedule_data, original_decision)

    # -- utils.py:86-88 save_gan: Gen with (epoch, accuracy_list), Disc with (0, []) --
    def save_gan_checkpoints(self, folder):
        self.flush_checkpoints()
        save_checkpoints(self.trainer, folder, self.env_name, self.epoch, self.accuracy_list,
                         [("gen", self.gen_name, None)])
        save_checkpoints(self.trainer, folder, self.env_name, 0, [], [("disc", self.disc_name, None)])

    # -- utils.py:49-58 (checkpoint dict), written with torch.save: all three
    #    models (the reference rewrites only the GAN per call; this is the
    #    explicit full save, e.g. at shutdown).  The encoder checkpoint keeps
    #    its own epoch and accuracy_list, as load_model read them --
    def save_checkpoints(self, folder):
        self.flush_checkpoints()
        save_checkpoints(self.trainer, folder, self.env_name, self.model_epoch, self.model_accuracy_list,
                         [("transformer", self.model_name, self.tune_state.protos)])
        self.save_gan_checkpoints(folder)


def _ckpt_dict(trainer, sec, weights_sec, m, v, steps, epoch, accuracy_list, proto, base=0):
    """The reference's checkpoint dict (utils.py:53-58) for one section from host
    arrays: m / v hold the AdamW moments at blob offsets - base; steps[name] the
    per-parameter step counts (AdamW state per parameter index)."""
    state, idx = {}, 0
    for t in trainer.tensors:
        if t["section"] != sec or not t["trainable"]:
            continue
        sl = slice(t["offset"] - base, t["offset"] - base + t["n"])
        shp = weights_sec[t["name"]].shape
        state[idx] = {"step": torch.tensor(float(steps[t["name"]])),
                      "exp_avg": torch.tensor(m[sl].astype(np.float64).reshape(shp)),
                      "exp_avg_sq": torch.tensor(v[sl].astype(np.float64).reshape(shp))}
        idx += 1
    return {"epoch": epoch,
            "model_state_dict": {k: torch.tensor(np.asarray(a, dtype=np.float64)) for k, a in weights_sec.items()},
            "model_prototypes": [torch.tensor(x) for x in proto] if proto is not None else {},
            "optimizer_state_dict": {"state": state, "param_groups": [{
                "lr": trainer.lrs[sec], "betas": (trainer.b1, trainer.b2),
                "eps": trainer.eps, "weight_decay": trainer.wd, "amsgrad": False,
                "params": list(range(idx))}]},
            "accuracy_list": list(accuracy_list)}


def _save_atomic(ck, path):
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)   # a reader never sees a half-written checkpoint


def save_checkpoints(trainer, folder, env_name, epoch, accuracy_list, entries):
    """Write ``{env}_{name}.ckpt`` per (section, name, prototypes) in the
    reference's checkpoint format (utils.py:49-58, AdamW state per parameter)."""
    os.makedirs(folder, exist_ok=True)
    w = trainer.weights_numpy()
    mm, vv = trainer.m.cpu().numpy(), trainer.v.cpu().numpy()
    for sec, name, proto in entries:
        steps = {t["name"]: t["step"] for t in trainer.tensors if t["section"] == sec}
        _save_atomic(_ckpt_dict(trainer, sec, w[sec], mm, vv, steps, epoch, accuracy_list, proto),
                     os.path.join(folder, f"{env_name}_{name}.ckpt"))


_LIVE_WRITERS = weakref.WeakSet()


@atexit.register
def _flush_live_writers():
    """At exit, every writer still alive writes its newest snapshot (one
    handler for all of them: a per-writer atexit entry would keep each writer,
    its Trainer and its device buffers alive for the whole process)."""
    for w in list(_LIVE_WRITERS):
        try:
            w.flush()
        except Exception:
            pass


class _GanCheckpointWriter:
    """save_gan (utils.py:86-88) after every train_gan, off the critical path.
    ``post()`` snapshots the Gen / Disc master weights and AdamW moments into a
    pinned host buffer with a copy on a side stream (ordered after the GAN step
    on the caller's stream, no host synchronisation) plus the host-side epoch,
    accuracy_list and step counts; a writer thread waits for that copy and
    writes the two checkpoints (Gen with (epoch, accuracy_list), Disc with
    (0, []), atomic renames).  Snapshots still queued when a newer one is posted
    are superseded (the files on disk always end at the newest call, as the
    reference's do).  ``fence()`` makes the caller's stream wait for the last
    snapshot copy before the next GAN update; ``flush()`` waits for the disk;
    ``close()`` flushes and ends the thread.
    Pickling a checkpoint holds the GIL for milliseconds, so after each write the
    writer pauses ``min_interval`` seconds (default 0.05)
    before taking the newest snapshot: calls that come faster than that do not
    wait on the GIL; the files then lag the plugin by at most one pause, and
    ``flush()`` (also at exit) writes the newest state at once.
    The writer holds the Trainer and the two model names, never the plugin, so
    a plugin that goes out of scope is collected and its finalizer closes the
    writer (the thread then releases the Trainer too)."""

    def __init__(self, trainer, gen_name, disc_name, min_interval=None):
        tr = trainer
        self.tr, self.gen_name, self.disc_name = tr, gen_name, disc_name
        self.lo, self.hi = tr.sec_off["gen"], tr.sec_end["disc"]
        n = self.hi - self.lo
        self.bufs = [torch.empty((3, n), dtype=torch.float32).pin_memory() for _ in range(2)]
        self.events = [torch.cuda.Event() for _ in range(2)]
        self.busy = [False, False]
        self.stream = torch.cuda.Stream(tr.device)
        self.next = 0
        self.last_event = None
        self.cv = threading.Condition()
        self.job = None
        self.writing = False
        self.error = None
        self.urgent = False
        self.stopping = False
        self.min_interval = 0.05 if min_interval is None else float(min_interval)
        self.thread = threading.Thread(target=self._run, daemon=True, name="pgp-save-gan")
        self.thread.start()
        _LIVE_WRITERS.add(self)

    def fence(self):
        if self.last_event is not None:
            torch.cuda.current_stream(self.tr.device).wait_event(self.last_event)

    def post(self, folder, env_name, epoch, accuracy_list):
        tr = self.tr
        if self.stopping:
            raise RuntimeError("save_gan writer is closed")
        with self.cv:
            while self.busy[self.next]:
                self.cv.wait()
            k = self.next
            self.busy[k] = True
            self.next ^= 1
        self.stream.wait_stream(torch.cuda.current_stream(tr.device))
        with torch.cuda.stream(self.stream):
            b = self.bufs[k]
            b[0].copy_(tr.P[self.lo:self.hi], non_blocking=True)
            b[1].copy_(tr.m[self.lo:self.hi], non_blocking=True)
            b[2].copy_(tr.v[self.lo:self.hi], non_blocking=True)
            self.events[k].record(self.stream)
        self.last_event = self.events[k]
        # accuracy_list only grows (append): the writer slices the first n entries itself
        job = (k, folder, env_name, epoch, (accuracy_list, len(accuracy_list)),
               {t["name"] + "@" + t["section"]: t["step"] for t in tr.tensors if t["section"] in ("gen", "disc")})
        with self.cv:
            if self.job is not None:          # superseded, never written
                self.busy[self.job[0]] = False
            self.job = job
            self.cv.notify_all()
        if self.error is not None:
            raise RuntimeError("save_gan writer failed") from self.error

    def _run(self):
        while True:
            with self.cv:
                while self.job is None and not self.stopping:
                    self.cv.wait()
                if self.job is None:      # stopping, nothing queued
                    return
                k, folder, env_name, epoch, acc, steps = self.job
                self.job = None
                self.writing = True
            released = False   # buffer k handed back (after its host copy): post() may take it again
            try:
                self.events[k].synchronize()
                host = self.bufs[k].numpy().copy()
                with self.cv:
                    self.busy[k] = False
                    released = True
                    self.cv.notify_all()
                self._write(host, folder, env_name, epoch, acc, steps)
            except Exception as e:  # surfaced on the next post()
                self.error = e
            finally:
                with self.cv:
                    if not released:   # failed before the copy: free the buffer here, never a re-taken one
                        self.busy[k] = False
                    self.writing = False
                    self.cv.notify_all()
                    # pause before the next write unless a flush is waiting
                    if self.min_interval > 0 and not self.urgent and not self.stopping:
                        self.cv.wait_for(lambda: self.urgent or self.stopping, timeout=self.min_interval)

    def _write(self, host, folder, env_name, epoch, acc, steps):
        tr = self.tr
        os.makedirs(folder, exist_ok=True)
        p, m, v = host
        shapes = {(sec, name): shp for sec, name, shp in W.blob_layout(tr.H)[:-1]}
        acc = acc[0][:acc[1]]
        for sec, name, ep, al in (("gen", self.gen_name, epoch, acc), ("disc", self.disc_name, 0, [])):
            wsec = {t["name"]: p[t["offset"] - self.lo:t["offset"] - self.lo + t["n"]].reshape(shapes[(sec, t["name"])])
                    for t in tr.tensors if t["section"] == sec}
            st = {t["name"]: steps[t["name"] + "@" + sec] for t in tr.tensors if t["section"] == sec}
            _save_atomic(_ckpt_dict(tr, sec, wsec, m, v, st, ep, al, None, base=self.lo),
                         os.path.join(folder, f"{env_name}_{name}.ckpt"))

    def flush(self):
        with self.cv:
            self.urgent = True
            self.cv.notify_all()
            while self.job is not None or self.writing:
                self.cv.wait()
            self.urgent = False
        if self.error is not None:
            raise RuntimeError("save_gan writer failed") from self.error

    def close(self):
        """Write what is queued, end the thread (idempotent)."""
        if self.stopping:
            return
        on_writer = self.thread is threading.current_thread()
        try:
            # on the writer thread itself (the plugin collected by a GC pass that
            # runs there, e.g. while _write pickles): flush() would wait for this
            # very thread; the loop writes what is queued before it sees stopping
            if not on_writer:
                self.flush()
        finally:
            with self.cv:
                self.stopping = True
                self.cv.notify_all()
            if not on_writer:
                self.thread.join()
            _LIVE_WRITERS.discard(self)


def _close_writer(writer):
    try:
        writer.close()
    except Exception:
        pass


class _RecoverIO:
    """Pinned / device staging of one K5 call: keep | final_target | cur_host in
    one upload, moves | hosts_from in one download."""

    def __init__(self, C, device):
        self.C = C
        self.hin = torch.zeros(1 + 2 * C, dtype=torch.int32).pin_memory()
        self.din = torch.zeros(1 + 2 * C, dtype=torch.int32, device=device)
        self.dout = torch.zeros((2, 1, C), dtype=torch.int32, device=device)
        self.hout = torch.zeros((2, 1, C), dtype=torch.int32).pin_memory()

    def run(self, final_target, cur):
        C = self.C
        h = self.hin.numpy()
        h[0] = 0
        h[1:1 + C] = final_target
        h[1 + C:] = cur
        self.din.copy_(self.hin, non_blocking=True)
        migrations(self.din[:1], self.din[1:1 + C].view(1, C), self.din[1 + C:].view(1, C),
                   out=(self.dout[0], self.dout[1]))
        self.hout.copy_(self.dout, non_blocking=True)
        torch.cuda.current_stream(self.din.device).synchronize()
        o = self.hout.numpy()
        return o[0, 0].copy(), o[1, 0].copy()


def _recover(env, hosts, schedule_data, original_decision, keep_original, device, final_target=None, io=None):
    """recover_decision's decision loop (PreGAN.py:77-95 == PreGANPlus.py:84-105)
    on the device (K5, pgp_migrations): every placed container moves to the first
    argmax of its ORIGINAL schedule row.  Returns (decision list, hosts_from)."""
    if keep_original:
        return original_decision, None
    cur = [-1] * hosts
    for c in env.containerlist:
        if c and c.getHostID() != -1:
            cur[c.id] = c.getHostID()
    if final_target is None:
        s = np.asarray(schedule_data)
        final_target = [row.index(max(row)) for row in s.tolist()]
    if io is None:
        io = _RecoverIO(hosts, device)
    moves, hosts_from = io.run(np.asarray(final_target, dtype=np.int32), np.asarray(cur, dtype=np.int32))
    return assemble_decision(original_decision, moves, cur), [int(v) for v in hosts_from]


MODEL_FOLDER = "recovery/PreGANSrc/checkpoints"   # constants.py:2 (PreGAN's model_folder)


class PreGANRecovery(_SaveGan, Recovery):
    """recovery/PreGAN.py:11-126 on MI355X.  As the reference's train_gan does
    (PreGAN.py:66-71), every GAN step rewrites the Gen / Disc checkpoints
    (save_gan, utils.py:86-88: Disc with epoch 0 and []) into the folder the
    models were loaded from, on the same writer thread as PreGANPlusRecovery;
    a plugin built from injected ``weights=`` (tests, benches) writes only when
    ``save_folder`` is given."""

    def __init__(self, hosts, env, training=False, device=None, model_folder=None, save_folder=_AUTO,
                 weights=None, extra=None, init_seed=0):
        super().__init__()
        self.init_seed = int(init_seed)   # seeds a fresh model's initialisation (no checkpoint, no packaged weights)
        self.model_name = f"FPE_{hosts}"
        self.gen_name = f"Gen_{hosts}"
        self.disc_name = f"Disc_{hosts}"
        self.hosts = hosts
        self.env_name = "simulator" if env == "" else "framework"
        self.training = training
        if save_folder is _AUTO:   # the reference's save_gan call in train_gan (PreGAN.py:70-71)
            save_folder = None if weights is not None else (model_folder or MODEL_FOLDER)
        self.save_folder = save_folder
        self.save_gan = save_folder is not None
        self.device = torch.device(device or "cuda")
        self.load_models(model_folder, weights, extra)

    # -- PreGAN.py:22-37 (the encoder is frozen; no encoder training path: a
    #    missing FPE checkpoint falls back to the packaged FPE_16 weights, and
    #    the GAN checkpoints save_gan keeps rewriting are loaded over them) --
    def load_models(self, model_folder=None, weights=None, extra=None):
        if weights is None:
            folder = model_folder or MODEL_FOLDER
            ck = os.path.join(folder, f"{self.env_name}_{self.model_name}.ckpt")
            if os.path.exists(ck):
                # load_gan creates a new Gen / Disc for an absent file (utils.py:81-84): a folder
                # holding only the FPE checkpoint (offline training, before the first train_gan)
                fresh = lambda: W.torch_default_fpe_weights(self.hosts, seed=self.init_seed)
                weights, state = W.load_reference_checkpoints(folder, self.env_name, self.hosts, encoder="FPE",
                                                              with_state=True, gan_fresh=fresh)
                extra = dict(state, **(extra or {}))
            else:
                packaged = os.path.join(_DATA, f"pregan_{self.env_name}_{self.hosts}.npz")
                if not os.path.exists(packaged):
                    # no checkpoint at all: a new FPE trained offline, as the
                    # reference's load_models does (PreGAN.py:24-27, 39-49)
                    self._load_new_model(folder)
                    return
                weights, extra = W.load_npz(packaged)
                gan = W.load_gan_checkpoints(folder, self.env_name, self.hosts)   # load_gan (PreGAN.py:31-33)
                if gan is not None:
                    weights = dict(weights, **gan[0])
                    extra = {k: v for k, v in extra.items()
                             if not k.startswith(("opt/gen/", "opt/disc/", "meta/gen/", "meta/disc/"))}
                    extra.update(gan[1])
        self.weights = weights
        self.extra = extra or {}
        self.model = FPEDecisionModel(self.hosts, weights, device=self.device)
        self.epoch = int(self.extra.get("meta/gen/epoch", 0))
        self.accuracy_list = W.accuracy_list_from_arrays(self.extra, "meta/gen/accuracy_list")
        self.trainer = None
        if self.training:
            gan_only = {"transformer": {k: np.zeros(s) for k, s in W.transformer_shapes(self.hosts).items()},
                        "gen": weights["gen"], "disc": weights["disc"],
                        "prototypes": np.zeros((self.hosts, W.PROTO_DIM))}
            self.trainer = TR.Trainer(self.hosts, gan_only, self.extra, device=self.device)
        if "train_time_data" in self.extra:
            self.train_time_data = np.asarray(self.extra["train_time_data"], dtype=np.float64)
        else:
            self.train_time_data = np.load(os.path.join("recovery/PreGANSrc/data", self.env_name, "time_series.npy"))

    def _score(self, schedule):
        e, r = self.env.stats.runSimulation(torch.tensor(schedule))  # utils.py:97-100
        return COEFF_ENERGY * e + COEFF_LATENCY * r

    def _load_new_model(self, folder):
        """load_model without a checkpoint (utils.py:76-78: epoch -1, a new
        FPE_16 with torch's module initialisation distributions,
        weights.torch_default_fpe_weights, ``init_seed`` seeds it), train_model
        (PreGAN.py:39-49: num_epochs epochs of backprop + accuracy over
        load_dataset's whole data/<env>/time_series.npy, the FPE checkpoint
        rewritten after every epoch into the model folder), then the frozen
        encoder with load_gan's GAN (its checkpoints, else new: epoch -1)."""
        data = os.path.join("recovery/PreGANSrc/data", self.env_name, "time_series.npy")
        if not os.path.exists(data):
            raise FileNotFoundError(f"no checkpoint for {self.model_name} in {folder}, no packaged weights, and "
                                    f"no training data {data} (utils.py:27-31)")
        init = W.torch_default_fpe_weights(self.hosts, seed=self.init_seed)
        series = np.load(data)
        self.fpe_epoch, self.fpe_accuracy_list = -1, []
        fpe, protos = self.train_model(init["fpe"], init["prototypes"], series, folder)
        weights = {"fpe": fpe, "gen": init["gen"], "disc": init["disc"], "prototypes": protos}
        extra = {"meta/gen/epoch": np.array(-1), "train_time_data": series}
        gan = W.load_gan_checkpoints(folder, self.env_name, self.hosts)   # load_gan (PreGAN.py:31-33)
        if gan is not None:
            weights = dict(weights, **gan[0])
            extra.update(gan[1])
        self.load_models(weights=weights, extra=extra)

    # -- PreGAN.py:39-49 (offline training; the plotter is out of scope) --
    def train_model(self, fpe, prototypes, time_data, folder=None, num_epochs=None, generator=None):
        """num_epochs epochs of backprop + accuracy of the FPE on the device
        (preganplus_amd.fpetrain) over load_dataset(time_data) (utils.py:36-42),
        each appending (loss, factor, AScore, CScore) to the FPE's accuracy_list
        and, with a folder, rewriting {env}_FPE_{H}.ckpt (save_model,
        utils.py:49-58).  The GRU states are drawn as the reference's forwards
        draw them (torch.randn, models.py:70), backprop's then accuracy's.
        Returns the trained FPE weights (fp64 dict) and prototypes."""
        from . import fpetrain as FT
        wins, anom, cls = TR.load_dataset(time_data)
        n = len(wins)
        ft = FT.FPETrainer(fpe, device=self.device, H=self.hosts)
        st = TR.TuneState(prototypes)
        for _ in range(NUM_EPOCHS if num_epochs is None else num_epochs):
            self.fpe_epoch += 1
            losses = ft.backprop(st, wins, FT.draw_h0(n, generator), anom, cls)
            loss = float(np.mean([a for a, _ in losses]) + np.mean([t for _, t in losses]))   # train.py:56-57
            factor = st.factor + TR.PROTO_UPDATE_MIN
            asc, csc = ft.accuracy(st, wins, FT.draw_h0(n, generator), anom, cls)
            self.fpe_accuracy_list.append((loss, factor, asc, csc))
            if folder is not None:
                os.makedirs(folder, exist_ok=True)
                _save_atomic(ft.checkpoint(self.fpe_epoch, self.fpe_accuracy_list, st.protos),
                             os.path.join(folder, f"{self.env_name}_{self.model_name}.ckpt"))
        self.fpe_trainer, self.fpe_state = ft, st
        return ft.weights_numpy(), st.protos.copy()

    # -- PreGAN.py:97-103 --
    def run_encoder(self, schedule_data):
        td = TR.normalize_test_time_data(self.env.stats.time_series, self.train_time_data)
        if td.shape[0] >= 3:
            td = td[-3:]
        win = TR.convert_to_windows(td)[-1]
        h0 = torch.randn(1, 1, 3, dtype=torch.double)                     # models.py:70
        dev = self.model.device
        f32 = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32, device=dev).contiguous()
        return to_numpy(self.model.forward(f32(win[None]), f32(h0.reshape(1, 3)),
                                           f32(np.asarray(schedule_data)[None])))

    # -- PreGAN.py:51-71 --
    def train_gan(self, embedding, schedule_data):
        if self._writer is not None:
            self._writer.fence()   # the previous call's snapshot copy precedes this update
        _, _, _, gen_loss, disc_loss = TR.train_gan(self.trainer, embedding, schedule_data, self._score)
        self.epoch += 1
        self.accuracy_list.append((gen_loss, disc_loss))                          # PreGAN.py:67
        w = self.trainer.weights_numpy()
        self.weights = dict(self.weights, gen=w["gen"], disc=w["disc"])
        self.model.load_weights(self.weights)     # keep K3's packed GAN in step with the master
        if self.save_gan:                          # save_gan (utils.py:86-88): Disc with epoch 0, []
            self._post_gan_checkpoint()

    # -- PreGAN.py:73-95 --
    def recover_decision(self, embedding, schedule_data, original_decision):
        if self.trainer is not None:
            _, probs = self.trainer.gan_forward(np.asarray(embedding)[None], np.asarray(schedule_data)[None])
            p = probs[0].cpu().numpy()
        else:
            p = self._probs
        res, hf = _recover(self.env, self.hosts, schedule_data, original_decision, bool(p[0] > p[1]),
                           self.model.device, getattr(self, "_final_target", None))
        if hf is not None:
            self.hosts_from = hf
        return res

    # -- PreGAN.py:105-126 --
    def run_model(self, time_series, original_decision):
        schedule_data = np.asarray(self.env.scheduler.result_cache, dtype=np.float64)
        out = self.run_encoder(schedule_data)
        if not out["any"][0]:
            return original_decision
        sc = out["scores"][0]
        anom = sc[:, 1] > sc[:, 0]
        embedding = np.where(anom[:, None], out["protos"][0], 0.0)
        self.classes = out["cls"][0].tolist()
        self._probs = out["probs"][0]
        self._final_target = out["final_target"][0].tolist()
        if self.training:
            self.train_gan(embedding, schedule_data)
        return self.recover_decision(embedding, schedule_data, original_decision)
