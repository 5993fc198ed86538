"""Online training on MI355X: host side of the tuning and GAN steps.

Mirrors the reference's training code (recovery/PreGANSrc/src/train.py:13-57,
recovery/PreGANPlus.py:51-81, utils.py:65) with every tensor operation in the
HIP library (``pgp_tune_*``, ``pgp_gan_*``, ``pgp_adamw``).  The reference's
scalar, sequential bookkeeping — the per-host loop of ``custom_loss`` that
decides CE weights (num_zero/num_ones) and the prototype EMA of
``triplet_loss`` (it depends on the forward's outputs and must run host-by-host
in order) — runs on the device in the single-model ``backprop`` loop
(``pgp_tune_targets``, fp64, the reference's operation order), so the ten
sequential steps of one interval need no host round trip.  ``loss_targets`` is
the same bookkeeping in numpy; the data-parallel step keeps it on the host,
where the ranks' increments are reduced.
"""
from __future__ import annotations

import ctypes
import math
import os

import types

import numpy as np
import torch

from . import _native
from . import weights as W

PROTO_UPDATE_FACTOR = 0.2   # constants.py:13
PROTO_UPDATE_MIN = 0.02     # constants.py:14
PROTO_FACTOR_DECAY = 0.995  # constants.py:15
LATEST_WINDOW_SIZE = 10     # constants.py:16
PERCENTILES = 98            # constants.py:11


# the current stream's raw handle by device index (torch's C++ accessor; None
# if this torch lacks it, then Trainer._stream takes the public API)
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


class _AdamTensor(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_longlong), ("n", ctypes.c_int), ("active", ctypes.c_int),
                ("step_size", ctypes.c_float), ("bc2_sqrt", ctypes.c_float)]


def default_lrs(H):
    """Model lr attributes: Transformer_16.lr = 1e-4 (models.py:318); Gen/Disc
    5e-5 at 16 hosts (:122, :140), 3e-5 at 50 (:262, :280)."""
    g = 5e-5 if H <= 16 else 3e-5
    return {"transformer": 1e-4, "gen": g, "disc": g}


class Trainer:
    """fp32 master weights in the natural blob order (prototypes excluded),
    gradients and AdamW moments, all on the device."""

    SECTIONS = ("transformer", "gen", "disc")

    def __init__(self, H: int, weights: dict, extra: dict | None = None, lrs: dict | None = None,
                 device="cuda", max_batch: int = 16, weight_decay=1e-5, betas=(0.9, 0.999), eps=1e-8):
        self.H = int(H)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        L = _native.lib()
        self._L = L
        self._bind()
        self._desc_cache = {}
        n = L.pgp_master_len(self.H)
        if n == 0:
            raise ValueError(f"H={H} not compiled in")
        blob = W.pack_blob(weights, self.H)[:n]
        dev = self.device
        self.P = torch.tensor(blob, dtype=torch.float32, device=dev)
        self.G = torch.zeros_like(self.P)
        self.m = torch.zeros_like(self.P)
        self.v = torch.zeros_like(self.P)
        self.lrs = dict(default_lrs(self.H), **(lrs or {}))
        self.wd, self.b1, self.b2, self.eps = weight_decay, betas[0], betas[1], eps
        # tensor table in blob order
        self.tensors = []
        off = 0
        for sec, name, shp in W.blob_layout(self.H)[:-1]:
            cnt = int(np.prod(shp))
            self.tensors.append({"section": sec, "name": name, "offset": off, "n": cnt, "step": 0.0,
                                 "trainable": name != "pos_encoder.pe"})
            off += cnt
        assert off == n
        if extra:
            m = self.m.cpu().numpy()
            v = self.v.cpu().numpy()
            for t in self.tensors:
                key = f"opt/{t['section']}/{t['name']}"
                if f"{key}/exp_avg" in extra:
                    m[t["offset"]:t["offset"] + t["n"]] = np.asarray(extra[f"{key}/exp_avg"]).reshape(-1)
                    v[t["offset"]:t["offset"] + t["n"]] = np.asarray(extra[f"{key}/exp_avg_sq"]).reshape(-1)
                    t["step"] = float(extra[f"{key}/step"])
            self.m.copy_(torch.tensor(m))
            self.v.copy_(torch.tensor(v))
        self.sec_off = {s: int(L.pgp_master_offset(self.H, i)) for i, s in enumerate(self.SECTIONS)}
        self.sec_end = {"transformer": self.sec_off["gen"], "gen": self.sec_off["disc"], "disc": n}
        self._alloc(max_batch)

    def _bind(self):
        L = self._L
        if getattr(L, "_pgp_train_bound", False):
            return
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.pgp_master_len.argtypes = [i32]
        L.pgp_master_len.restype = sz
        L.pgp_master_offset.argtypes = [i32, i32]
        L.pgp_master_offset.restype = sz
        L.pgp_tune_workspace_len.argtypes = [i32, i32]
        L.pgp_tune_workspace_len.restype = sz
        L.pgp_gan_workspace_len.argtypes = [i32, i32]
        L.pgp_gan_workspace_len.restype = sz
        L.pgp_tune_forward.argtypes = [i32, i32] + [vp] * 6 + [vp]
        L.pgp_tune_backward.argtypes = [i32, i32] + [vp] * 8 + [vp]
        L.pgp_tune_backward_prefix.argtypes = [i32, i32, i32] + [vp] * 8 + [vp]
        L.pgp_gan_forward.argtypes = [i32, i32] + [vp] * 6 + [vp]
        L.pgp_gan_disc_backward.argtypes = [i32, i32] + [vp] * 4 + [vp]
        L.pgp_gan_gen_backward.argtypes = [i32, i32] + [vp] * 3 + [vp]
        L.pgp_gan_probs.argtypes = [i32, i32, vp, vp, vp]
        L.pgp_adamw.argtypes = [vp] * 4 + [ctypes.c_float] * 5 + [ctypes.POINTER(_AdamTensor), i32, vp]
        L.pgp_load_weights_master.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_double)]
        L.pgp_tune_targets.argtypes = [i32, i32] + [vp] * 5 + [ctypes.c_double] * 2 + [vp] * 3 + [vp]
        L.pgp_adamw_table.argtypes = ([vp] * 4 + [ctypes.c_float] * 5 + [ctypes.POINTER(_AdamTensor), i32, vp]
                                      + [vp])
        dbl = ctypes.c_double
        L.pgp_tune_step1.argtypes = [i32, i32] + [vp] * 6 + [dbl, dbl] + [vp] * 3 + [vp]
        L.pgp_forward1.argtypes = [i32, i32] + [vp] * 12 + [vp]
        L.pgp_tune_forward_many.argtypes = [i32, i32] + [vp] * 4 + [vp]
        L.pgp_gan_forward1.argtypes = [i32] + [vp] * 6 + [vp]
        f32 = ctypes.c_float
        L.pgp_gan_step1.argtypes = ([i32] + [vp] * 5 + [f32] * 6 + [ctypes.POINTER(_AdamTensor), i32, vp]
                                    + [ctypes.POINTER(_AdamTensor), i32, vp] + [vp] * 3 + [vp])
        L.pgp_tune_dataset.argtypes = [i32, i32, i32] + [vp] * 6 + [vp]
        L.pgp_tune_targets_dp_workspace_len.argtypes = [i32]
        L.pgp_tune_targets_dp_workspace_len.restype = sz
        L.pgp_tune_targets_dp.argtypes = [i32, i32, i32] + [vp] * 5 + [dbl] + [vp] * 5 + [vp]
        L.pgp_tune_state_apply.argtypes = [i32, vp, vp, dbl, i32, ctypes.POINTER(ctypes.c_int), vp, vp,
                                           dbl, dbl, dbl, vp]
        for f in ("pgp_tune_forward", "pgp_tune_backward", "pgp_tune_backward_prefix", "pgp_gan_forward", "pgp_gan_disc_backward",
                  "pgp_gan_gen_backward", "pgp_adamw", "pgp_load_weights_master", "pgp_tune_targets",
                  "pgp_adamw_table", "pgp_tune_dataset", "pgp_tune_targets_dp", "pgp_tune_state_apply",
                  "pgp_gan_probs", "pgp_tune_step1", "pgp_forward1", "pgp_tune_forward_many",
                  "pgp_gan_forward1", "pgp_gan_step1"):
            getattr(L, f).restype = i32
        L._pgp_train_bound = True

    def _alloc(self, B):
        H, dev, L = self.H, self.device, self._L
        f32 = torch.float32
        self.cap = B
        self.generation = getattr(self, "generation", 0) + 1  # captured graphs hold these buffers
        self._graphs = {}
        # token-major activations of the tuning forward (kept for the backward);
        # zero-filled once: feature pads must stay 0 (pgp_tune.hpp)
        self.ws = torch.zeros((L.pgp_tune_workspace_len(H, B),), dtype=f32, device=dev)
        self.gscr = torch.zeros((L.pgp_gan_workspace_len(H, B),), dtype=f32, device=dev)
        self.logits = torch.zeros((B, H, 2), dtype=f32, device=dev)
        self.protos = torch.zeros((B, H, 2), dtype=f32, device=dev)
        self._fwd_batch = 0
        self.ns = torch.zeros((B, H, H), dtype=f32, device=dev)
        self.probs = torch.zeros((B, 2), dtype=f32, device=dev)

    def _ensure(self, B):
        if B > self.cap:
            self._alloc(B)

    def _dev(self, a, dtype):
        if torch.is_tensor(a) and a.dtype == dtype and a.device == self.device and a.is_contiguous():
            return a   # already in place: no dispatcher round trip (host issue time, C3 at H = 16)
        t = a if torch.is_tensor(a) else torch.as_tensor(np.asarray(a))
        return t.to(self.device, dtype).contiguous()

    def _stream(self):
        # the current stream's raw handle straight from the C++ side:
        # torch.cuda.current_stream(device) costs ~4 us of argument parsing, and
        # a C3 step asks ~20 times (cProfile, profiles/r04/host_issue/)
        idx = self.device.index
        if idx is not None and _RAW_STREAM is not None:
            return ctypes.c_void_p(_RAW_STREAM(idx))
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def trainable(self, section: str) -> list:
        """The section's trainable tensor records (one list object per section,
        so its AdamW descriptor is built once)."""
        c = self._desc_cache.get(("sel", section))
        if c is None:
            c = [t for t in self.tensors if t["section"] == section and t["trainable"]]
            self._desc_cache[("sel", section)] = c
        return c

    def _adam_desc(self, sel):
        """ctypes descriptor array of an AdamW selection, cached by its
        (offset, n) ranges: the same tensors give the same descriptor whatever
        list object names them, and a list mutated in place gets a new one."""
        key = ("desc",) + tuple((t["offset"], t["n"]) for t in sel)
        c = self._desc_cache.get(key)
        if c is None:
            c = (_AdamTensor * len(sel))(*[_AdamTensor(t["offset"], t["n"], 1, 0.0, 0.0) for t in sel])
            self._desc_cache[key] = c
        return c

    # ---------------- ops ----------------
    def zero_grad(self, section: str):
        self.G[self.sec_off[section]:self.sec_end[section]].zero_()

    def forward_context(self, B):
        """A workspace and outputs of their own for a forward that runs beside
        the tuning step (the C3 detect on a second stream): tune_forward(...,
        ctx=) leaves the tuning step's activations alone."""
        L, dev, f32 = self._L, self.device, torch.float32
        return types.SimpleNamespace(
            cap=B, ws=torch.zeros((L.pgp_tune_workspace_len(self.H, B),), dtype=f32, device=dev),
            logits=torch.zeros((B, self.H, 2), dtype=f32, device=dev),
            protos=torch.zeros((B, self.H, 2), dtype=f32, device=dev))

    def tune_forward(self, windows: torch.Tensor, latent: torch.Tensor | None = None, ctx=None):
        """Transformer forward of a batch of windows [B,3,3H], activations kept
        in the workspace for tune_backward; optional latent tap [B,3H^2].  With
        ``ctx`` (forward_context) the workspace and outputs are the context's
        (no tune_backward may follow from them)."""
        B = windows.shape[0]
        if ctx is None:
            self._ensure(B)
            ws, lg, pr = self.ws, self.logits, self.protos
        else:
            if B > ctx.cap:
                raise ValueError(f"batch {B} > forward context capacity {ctx.cap}")
            ws, lg, pr = ctx.ws, ctx.logits, ctx.protos
        windows = windows.to(self.device, torch.float32).contiguous()
        _native.check(self._L.pgp_tune_forward(
            self.H, B, windows.data_ptr(), self.P.data_ptr(), ws.data_ptr(),
            None if latent is None else latent.data_ptr(),
            lg.data_ptr(), pr.data_ptr(), self._stream()), "pgp_tune_forward")
        if ctx is None:
            self._fwd_batch = B
        return lg[:B], pr[:B]

    def tune_backward(self, B, y, mult, tgt):
        """y [B,H] int, mult [B,H], tgt [B,H,2] (host arrays or tensors).  B is
        the batch of the preceding tune_forward, or fewer: then the gradient is
        of its FIRST B windows' losses (``pgp_tune_backward_prefix``; the rest
        were inference windows sharing the forward, e.g. C3's detect)."""
        if not 0 < B <= self._fwd_batch:
            raise ValueError(f"tune_backward batch {B} not in 1..{self._fwd_batch} (the tune_forward batch)")
        y = self._dev(y, torch.int32)
        mult = self._dev(mult, torch.float32)
        tgt = self._dev(tgt, torch.float32)
        # (the backward writes every trainable entry of the section: no zero_grad)
        if B == self._fwd_batch:
            _native.check(self._L.pgp_tune_backward(
                self.H, B, self.P.data_ptr(), self.G.data_ptr(), self.ws.data_ptr(),
                self.logits.data_ptr(), self.protos.data_ptr(), y.data_ptr(), mult.data_ptr(), tgt.data_ptr(),
                self._stream()), "pgp_tune_backward")
        else:
            _native.check(self._L.pgp_tune_backward_prefix(
                self.H, self._fwd_batch, B, self.P.data_ptr(), self.G.data_ptr(), self.ws.data_ptr(),
                self.logits.data_ptr(), self.protos.data_ptr(), y.data_ptr(), mult.data_ptr(), tgt.data_ptr(),
                self._stream()), "pgp_tune_backward_prefix")

    def tune_targets(self, y, cls, state, mult, tgt, loss):
        """custom_loss / triplet_loss bookkeeping of the preceding batch-1
        tune_forward on the device (``pgp_tune_targets``): y, cls [H] int32,
        state [9] fp64 (``TuneState.to_device``) updated in place; writes
        mult [H], tgt [H,2] (fp32) and loss [2] fp64.  All device tensors."""
        K = (state.numel() - 3) // 2
        if self._fwd_batch != 1:
            raise ValueError("tune_targets follows a batch-1 tune_forward (train.py:47-53)")
        _native.check(self._L.pgp_tune_targets(
            self.H, K, self.logits.data_ptr(), self.protos.data_ptr(), y.data_ptr(), cls.data_ptr(),
            state.data_ptr(), PROTO_UPDATE_MIN, PROTO_FACTOR_DECAY, mult.data_ptr(), tgt.data_ptr(),
            loss.data_ptr(), self._stream()), "pgp_tune_targets")

    def tune_step1(self, window, y, cls, state, loss):
        """tune_forward + tune_targets + tune_backward of ONE window as a single
        launch (``pgp_tune_step1``, n_hosts 8 or 16): window [1,3,3H] (or
        [3,3H]), y, cls [H] int32, state as tune_targets; writes logits /
        protos, loss [2] fp64 and the transformer section of G.  Device
        tensors."""
        K = (state.numel() - 3) // 2
        _native.check(self._L.pgp_tune_step1(
            self.H, K, window.data_ptr(), y.data_ptr(), cls.data_ptr(), self.P.data_ptr(), self.G.data_ptr(),
            state.data_ptr(), PROTO_UPDATE_MIN, PROTO_FACTOR_DECAY, self.logits.data_ptr(),
            self.protos.data_ptr(), loss.data_ptr(), self._stream()), "pgp_tune_step1")
        self._fwd_batch = 0   # the fused step keeps no activations for tune_backward

    def tune_forward_many(self, windows, logits64, protos64):
        """n independent batch-1 forwards from the master (``pgp_tune_forward_many``,
        n_hosts 8 or 16; the fused step's forward, one workgroup per window):
        windows [n,3,3H] fp32 -> logits64 / protos64 [n*H*2] fp64 device tensors
        (accuracy()'s batched forward, train.py:94-109)."""
        n = windows.shape[0]
        _native.check(self._L.pgp_tune_forward_many(
            self.H, n, windows.data_ptr(), self.P.data_ptr(), logits64.data_ptr(), protos64.data_ptr(),
            self._stream()), "pgp_tune_forward_many")

    def forward1(self, window, sched, protos_dev, out):
        """run_model's forward of ONE window from the master weights
        (``pgp_forward1``, n_hosts 8 or 16): window [3,3H], sched [H,H] fp32,
        protos_dev [K,2] fp64, all device tensors; out: a DecisionModel output
        dict for batch 1 (logits, protos, cls, any, probs, keep, final_target,
        gen_target)."""
        K = protos_dev.numel() // 2
        p = lambda k: out[k].data_ptr()
        _native.check(self._L.pgp_forward1(
            self.H, K, window.data_ptr(), sched.data_ptr(), self.P.data_ptr(), protos_dev.data_ptr(),
            p("logits"), p("protos"), p("cls"), p("any"), p("probs"), p("keep"), p("final_target"),
            p("gen_target"), self._stream()), "pgp_forward1")
        return out

    def gan_forward(self, emb, sched):
        emb = self._dev(emb, torch.float32)
        emb = emb.reshape(emb.shape[0], -1).contiguous()
        sched = self._dev(sched, torch.float32)
        B = sched.shape[0]
        self._ensure(B)
        self._gan_in = (emb, sched)
        _native.check(self._L.pgp_gan_forward(
            self.H, B, emb.data_ptr(), sched.data_ptr(), self.P.data_ptr(), self.gscr.data_ptr(),
            self.ns.data_ptr(), self.probs.data_ptr(), self._stream()), "pgp_gan_forward")
        return self.ns[:B], self.probs[:B]

    def gan_forward1(self, emb, sched, ns_out, probs_out):
        """Gen + Disc forward of ONE window (``pgp_gan_forward1``, n_hosts 8 or
        16): emb [2H], sched [H,H] fp32 device tensors -> ns_out [H*H],
        probs_out [2]; the activations stay in the GAN workspace for
        ``gan_step1``."""
        self._ensure(1)
        _native.check(self._L.pgp_gan_forward1(
            self.H, emb.data_ptr(), sched.data_ptr(), self.P.data_ptr(), self.gscr.data_ptr(), ns_out.data_ptr(),
            probs_out.data_ptr(), self._stream()), "pgp_gan_forward1")

    def gan_step1(self, target, selD, tabD, selG, tabG, probs_gen, probs_after):
        """The rest of train_gan for that window in one launch (``pgp_gan_step1``):
        Disc BCE step + AdamW (device table tabD [len(selD),3]), Gen step through
        the updated Disc + AdamW (tabG), the updated GAN's probabilities.
        target [2] device fp32; probs_gen / probs_after [2] device outputs."""
        desc = lambda sel: (_AdamTensor * len(sel))(*[_AdamTensor(t["offset"], t["n"], 1, 0.0, 0.0) for t in sel])
        _native.check(self._L.pgp_gan_step1(
            self.H, target.data_ptr(), self.P.data_ptr(), self.G.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
            self.lrs["disc"], self.lrs["gen"], self.wd, self.b1, self.b2, self.eps,
            desc(selD), len(selD), tabD.data_ptr(), desc(selG), len(selG), tabG.data_ptr(),
            self.gscr.data_ptr(), probs_gen.data_ptr(), probs_after.data_ptr(), self._stream()), "pgp_gan_step1")

    def gan_disc_backward(self, target):
        """The Disc's BCE gradients toward target [B,2], WRITTEN into G's disc
        section (every element: no zero-fill needed)."""
        target = self._dev(target, torch.float32)
        B = target.shape[0]
        _native.check(self._L.pgp_gan_disc_backward(
            self.H, B, target.data_ptr(), self.P.data_ptr(), self.G.data_ptr(), self.gscr.data_ptr(),
            self._stream()), "pgp_gan_disc_backward")

    def gan_gen_backward(self, B):
        """The Gen's BCE gradients toward [0,1] through the current Disc, WRITTEN
        into G's gen section."""
        _native.check(self._L.pgp_gan_gen_backward(
            self.H, B, self.P.data_ptr(), self.G.data_ptr(), self.gscr.data_ptr(), self._stream()),
            "pgp_gan_gen_backward")

    def gan_probs(self, B):
        """The Disc probabilities of the last Disc head in the GAN workspace
        [B,2] (after gan_gen_backward: gen_loss's, PreGANPlus.py:71-73)."""
        out = torch.empty((B, 2), dtype=torch.float32, device=self.device)
        _native.check(self._L.pgp_gan_probs(self.H, B, self.gscr.data_ptr(), out.data_ptr(), self._stream()),
                      "pgp_gan_probs")
        return out

    def adam_step(self, section: str, inactive: tuple = ()):
        """torch.optim.AdamW.step for the tensors of `section` (utils.py:65);
        tensors named in `inactive` had no gradient and are skipped, as torch
        skips params whose .grad is None."""
        lr = self.lrs[section]
        arr = []
        for t in self.tensors:
            if t["section"] != section or not t["trainable"]:
                continue
            active = t["name"] not in inactive
            if active:
                t["step"] += 1
            st = max(t["step"], 1.0)
            arr.append(_AdamTensor(t["offset"], t["n"], int(active), lr / (1 - self.b1 ** st),
                                   math.sqrt(1 - self.b2 ** st)))
        desc = (_AdamTensor * len(arr))(*arr)
        _native.check(self._L.pgp_adamw(
            ctypes.c_void_p(self.P.data_ptr()), ctypes.c_void_p(self.G.data_ptr()),
            ctypes.c_void_p(self.m.data_ptr()), ctypes.c_void_p(self.v.data_ptr()),
            lr, self.wd, self.b1, self.b2, self.eps, desc, len(arr), self._stream()), "pgp_adamw")

    def adam_schedule(self, section: str, inactive_per_step):
        """adam_step's host bookkeeping for a sequence of steps, done ahead:
        returns the section's trainable tensors and a [steps, T, 3] fp32 table
        of (active, step_size, bc2_sqrt) — the values adam_step would pass —
        and advances the tensors' step counts as those steps would."""
        lr = self.lrs[section]
        sel = [t for t in self.tensors if t["section"] == section and t["trainable"]]
        tab = np.zeros((len(inactive_per_step), len(sel), 3), dtype=np.float32)
        for s, inactive in enumerate(inactive_per_step):
            for k, t in enumerate(sel):
                active = t["name"] not in inactive
                if active:
                    t["step"] += 1
                st = max(t["step"], 1.0)
                tab[s, k] = (float(active), lr / (1 - self.b1 ** st), math.sqrt(1 - self.b2 ** st))
        return sel, tab

    def adam_schedule_np(self, section: str, positive, cond_names):
        """adam_schedule for the tuning loop's pattern, vectorised: step s of a
        call skips the tensors named in cond_names unless positive[s] (the
        prototype decoder gets no gradient from a window without a positive
        label).  Same values as adam_schedule, same step-count advance."""
        lr = self.lrs[section]
        sel = [t for t in self.tensors if t["section"] == section and t["trainable"]]
        positive = np.asarray(positive, dtype=bool)
        cond = np.array([t["name"] in cond_names for t in sel])
        active = np.where(cond[None, :], positive[:, None], True)                # [steps, T]
        step0 = np.array([t["step"] for t in sel], dtype=np.float64)
        steps = step0[None, :] + np.cumsum(active, axis=0)
        st = np.maximum(steps, 1.0)
        tab = np.empty(active.shape + (3,), dtype=np.float32)
        tab[..., 0] = active
        tab[..., 1] = lr / (1 - self.b1 ** st)
        tab[..., 2] = np.sqrt(1 - self.b2 ** st)
        for k, t in enumerate(sel):
            t["step"] = float(steps[-1, k])
        return tab

    def adam_step_table(self, section: str, sel, sched):
        """AdamW over `sel` with the per-step scalars in the device row `sched`
        [T,3] (``pgp_adamw_table``): fixed kernel arguments, graph-capturable."""
        desc = self._adam_desc(sel)
        _native.check(self._L.pgp_adamw_table(
            ctypes.c_void_p(self.P.data_ptr()), ctypes.c_void_p(self.G.data_ptr()),
            ctypes.c_void_p(self.m.data_ptr()), ctypes.c_void_p(self.v.data_ptr()),
            self.lrs[section], self.wd, self.b1, self.b2, self.eps, desc, len(sel), sched.data_ptr(),
            self._stream()), "pgp_adamw_table")

    def all_reduce_grads(self, section: str, group=None):
        """Data-parallel tuning: sum the section's gradients over
        ranks with one flat RCCL all-reduce before the identical AdamW step."""
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(self.G[self.sec_off[section]:self.sec_end[section]], group=group)

    def weights_numpy(self) -> dict:
        """Master weights as reference-named float64 arrays."""
        p = self.P.detach().cpu().numpy().astype(np.float64)
        out = {s: {} for s in self.SECTIONS}
        shapes = {(sec, name): shp for sec, name, shp in W.blob_layout(self.H)[:-1]}
        for t in self.tensors:
            out[t["section"]][t["name"]] = p[t["offset"]:t["offset"] + t["n"]].reshape(
                shapes[(t["section"], t["name"])])
        return out


# ---------------------------------------------------------------------------
# host-side sequential logic of custom_loss / triplet_loss (train.py:13-40)
# ---------------------------------------------------------------------------
class TuneState:
    """train.py's module globals (PROTO_UPDATE_FACTOR, num_zero, num_ones) and
    model.prototype, per model instance."""

    def __init__(self, prototypes, factor=PROTO_UPDATE_FACTOR):
        self.protos = np.array(prototypes, dtype=np.float64)
        self.factor = float(factor)
        self.num_zero, self.num_ones = 1, 1

    def to_device(self, device):
        """[2K+3] fp64 = prototypes [K][2], factor, num_zero, num_ones (the
        layout pgp_tune_targets updates)."""
        v = np.concatenate([self.protos.reshape(-1), [self.factor, self.num_zero, self.num_ones]])
        return torch.tensor(v, dtype=torch.float64, device=device)

    def vector(self):
        """[2K+3] fp64 = prototypes [K][2], factor, num_zero, num_ones."""
        return np.concatenate([self.protos.reshape(-1), [self.factor, self.num_zero, self.num_ones]])

    def from_vector(self, v):
        K = (v.size - 3) // 2
        self.protos = np.array(v[:2 * K], dtype=np.float64).reshape(K, 2)
        self.factor = float(v[2 * K])
        self.num_zero, self.num_ones = int(v[2 * K + 1]), int(v[2 * K + 2])

    def from_device(self, t):
        v = t.cpu().numpy()
        K = (v.size - 3) // 2
        self.protos = v[:2 * K].reshape(K, 2).copy()
        self.factor = float(v[2 * K])
        self.num_zero, self.num_ones = int(v[2 * K + 1]), int(v[2 * K + 2])


def loss_targets(logits, protos, y, c, st: TuneState):
    """One window: CE weights, positive prototype targets, loss values; updates
    the prototype EMA and counters in reference order (train.py:27-40)."""
    H = logits.shape[0]
    mult = np.ones(H)
    tgt = np.zeros((H, 2))
    nz = no = 0
    aloss = 0.0
    for i in range(H):
        mult[i] = 1.0 if y[i] == 0 else st.num_zero / st.num_ones
        nz += 1
        no += 1 if y[i] == 1 else 0
        l = logits[i].astype(np.float64)
        m = l.max()
        aloss += (np.log(np.exp(l - m).sum()) + m - l[int(y[i])]) * mult[i]
    tloss = 0.0
    for i in range(H):
        if y[i] > 0:
            cc = int(c[i])
            a = protos[i].astype(np.float64)
            tgt[i] = st.protos[cc]
            pos = float(np.mean((a - st.protos[cc]) ** 2))
            negs = [float(np.mean((a - st.protos[nc]) ** 2)) for nc in (0, 1, 2) if nc != cc]
            tloss += pos - sum(negs)
            if pos <= negs[0] and pos <= negs[1]:
                f = st.factor + PROTO_UPDATE_MIN
                st.protos[cc] = f * a + (1 - f) * st.protos[cc]
    st.factor *= PROTO_FACTOR_DECAY
    st.num_zero += nz
    st.num_ones += no
    return mult, tgt, aloss, tloss


class TuneIncrements:
    """One rank's contribution to a data-parallel tuning step's host state
    (SURVEY §8e): prototype EMA deltas and counts per class, counter
    increments, windows seen.  Summed over ranks by ``dp_state_update``."""

    def __init__(self, K):
        self.delta = np.zeros((K, 2))
        self.count = np.zeros(K)
        self.num_zero = 0.0
        self.num_ones = 0.0
        self.windows = 0.0

    def flat(self):
        return np.concatenate([self.delta.reshape(-1), self.count, [self.num_zero, self.num_ones, self.windows]])

    @classmethod
    def from_flat(cls, v, K):
        t = cls(K)
        t.delta = v[:2 * K].reshape(K, 2).copy()
        t.count = v[2 * K:3 * K].copy()
        t.num_zero, t.num_ones, t.windows = (float(x) for x in v[3 * K:3 * K + 3])
        return t


def loss_targets_dp(logits, protos, y, c, st: TuneState):
    """Data-parallel form of loss_targets (train.py:27-40) for a local batch
    [B,H,...]: every window is scored against the step-START state (counters,
    prototypes, factor) instead of the state left by the previous window, and
    the state changes are returned as increments instead of applied:
    a qualifying (window, host) contributes f·(a − P[c]) to class c's delta
    (f = factor + PROTO_UPDATE_MIN), each window adds H to num_zero and its
    positives to num_ones.  With one window on one rank this is the reference's
    update exactly.  Returns (mult [B,H], tgt [B,H,2], aloss [B], tloss [B],
    TuneIncrements)."""
    B, H = logits.shape[0], logits.shape[1]
    K = st.protos.shape[0]
    inc = TuneIncrements(K)
    mult = np.where(np.asarray(y) == 0, 1.0, st.num_zero / st.num_ones)
    tgt = np.zeros((B, H, 2))
    aloss = np.zeros(B)
    tloss = np.zeros(B)
    f = st.factor + PROTO_UPDATE_MIN
    for b in range(B):
        for i in range(H):
            l = logits[b, i].astype(np.float64)
            m = l.max()
            aloss[b] += (np.log(np.exp(l - m).sum()) + m - l[int(y[b, i])]) * mult[b, i]
            if y[b, i] > 0:
                cc = int(c[b, i])
                a = protos[b, i].astype(np.float64)
                tgt[b, i] = st.protos[cc]
                pos = float(np.mean((a - st.protos[cc]) ** 2))
                negs = [float(np.mean((a - st.protos[nc]) ** 2)) for nc in (0, 1, 2) if nc != cc]
                tloss[b] += pos - sum(negs)
                if pos <= negs[0] and pos <= negs[1]:
                    inc.delta[cc] += f * (a - st.protos[cc])
                    inc.count[cc] += 1
        inc.num_zero += H
        inc.num_ones += float(np.sum(np.asarray(y[b]) == 1))
        inc.windows += 1
    return mult, tgt, aloss, tloss, inc


def dp_state_update(st: TuneState, inc: TuneIncrements, group=None):
    """Sum the increments over ranks (one all-reduce of 3K+3 doubles; a no-op
    without a process group) and apply them identically everywhere: counters
    += sums; each prototype moves by the MEAN of its qualifying deltas (so one
    update reproduces the reference's f·a + (1−f)·P); the factor decays once
    per window of the global batch (train.py:39)."""
    import torch.distributed as dist
    K = st.protos.shape[0]
    v = inc.flat()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor(v, dtype=torch.float64)
        if dist.get_backend(group) == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=group)
        v = t.cpu().numpy()
    tot = TuneIncrements.from_flat(v, K)
    upd = tot.count > 0
    st.protos[upd] += tot.delta[upd] / tot.count[upd][:, None]
    st.num_zero += tot.num_zero
    st.num_ones += tot.num_ones
    st.factor *= PROTO_FACTOR_DECAY ** tot.windows
    return tot


def dataset_buffers(tr: "Trainer", E: int, R: int = LATEST_WINDOW_SIZE, joint: bool = False):
    """Preallocated outputs of tune_dataset for E environments of R rows.
    With ``joint`` the tuning windows and run_encoder's windows are views of
    ONE [E*R + E, 3, 3H] buffer (returned fifth), so a single forward covers
    both (``DPTuner.step`` trains on the first E*R)."""
    H, dev = tr.H, tr.device
    if joint:
        allw = torch.empty((E * R + E, 3, 3 * H), dtype=torch.float32, device=dev)
        return (allw[:E * R], torch.empty((E * R, H), dtype=torch.int32, device=dev),
                torch.empty((E * R, H), dtype=torch.int32, device=dev), allw[E * R:], allw)
    return (torch.empty((E * R, 3, 3 * H), dtype=torch.float32, device=dev),
            torch.empty((E * R, H), dtype=torch.int32, device=dev),
            torch.empty((E * R, H), dtype=torch.int32, device=dev),
            torch.empty((E, 3, 3 * H), dtype=torch.float32, device=dev))


def tune_dataset(tr: "Trainer", series, train_max, infer: bool = True, out=None):
    """load_on_the_fly_dataset (utils.py:40-47) for a batch of environments on
    the device (``pgp_tune_dataset``): series [E,R,3H] fp64 (each environment's
    last R rows of stats.time_series), train_max [3H] fp64 = the training
    series' column max.  Returns windows [E*R,3,3H] fp32, y / cls [E*R,H] int32
    (form_test_dataset, utils.py:16-24) and run_encoder's window [E,3,3H] of the
    same rows (PreGANPlus.py:107-112) or None."""
    series = tr._dev(series, torch.float64)
    train_max = tr._dev(train_max, torch.float64)
    E, R, F = series.shape
    H = tr.H
    if F != 3 * H:
        raise ValueError(f"series must be [E,R,{3 * H}]")
    wins, y, cls, inf = out[:4] if out is not None else dataset_buffers(tr, E, R)
    if tuple(wins.shape) != (E * R, 3, F) or tuple(y.shape) != (E * R, H) or tuple(inf.shape) != (E, 3, F):
        raise ValueError("tune_dataset: output buffers do not match the series")
    inf = inf if infer else None
    _native.check(tr._L.pgp_tune_dataset(H, E, R, series.data_ptr(), train_max.data_ptr(), wins.data_ptr(),
                                         y.data_ptr(), cls.data_ptr(), None if inf is None else inf.data_ptr(),
                                         tr._stream()), "pgp_tune_dataset")
    return wins, y, cls, inf


class DPTuner:
    """The data-parallel tuning step with its state on the device (SURVEY §8e,
    config C3): forward, custom_loss / triplet_loss bookkeeping against the
    step-start state (``pgp_tune_targets_dp``), backward, ONE gradient
    all-reduce and ONE all-reduce of the 3K+3 fp64 state increments (device
    buffers, RCCL), the state update and AdamW from a device table
    (``pgp_tune_state_apply`` decides the prototype decoder's activity there).
    No host round trip: the step is launch-only.  ``loss_targets_dp`` /
    ``dp_state_update`` are the same semantics in numpy (the tests restate with
    them).  ``sync(st)`` copies the state back to a host ``TuneState`` and the
    AdamW step counts back to the Trainer."""

    COND = ("prototype_decoder.0.weight", "prototype_decoder.0.bias")
    CHUNK = 64   # AdamW table rows precomputed per upload

    def __init__(self, tr: "Trainer", st: TuneState, max_batch: int, group=None):
        self.tr, self.group = tr, group
        H, dev, L = tr.H, tr.device, tr._L
        self.K = st.protos.shape[0]
        tr._ensure(max_batch)
        self.cap = max_batch
        self.state = st.to_device(dev)
        self.mult = torch.zeros((max_batch, H), dtype=torch.float32, device=dev)
        self.tgt = torch.zeros((max_batch, H, 2), dtype=torch.float32, device=dev)
        self.loss = torch.zeros((max_batch, 2), dtype=torch.float64, device=dev)
        self.inc = torch.zeros(3 * self.K + 3, dtype=torch.float64, device=dev)
        self.ws = torch.zeros(max(int(L.pgp_tune_targets_dp_workspace_len(max_batch)), 1), dtype=torch.float64,
                              device=dev)
        self.sel = [t for t in tr.tensors if t["section"] == "transformer" and t["trainable"]]
        self.cond = [k for k, t in enumerate(self.sel) if t["name"] in self.COND]
        self.cond_rows = (ctypes.c_int * len(self.cond))(*self.cond)
        self.cond_steps = torch.tensor([self.sel[k]["step"] for k in self.cond], dtype=torch.float64, device=dev)
        self.base = [t["step"] for t in self.sel]
        self.n = 0
        self.table = torch.zeros((self.CHUNK, len(self.sel), 3), dtype=torch.float32, device=dev)

    def _fill_table(self):
        """Rows (active, lr/(1-b1^step), sqrt(1-b2^step)) of the next CHUNK
        steps for the always-active tensors (their step counts are known ahead);
        the prototype decoder's rows are written per step on the device."""
        tr = self.tr
        lr = tr.lrs["transformer"]
        tab = np.zeros((self.CHUNK, len(self.sel), 3), dtype=np.float32)
        for i in range(self.CHUNK):
            for k, b in enumerate(self.base):
                stp = max(b + self.n + i + 1, 1.0)
                tab[i, k] = (1.0, lr / (1 - tr.b1 ** stp), math.sqrt(1 - tr.b2 ** stp))
        self.table.copy_(torch.from_numpy(tab).pin_memory(), non_blocking=True)

    SUBSTAGES = ("forward", "targets", "backward", "all_reduce", "apply_adamw")

    def next_row(self, out: torch.Tensor | None = None):
        """The AdamW table row of the next step (host bookkeeping: the table is
        refilled every CHUNK steps).  With ``out`` (a fixed [T,3] device buffer
        that a captured step reads, ``step(row=out)``) the row is copied there
        on the current stream: call it before each replay."""
        i = self.n % self.CHUNK
        if i == 0:
            self._fill_table()
        self.n += 1
        row = self.table[i]
        if out is None:
            return row
        out.copy_(row)
        return out

    def step(self, wins: torch.Tensor, y: torch.Tensor, cls: torch.Tensor, mark=None, before_update=None,
             after_forward=None, before_backward=None, row: torch.Tensor | None = None, after_backward=None):
        """wins [B',3,3H] fp32, y / cls [B,H] int32, all on the device, B <= B':
        the forward runs over all B' windows and the step trains on the first
        B (windows B.. are inference windows sharing the forward, e.g. C3's
        detect: their logits / protos are ``tr.logits[B:B']`` afterwards).
        Returns the per-window (aloss, tloss) [B,2] fp64 device view.
        ``row``: the AdamW row buffer ``next_row(out=row)`` filled for this
        step (graph capture); by default the step takes ``next_row()`` itself.
        ``mark(k)``, if given, is called before sub-stage k of SUBSTAGES and
        once more at the end (the bench records HIP events there).
        ``before_update``, if given, is an event the step's stream waits for
        before the state update and AdamW (work on another stream that still
        reads the step-start weights), or a callable returning one, called at
        that point of the host's issue order (so the work it issues elsewhere
        is queued after this step's forward and backward).  ``after_forward``,
        if given, is called once the forward is issued (work for another stream
        that should queue behind the forward's launches but ahead of the
        backward's); ``before_backward``, if given, once the targets are issued,
        right before the backward (work for another stream that should start
        with the backward: the caller makes its stream wait for this one);
        ``after_backward``, if given, once the backward is issued (the same,
        issued after the backward's launches)."""
        mark = mark or (lambda k: None)
        import torch.distributed as dist
        tr, L = self.tr, self.tr._L
        B = y.shape[0]
        if B > self.cap or B > wins.shape[0] or cls.shape[0] != B:
            raise ValueError(f"batch {B} (labels) vs windows {wins.shape[0]} / DPTuner capacity {self.cap}")
        if y.dtype != torch.int32 or cls.dtype != torch.int32 or y.device != tr.device or cls.device != tr.device:
            raise ValueError("y / cls must be int32 device tensors")
        if row is None:
            row = self.next_row()
        s = tr._stream()
        mark(0)
        tr.tune_forward(wins)
        mark(1)
        if after_forward is not None:
            after_forward()
        _native.check(L.pgp_tune_targets_dp(
            tr.H, self.K, B, tr.logits.data_ptr(), tr.protos.data_ptr(), y.data_ptr(), cls.data_ptr(),
            self.state.data_ptr(), PROTO_UPDATE_MIN, self.mult.data_ptr(), self.tgt.data_ptr(), self.loss.data_ptr(),
            self.inc.data_ptr(), self.ws.data_ptr(), s), "pgp_tune_targets_dp")
        mark(2)
        if before_backward is not None:
            before_backward()
        tr.tune_backward(B, y, self.mult[:B], self.tgt[:B])
        if after_backward is not None:
            after_backward()
        mark(3)
        tr.all_reduce_grads("transformer", self.group)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(self.inc, group=self.group)
        mark(4)
        if before_update is not None:
            ev = before_update() if callable(before_update) else before_update
            torch.cuda.current_stream(tr.device).wait_event(ev)
        _native.check(L.pgp_tune_state_apply(
            self.K, self.state.data_ptr(), self.inc.data_ptr(), PROTO_FACTOR_DECAY, len(self.cond), self.cond_rows,
            self.cond_steps.data_ptr(), row.data_ptr(), tr.lrs["transformer"], tr.b1, tr.b2, s),
            "pgp_tune_state_apply")
        tr.adam_step_table("transformer", self.sel, row)
        mark(5)
        return self.loss[:B]

    def sync(self, st: TuneState):
        """State and AdamW step counts back to the host (one device sync)."""
        st.from_device(self.state)
        cs = self.cond_steps.cpu().numpy()
        for k, t in enumerate(self.sel):
            t["step"] = float(cs[self.cond.index(k)]) if k in self.cond else self.base[k] + self.n


def dp_tune_step(tr: "Trainer", st: TuneState, wins, anom, cls, group=None):
    """One data-parallel tuning step on this rank's windows,
    through ``DPTuner`` (device bookkeeping, device state): forward, targets
    against the step-start state, backward, one gradient all-reduce, the state
    increments all-reduced, AdamW.  The loss is the sum over the global batch.
    ``st`` is updated from the device afterwards.  Returns (aloss [B], tloss [B])."""
    wins = tr._dev(wins, torch.float32)
    B = wins.shape[0]
    tun = DPTuner(tr, st, B, group)
    loss = tun.step(wins, tr._dev(anom, torch.int32), tr._dev(cls, torch.int32))
    tun.sync(st)
    out = loss.cpu().numpy()
    return out[:, 0].copy(), out[:, 1].copy()


def normalize_test_time_data(time_data, train_time_data):
    """utils.py:94-95."""
    return np.asarray(time_data, dtype=np.float64) / (np.max(train_time_data, axis=0) + 1e-8)


def convert_to_windows(data, n_window=3):
    """utils.py:7-14: window i = rows i-n..i-1, row 0 repeated for i < n (one
    gather)."""
    data = np.asarray(data, dtype=np.float64)
    i = np.arange(data.shape[0])[:, None] - n_window + np.arange(n_window)[None, :]
    return data[np.maximum(i, 0)]


def percentile_linear(data, q):
    """np.percentile(data, q, axis=0) (method 'linear'), from one sort: numpy's
    virtual index (n-1)*q/100 and its lerp (b - (b-a)(1-g) for g >= 0.5, else
    a + (b-a) g), so the thresholds are bit-identical to numpy's."""
    n = data.shape[0]
    vi = (n - 1) * (q / 100.0)
    lo = np.floor(vi)
    gm = vi - lo
    ilo = int(lo)
    ihi = min(ilo + 1, n - 1)
    srt = np.sort(data, axis=0)
    a, b = srt[ilo], srt[ihi]
    d = b - a
    return b - d * (1.0 - gm) if gm >= 0.5 else a + d * gm


def form_test_dataset(data):
    """utils.py:16-24: per host (3 columns), anomalous if any column exceeds its
    98th percentile; class = first argmax of the 3 columns (vectorised over hosts)."""
    data = np.asarray(data)
    anomaly_per_dim = data > percentile_linear(data, PERCENTILES)
    R, F = data.shape
    anydim = anomaly_per_dim.reshape(R, F // 3, 3).any(axis=2)
    which = np.argmax(data.reshape(R, F // 3, 3), axis=2)
    return anydim + 0, which


def normalize_time_data(time_data):
    """utils.py:91-92: each column over its own maximum."""
    d = np.asarray(time_data, dtype=np.float64)
    return d / (np.max(d, axis=0) + 1e-8)


def load_dataset(time_data):
    """utils.py:36-42 (the offline training set of train_model) from the series
    the reference reads from data/<env>/time_series.npy: normalised over its
    own maxima, windows of every row, labels from the normalised series.  (The
    schedules it also loads do not enter the Transformer's backprop.)"""
    td = normalize_time_data(time_data)
    anom, cls = form_test_dataset(td)
    return convert_to_windows(td), anom, cls


def on_the_fly_dataset(time_series, schedule_series, train_time_data):
    """utils.py:40-47: the last 10 rows, normalised; windows and labels."""
    td = normalize_test_time_data(np.asarray(time_series)[-LATEST_WINDOW_SIZE:], train_time_data)
    sched = np.asarray(schedule_series)[-LATEST_WINDOW_SIZE:]
    anom, cls = form_test_dataset(td)
    return convert_to_windows(td), sched, anom, cls


FUSED_STEP_HOSTS = (8, 16)   # pgp_tune_step1's compiled host counts


class _TuneGraph:
    """One backprop() call of n sequential batch-1 steps captured as a HIP
    graph.  Per step, at 8 / 16 hosts: the fused step (``tune_step1``: forward,
    bookkeeping and backward in one workgroup) -> AdamW from a device table —
    2 launches; otherwise tune_forward -> tune_targets -> tune_backward
    (zero_grad + kernels) -> AdamW, ~45 launches.  With ``score``, the graph
    ends with the batched forward of accuracy() (train.py:94-109) on the
    updated weights.

    Host traffic per call: ONE upload of every input (windows, labels,
    classes, state, AdamW table) from a pinned staging buffer into the device
    buffer the graph reads, and ONE download of every output (losses, state,
    accuracy logits / prototypes, gathered into one fp64 buffer inside the
    graph)."""

    def __init__(self, tr: Trainer, n: int, win_shape, K: int, fused: bool | None = None, score: bool = False):
        H, dev = tr.H, tr.device
        if fused is None:
            fused = H in FUSED_STEP_HOSTS
        self.n, self.fused, self.score, self.K = n, fused, score, K
        self.sel = [t for t in tr.tensors if t["section"] == "transformer" and t["trainable"]]
        nw = int(np.prod(win_shape))
        # input staging: windows f32 | y i32 | cls i32 | AdamW table f32 | state f64 (8-byte aligned)
        parts = [("W", torch.float32, (n,) + tuple(win_shape)), ("Y", torch.int32, (n, H)),
                 ("C", torch.int32, (n, H)), ("sched", torch.float32, (n, len(self.sel), 3)),
                 ("state", torch.float64, (2 * K + 3,))]
        off, lay = 0, []
        for name, dt, shp in parts:
            nb = int(np.prod(shp)) * torch.tensor([], dtype=dt).element_size()
            off = (off + 7) // 8 * 8
            lay.append((name, dt, shp, off, nb))
            off += nb
        self.din = torch.zeros(off, dtype=torch.uint8, device=dev)
        self.hin = torch.zeros(off, dtype=torch.uint8).pin_memory()
        self.hviews = {}
        for name, dt, shp, o, nb in lay:
            setattr(self, name, self.din[o:o + nb].view(dt).view(shp))
            self.hviews[name] = self.hin[o:o + nb].view(dt).view(shp).numpy()
        # output gather: loss [n,2] | state [2K+3] | logits [n,H,2] | protos [n,H,2] (fp64)
        nout = 2 * n + 2 * K + 3 + (4 * n * H if score else 0)
        self.dout = torch.zeros(nout, dtype=torch.float64, device=dev)
        self.hout = torch.zeros(nout, dtype=torch.float64).pin_memory()
        self.loss = self.dout[:2 * n].view(n, 2)
        self.mult = torch.zeros((1, H), dtype=torch.float32, device=dev)
        self.tgt = torch.zeros((1, H, 2), dtype=torch.float32, device=dev)
        tr._ensure(n if score and not fused else 1)
        self.generation = tr.generation
        self.graph = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        with torch.cuda.graph(self.graph):
            for i in range(n):
                if fused:
                    tr.tune_step1(self.W[i], self.Y[i], self.C[i], self.state, self.loss[i])
                else:
                    tr.tune_forward(self.W[i:i + 1])
                    tr.tune_targets(self.Y[i], self.C[i], self.state, self.mult, self.tgt, self.loss[i])
                    tr.tune_backward(1, self.Y[i:i + 1], self.mult, self.tgt)
                tr.adam_step_table("transformer", self.sel, self.sched[i])
            o = 2 * n
            self.dout[o:o + 2 * K + 3].copy_(self.state)
            if score:
                o += 2 * K + 3
                if fused:  # one launch, fp64 straight into the gather buffer
                    tr.tune_forward_many(self.W, self.dout[o:o + 2 * n * H], self.dout[o + 2 * n * H:o + 4 * n * H])
                else:
                    lg, pr = tr.tune_forward(self.W)
                    self.dout[o:o + 2 * n * H].copy_(lg.reshape(-1))
                    self.dout[o + 2 * n * H:o + 4 * n * H].copy_(pr.reshape(-1))

    def launch(self, tr, wins, anom, cls, state_vec, tab, stream=None):
        """Upload, replay and download on ``stream`` (default: the current
        one) without waiting; ``wait()`` returns the gathered outputs."""
        hv = self.hviews
        hv["W"][...] = wins
        hv["Y"][...] = anom
        hv["C"][...] = cls
        hv["sched"][...] = tab
        hv["state"][...] = state_vec
        st = stream if stream is not None else torch.cuda.current_stream(tr.device)
        with torch.cuda.stream(st):
            self.din.copy_(self.hin, non_blocking=True)
            self.graph.replay()
            self.hout.copy_(self.dout, non_blocking=True)
        if getattr(self, "done", None) is None:
            self.done = torch.cuda.Event()
        self.done.record(st)

    def wait(self):
        self.done.synchronize()
        return self.hout.numpy()

    def run(self, tr, wins, anom, cls, state_vec, tab):
        self.launch(tr, wins, anom, cls, state_vec, tab)
        return self.wait()


def backprop(tr: Trainer, st: TuneState, wins, anom, cls, fused: bool | None = None, score: bool = False,
             stream=None, defer: bool = False):
    """train.py:42-57: sequential batch-1 steps (forward, custom_loss, backward,
    AdamW).  Returns the per-window (aloss, tloss); with ``score`` also
    accuracy()'s (AScore, CScore) of the updated model on the same windows
    (train.py:94-109, as tune_model calls it, PreGANPlus.py:56), computed in
    the same graph.

    Every step stays on the device: custom_loss's sequential bookkeeping runs
    in a kernel (state in fp64), AdamW's per-step scalars come from a table
    computed ahead on the host (``Trainer.adam_schedule``), and the n steps
    replay as one captured HIP graph (``_TuneGraph``, cached per shape).  The
    host uploads the inputs and reads back the results once per call.
    ``loss_targets`` is the same bookkeeping in numpy (the tests restate with
    it).

    With ``defer`` the graph is launched on ``stream`` (default: the current
    one) and a function is returned that waits for it and returns what
    backprop would (the plugin overlaps the tuning graph with train_gan's host
    simulation this way); the host state ``st`` is updated when it is called."""
    st.num_zero, st.num_ones = 1, 1
    wins = np.asarray(wins)
    n, H = wins.shape[0], tr.H
    if n == 0:
        res = ([], None) if score else []
        return (lambda: res) if defer else res
    anom = np.asarray(anom).reshape(n, H)
    cls = np.asarray(cls).reshape(n, H)
    bad = (anom > 0) & ((cls < 0) | (cls > 2))
    if bad.any():
        raise ValueError("anomalous host with a class outside 0..2 (triplet_loss, train.py:15-17)")
    K = st.protos.shape[0]
    if fused is None:
        fused = H in FUSED_STEP_HOSTS
    key = (n, wins.shape[1:], K, bool(fused), bool(score))
    g = tr._graphs.get(key)
    if g is None or g.generation != tr.generation:
        g = _TuneGraph(tr, n, wins.shape[1:], K, fused, score)
        tr._graphs[key] = g
    positive = np.any(anom > 0, axis=1)
    tab = tr.adam_schedule_np("transformer", positive, ("prototype_decoder.0.weight", "prototype_decoder.0.bias"))
    g.launch(tr, wins, anom, cls, st.vector(), tab, stream)

    def finish():
        out = g.wait()
        tr.tune_state_dev = g.state     # the updated state, on the device (prototypes first: the device repack)
        st.from_vector(out[2 * n:2 * n + 2 * K + 3])
        losses = [tuple(r) for r in out[:2 * n].reshape(n, 2).tolist()]
        if not score:
            return losses
        o = 2 * n + 2 * K + 3
        lg = out[o:o + 2 * n * H].reshape(n, H, 2)
        pr = out[o + 2 * n * H:o + 4 * n * H].reshape(n, H, 2)
        return losses, accuracy_scores(lg, pr, anom, cls, st.protos)

    return finish if defer else finish()


def bce_target(new_score, orig_score):
    """PreGANPlus.py:65-66: label [0,1] if the generator's schedule scores no
    worse than the original, else [1,0]."""
    return [0.0, 1.0] if new_score <= orig_score else [1.0, 0.0]


def bce(p, target):
    """nn.BCELoss (mean over the 2 probabilities, log clamped at -100), fp64."""
    p = np.asarray(p, dtype=np.float64)
    t = np.asarray(target, dtype=np.float64)
    lp = np.maximum(np.log(p), -100.0)
    l1p = np.maximum(np.log(1.0 - p), -100.0)
    return float(-np.mean(t * lp + (1 - t) * l1p))


def train_gan_eager(tr: Trainer, emb, sched, simulate):
    """PreGANPlus.py:60-75 (one window) as individual launches with host
    round trips.  simulate(schedule ndarray) -> score.  Returns (ns,
    new_score, orig_score, gen_loss, disc_loss).  ``train_gan`` is the same
    sequence replayed from two captured graphs (the tests hold them equal)."""
    ns, probs = tr.gan_forward(np.asarray(emb)[None], np.asarray(sched)[None])
    ns_h = ns[0].cpu().numpy().astype(np.float64)
    p_d = probs[0].cpu().numpy()
    new_score, orig_score = simulate(ns_h), simulate(np.asarray(sched, dtype=np.float64))
    target = bce_target(new_score, orig_score)
    tr.gan_disc_backward(np.array([target]))
    tr.adam_step("disc")
    tr.gan_gen_backward(1)
    p_g = tr.gan_probs(1)[0].cpu().numpy()
    tr.adam_step("gen")
    return ns_h, new_score, orig_score, bce(p_g, [0.0, 1.0]), bce(p_d, target)


class _GanGraph:
    """train_gan for one window as two captured graphs around the host
    simulator call (PreGANPlus.py:62-66 scores the generator's schedule with
    the environment's simulator, a host object):
      A: Gen + Disc forward (the new schedule and the Disc probabilities);
      B: Disc BCE backward + AdamW, Gen backward + the Disc probabilities it
         saw + AdamW, then the updated GAN's forward on the same inputs (the
         gate recover_decision reads, PreGANPlus.py:84-87: tune_model does not
         touch the GAN, so it is computed here).
    Each graph has one upload (pinned staging -> device) and one download.
    At 8 / 16 hosts (``fused``, the default there) each graph is ONE launch:
    ``pgp_gan_forward1`` and ``pgp_gan_step1`` (csrc/pgp_gan1.hip)."""

    def __init__(self, tr: Trainer, fused: bool | None = None):
        H, dev = tr.H, tr.device
        self.generation_in = tr.generation
        tr._ensure(1)
        self.generation = tr.generation
        self.selD = [t for t in tr.tensors if t["section"] == "disc" and t["trainable"]]
        self.selG = [t for t in tr.tensors if t["section"] == "gen" and t["trainable"]]
        nA = 2 * H + H * H
        nB = 2 + 3 * len(self.selD) + 3 * len(self.selG)
        self.nA, self.nB = nA, nB
        self.din = torch.zeros(nA + nB, dtype=torch.float32, device=dev)
        self.hin = torch.zeros(nA + nB, dtype=torch.float32).pin_memory()
        nout = H * H + 2 + 2 + 2
        self.dout = torch.zeros(nout, dtype=torch.float32, device=dev)
        self.hout = torch.zeros(nout, dtype=torch.float32).pin_memory()
        emb = self.din[:2 * H].view(1, 2 * H)
        sch = self.din[2 * H:nA].view(1, H, H)
        tgt = self.din[nA:nA + 2].view(1, 2)
        o = nA + 2
        tabD = self.din[o:o + 3 * len(self.selD)].view(len(self.selD), 3)
        tabG = self.din[o + 3 * len(self.selD):].view(len(self.selG), 3)
        HH = H * H
        torch.cuda.synchronize(dev)
        self.gA, self.gB = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        self.fused = (H in FUSED_STEP_HOSTS) if fused is None else fused
        if self.fused:  # two single-workgroup launches (pgp_gan_forward1 / pgp_gan_step1)
            with torch.cuda.graph(self.gA):
                tr.gan_forward1(emb.reshape(-1), sch.reshape(-1), self.dout[:HH], self.dout[HH:HH + 2])
            with torch.cuda.graph(self.gB):
                tr.gan_step1(tgt.reshape(-1), self.selD, tabD, self.selG, tabG, self.dout[HH + 2:HH + 4],
                             self.dout[HH + 4:HH + 6])
            return
        with torch.cuda.graph(self.gA):
            ns, probs = tr.gan_forward(emb, sch)
            self.dout[:HH].copy_(ns.reshape(-1))
            self.dout[HH:HH + 2].copy_(probs.reshape(-1))
        with torch.cuda.graph(self.gB):
            tr.gan_disc_backward(tgt)
            tr.adam_step_table("disc", self.selD, tabD)
            tr.gan_gen_backward(1)
            self.dout[HH + 2:HH + 4].copy_(tr.gan_probs(1).reshape(-1))
            tr.adam_step_table("gen", self.selG, tabG)
            _, probs = tr.gan_forward(emb, sch)
            self.dout[HH + 4:HH + 6].copy_(probs.reshape(-1))

    def forward(self, tr, emb, sched):
        H = tr.H
        h = self.hin.numpy()
        h[:2 * H] = np.asarray(emb, dtype=np.float32).reshape(-1)
        h[2 * H:self.nA] = np.asarray(sched, dtype=np.float32).reshape(-1)
        self.din[:self.nA].copy_(self.hin[:self.nA], non_blocking=True)
        self.gA.replay()
        self.hout[:H * H + 2].copy_(self.dout[:H * H + 2], non_blocking=True)
        torch.cuda.current_stream(tr.device).synchronize()
        o = self.hout.numpy()
        return o[:H * H].reshape(H, H).astype(np.float64), o[H * H:H * H + 2].copy()

    def step(self, tr, target):
        h = self.hin.numpy()
        nA = self.nA
        h[nA:nA + 2] = target
        tabD = tr.adam_schedule_np("disc", [True], ())
        tabG = tr.adam_schedule_np("gen", [True], ())
        o = nA + 2
        h[o:o + tabD.size] = tabD.reshape(-1)
        h[o + tabD.size:o + tabD.size + tabG.size] = tabG.reshape(-1)
        self.din[nA:].copy_(self.hin[nA:], non_blocking=True)
        self.gB.replay()
        HH = tr.H * tr.H
        self.hout[HH + 2:].copy_(self.dout[HH + 2:], non_blocking=True)
        torch.cuda.current_stream(tr.device).synchronize()
        out = self.hout.numpy()
        return out[HH + 2:HH + 4].copy(), out[HH + 4:HH + 6].copy()


def train_gan(tr: Trainer, emb, sched, simulate, fused: bool | None = None):
    """PreGANPlus.py:60-75 (one window).  simulate(schedule ndarray) -> score.
    Returns (ns, new_score, orig_score, gen_loss, disc_loss); the updated
    GAN's Disc probabilities on the same (emb, sched) — recover_decision's
    gate — are left in ``tr.gan_probs_after``.  Two graph replays
    (``_GanGraph``) around the two simulator calls."""
    g = getattr(tr, "_gan_graph", None)
    want = (tr.H in FUSED_STEP_HOSTS) if fused is None else fused
    if g is None or g.generation != tr.generation or g.fused != want:
        g = tr._gan_graph = _GanGraph(tr, want)
    ns_h, p_d = g.forward(tr, emb, sched)
    new_score, orig_score = simulate(ns_h), simulate(np.asarray(sched, dtype=np.float64))
    target = bce_target(new_score, orig_score)
    p_g, p_after = g.step(tr, target)
    tr.gan_probs_after = p_after
    return ns_h, new_score, orig_score, bce(p_g, [0.0, 1.0]), bce(p_d, target)


def accuracy(tr: Trainer, st: TuneState, wins, anom, cls):
    """train.py:94-109 after a tuning call (PreGANPlus.py:56): the updated model
    on the same windows (one batched forward: pgp_tune_forward_many at 8 / 16
    hosts, else pgp_tune_forward), then the
    reference's per-window scores (``accuracy_scores``).  Returns (AScore,
    CScore).  ``backprop(..., score=True)`` computes the same inside the tuning
    graph."""
    wins = np.asarray(wins)
    n, H = wins.shape[0], tr.H
    if H in FUSED_STEP_HOSTS:  # the fused forward, as backprop(score=True)'s graph runs it
        w = torch.as_tensor(wins, dtype=torch.float32).to(tr.device).contiguous()
        out = torch.empty(4 * n * H, dtype=torch.float64, device=tr.device)
        tr.tune_forward_many(w, out[:2 * n * H], out[2 * n * H:])
        o = out.cpu().numpy()
        lg, pr = o[:2 * n * H].reshape(n, H, 2), o[2 * n * H:].reshape(n, H, 2)
    else:
        logits, protos = tr.tune_forward(torch.as_tensor(wins, dtype=torch.float32))
        lg = logits[:n].cpu().numpy().astype(np.float64)
        pr = protos[:n].cpu().numpy().astype(np.float64)
    return accuracy_scores(lg, pr, anom, cls, st.protos)


def accuracy_scores(lg, pr, anom, cls, P):
    """The reference's per-window scores in its order — anomaly_accuracy
    (train.py:60-73, the fraction of hosts whose argmax matches the label) and
    class_accuracy (:75-92, positives closer to their class prototype than to
    both others, over 1e-4 + positives) — from the forward's logits / protos
    [n,H,2] and prototypes P.  Like the reference it raises ZeroDivisionError
    when no window of the set has a positive label (class_total = 0,
    train.py:109)."""
    n, H = lg.shape[0], lg.shape[1]
    anom = np.asarray(anom).reshape(n, H)
    cls = np.asarray(cls).reshape(n, H).astype(np.int64)
    P = np.asarray(P, dtype=np.float64)
    res = (lg[:, :, 1] > lg[:, :, 0]).astype(np.int64)           # torch.argmax, ties -> 0
    per_window = np.sum(res == anom, axis=1)
    # class distances of every host to prototypes 0-2: MSE over the 2 dims
    dist = np.mean((pr[:, :, None, :] - P[None, None, :3, :]) ** 2, axis=-1)   # [n, H, 3]
    c = np.clip(cls, 0, 2)
    pos = np.take_along_axis(dist, c[..., None], axis=-1)[..., 0]
    n0 = np.where(c == 0, dist[..., 1], dist[..., 0])                 # negatives in class order
    n1 = np.where(c == 2, dist[..., 1], dist[..., 2])
    hit = (anom > 0) & (pos <= n0) & (pos <= n1)
    anomaly_correct, class_correct, class_total = 0, 0, 0
    for i in range(n):                                                 # the reference's accumulation order
        anomaly_correct += int(per_window[i]) / H
        npos = int(np.sum(anom[i] > 0))
        if np.sum(anom[i]) > 0:
            class_total += 1
            total = 1e-4
            for _ in range(npos):
                total += 1
            class_correct += int(np.sum(hit[i])) / total
    return anomaly_correct / n, class_correct / class_total


def dp_groups():
    """Process groups of the data-parallel C3 step: (tuning group,
    GAN group).  At world size > 1 the GAN step's gradient all-reduces get a
    communicator of their own: the GAN step runs on a second stream beside the
    tuning step, and collectives that share one communicator run in issue
    order on its one internal stream, so the GAN's Disc all-reduce would wait
    for the tuning backward and its gradient all-reduce (the two streams'
    overlap would collapse).  With two communicators each chain waits only for
    its own peers.  Both groups span all ranks and are created in the same
    order on every rank (torch.distributed.new_group is collective).
    (None, None) without a process group or at world size 1."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return None, None
    return None, dist.new_group(ranks=list(range(dist.get_world_size())))


class SectionRows:
    """AdamW's per-step scalars for a section whose tensors all step on every
    call (the GAN's Gen and Disc: both sections get a gradient each
    train_gan), for a captured step: ``next_row(out)`` (host, before each
    replay) writes the next step's row into the fixed buffer the graph's
    ``adam_step_table`` reads and advances the host step counts as
    ``adam_step`` would.  A table of CHUNK rows is filled ahead on the host and
    uploaded once per CHUNK steps (same values as adam_step)."""

    CHUNK = 64

    def __init__(self, tr: Trainer, section: str):
        self.tr, self.section = tr, section
        self.sel = [t for t in tr.tensors if t["section"] == section and t["trainable"]]
        self.table = torch.zeros((self.CHUNK, len(self.sel), 3), dtype=torch.float32, device=tr.device)
        self.i = 0

    def buffer(self):
        return torch.zeros((len(self.sel), 3), dtype=torch.float32, device=self.tr.device)

    def next_row(self, out: torch.Tensor | None = None):
        """The next step's row: a view of the table, or copied into ``out``."""
        if self.i % self.CHUNK == 0:
            tab = self.tr.adam_schedule_np(self.section, np.ones(self.CHUNK, dtype=bool), ())
            for t in self.sel:            # adam_schedule_np advanced the counts by CHUNK; one step at a time here
                t["step"] -= self.CHUNK
            self.table.copy_(torch.from_numpy(tab).pin_memory(), non_blocking=True)
        row = self.table[self.i % self.CHUNK]
        self.i += 1
        for t in self.sel:
            t["step"] += 1
        if out is None:
            return row
        out.copy_(row)
        return out


def train_gan_batched(tr: Trainer, sim, envs, emb, sched, out=None, target=None, all_reduce=False, group=None,
                      rows=None):
    """PreGANPlus.py:60-75 for a batch of environments with the label simulated
    on the device (``simulate.Simulation`` -> ``pgp_simulate``):
    Gen + Disc forward, both schedules scored, Disc BCE step on the label, Gen
    BCE step toward [0, 1] — no host round trip.  envs [B, env_len(H)] fp64
    records (``simulate.pack_env``).  With ``all_reduce`` each section's
    gradients are summed over ranks before its AdamW step (data parallel).
    ``rows`` = (disc row, gen row): AdamW reads its per-step scalars from
    these device buffers (``SectionRows.next_row``, graph capture) instead of
    kernel arguments.
    Returns (out [B,4] energy/score of new and original, target [B,2])."""
    ns, _ = tr.gan_forward(emb, sched)
    out, target = sim.score(envs, ns, tr._gan_in[1], out=out, target=target)
    tr.gan_disc_backward(target)
    if all_reduce:
        tr.all_reduce_grads("disc", group)
    if rows is None:
        tr.adam_step("disc")
    else:
        tr.adam_step_table("disc", tr.trainable("disc"), rows[0])
    tr.gan_gen_backward(ns.shape[0])
    if all_reduce:
        tr.all_reduce_grads("gen", group)
    if rows is None:
        tr.adam_step("gen")
    else:
        tr.adam_step_table("gen", tr.trainable("gen"), rows[1])
    return out, target

class _OnlineTensor(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_longlong), ("n", ctypes.c_int), ("section", ctypes.c_int),
                ("cond", ctypes.c_int), ("step", ctypes.c_double)]


_vp, _dp = ctypes.c_void_p, ctypes.c_double


class _OnlineDesc(ctypes.Structure):
    """pgp_online_desc (include/preganplus.h)."""
    _fields_ = ([(n, ctypes.c_int) for n in ("n_hosts", "n_env", "n_rows", "n_protos")]
                + [(n, _vp) for n in ("series", "train_max", "sched", "envs", "P", "G", "exp_avg", "exp_avg_sq",
                                      "tune_ws", "logits", "protos", "windows", "y", "cls", "state", "mult", "tgt",
                                      "loss", "inc", "dp_ws", "adam_rows", "cond_steps", "gan_ws", "ns", "probs",
                                      "emb", "sim_out", "target")]
                + [("tensors", ctypes.POINTER(_OnlineTensor)), ("n_tensors", ctypes.c_int), ("n_cond", ctypes.c_int),
                   ("lr", _dp * 3)]
                + [(n, _dp) for n in ("weight_decay", "beta1", "beta2", "eps", "update_min", "decay")])


_COLL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p)
ONLINE_STAGES = ("dataset", "embedding", "train_gan", "tune_model", "forward", "targets", "backward", "exchange",
                 "apply_adamw", "main")


def _bind_online(L):
    if getattr(L, "_pgp_online_bound", False):
        return
    L.pgp_online_create.argtypes = [ctypes.POINTER(_OnlineDesc), ctypes.POINTER(ctypes.c_void_p)]
    L.pgp_online_destroy.argtypes = [ctypes.c_void_p]
    L.pgp_online_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _COLL_FN, ctypes.c_void_p]
    L.pgp_online_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.pgp_online_stage_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.pgp_online_steps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.pgp_online_gan_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.pgp_online_issue_worker.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for f in ("pgp_online_create", "pgp_online_destroy", "pgp_online_step", "pgp_online_timing",
              "pgp_online_stage_ms", "pgp_online_steps", "pgp_online_gan_step", "pgp_online_issue_worker"):
        getattr(L, f).restype = ctypes.c_int
    L._pgp_online_bound = True


def _destroy_online(L, h):
    try:
        L.pgp_online_destroy(h)
    except Exception:
        pass


class OnlineTrainStep:
    """run_model's semi-supervised training (PreGANPlus.py:115-136, all but the
    decision) for E environments on this rank, data parallel,
    as one launch-only step on the device:
      1. tune_model's on-the-fly dataset (utils.py:40-47, ``pgp_tune_dataset``):
         each environment's last R rows -> R tuning windows with labels and
         classes, and run_encoder's window (PreGANPlus.py:107-112) — the latter
         as the last E rows of the same window buffer;
      2. ONE Transformer forward over the R*E + E windows (the tuning windows
         and detect's read the same step-start weights), then the tuning
         bookkeeping over the first R*E (``DPTuner``);
      3. on the second stream ``side``: detect's masked embedding
         (PreGANPlus.py:129) and train_gan (PreGANPlus.py:60-81, ``
         train_gan_batched``: device-simulated label, Disc step, Gen step);
      4. the tuning backward over the R*E windows, gradient / state all-reduce,
         state update and AdamW (``DPTuner``).
    The GAN and tuning steps share no data, so 3 runs beside 4.

    ``native`` (default): ``run()`` issues the whole step from ONE C-ABI call
    (``pgp_online_step``, csrc/pgp_online.hip): the launches, the stream
    fork / join and AdamW's per-step scalars (from step counts the library
    keeps, ``sync()`` copies them back to the Trainer) come from C++, and the
    data-parallel exchange calls back into ``_collective`` (torch.distributed
    on the step's streams and groups) at its four points.
    ``native=False``: the same step composed from the per-op calls in Python
    (``issue()``; AdamW's scalars from fixed device rows written by
    ``prep()``, so ``capture()`` can record it once as a HIP graph that
    ``run()`` replays at world size 1) — the reference composition the native
    step is tested against.  ``issue()`` takes optional ``stage`` / ``sub``
    HIP-event lists as bench.py records them."""

    def __init__(self, tr: "Trainer", st: "TuneState", sim, series, train_max, sched, envs, R: int = 10,
                 side=None, groups=(None, None), out=None, native: bool = True):
        self.tr, self.sim, self.st = tr, sim, st
        self.series, self.tmax = tr._dev(series, torch.float64), tr._dev(train_max, torch.float64)
        E = self.series.shape[0]
        self.E, self.R, self.B = E, R, E * R
        H, dev = tr.H, tr.device
        tr._ensure(self.B + E)
        self.tun = DPTuner(tr, st, self.B, group=groups[0])
        self.gan_group = groups[1]
        self.sched = tr._dev(sched, torch.float32)
        self.envs = tr._dev(envs, torch.float64)
        self.bufs = dataset_buffers(tr, E, R, joint=True)
        self.emb = torch.zeros((E, H, 2), dtype=torch.float32, device=dev)
        self.sim_out = torch.zeros((E, 4), dtype=torch.float64, device=dev)
        self.target = torch.zeros((E, 2), dtype=torch.float32, device=dev)
        self.side = side
        self.rowT = torch.zeros_like(self.tun.table[0])
        self.rows_d, self.rows_g = SectionRows(tr, "disc"), SectionRows(tr, "gen")
        self.rowD, self.rowG = self.rows_d.buffer(), self.rows_g.buffer()
        self._rows = (self.rowT, self.rowD, self.rowG)
        self.graph = None
        self._gate = torch.cuda.Event()   # the forward is issued: the GAN stream may start
        self.native = bool(native)
        self._h = None
        if self.native:
            self._create_native(sim)

    # -- the native step (pgp_online_*) --
    def _create_native(self, sim):
        tr, tun, L = self.tr, self.tun, self.tr._L
        _bind_online(L)
        H, E, R, B = tr.H, self.E, self.R, self.B
        wins, y, cls, _, allw = self.bufs
        sel = [t for t in tr.tensors if t["trainable"]]
        secs = {"transformer": 0, "gen": 1, "disc": 2}
        self._tensors = (_OnlineTensor * len(sel))(*[
            _OnlineTensor(t["offset"], t["n"], secs[t["section"]], int(t["name"] in DPTuner.COND and
                                                                       t["section"] == "transformer"), t["step"])
            for t in sel])
        self._sel = sel
        self.ns = torch.zeros((E, H, H), dtype=torch.float32, device=tr.device)
        self.probs = torch.zeros((E, 2), dtype=torch.float32, device=tr.device)
        self.gscr = torch.zeros((L.pgp_gan_workspace_len(H, E),), dtype=torch.float32, device=tr.device)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())
        d = _OnlineDesc()
        d.n_hosts, d.n_env, d.n_rows, d.n_protos = H, E, R, tun.K
        for name, t in (("series", self.series), ("train_max", self.tmax), ("sched", self.sched), ("envs", self.envs),
                        ("P", tr.P), ("G", tr.G), ("exp_avg", tr.m), ("exp_avg_sq", tr.v), ("tune_ws", tr.ws),
                        ("logits", tr.logits), ("protos", tr.protos), ("windows", allw), ("y", y), ("cls", cls),
                        ("state", tun.state), ("mult", tun.mult), ("tgt", tun.tgt), ("loss", tun.loss),
                        ("inc", tun.inc), ("dp_ws", tun.ws), ("adam_rows", self.rowT),
                        ("cond_steps", tun.cond_steps), ("gan_ws", self.gscr), ("ns", self.ns),
                        ("probs", self.probs), ("emb", self.emb), ("sim_out", self.sim_out),
                        ("target", self.target)):
            setattr(d, name, ptr(t))
        d.tensors = self._tensors
        d.n_tensors = len(sel)
        d.n_cond = len(tun.cond)
        d.lr = (_dp * 3)(tr.lrs["transformer"], tr.lrs["gen"], tr.lrs["disc"])
        d.weight_decay, d.beta1, d.beta2, d.eps = tr.wd, tr.b1, tr.b2, tr.eps
        d.update_min, d.decay = PROTO_UPDATE_MIN, PROTO_FACTOR_DECAY
        if tr.cap < B + E or L.pgp_tune_workspace_len(H, B + E) > tr.ws.numel():
            raise ValueError("trainer workspace smaller than the step's batch")
        h = ctypes.c_void_p()
        _native.check(L.pgp_online_create(ctypes.byref(d), ctypes.byref(h)), "pgp_online_create")
        self._desc, self._h = d, h
        self._fin = __import__("weakref").finalize(self, _destroy_online, L, h)
        self._err = None
        import torch.distributed as dist
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self._cb = _COLL_FN(self._collective) if multi else _COLL_FN()
        self._timing = False

    def _collective(self, user, which, stream):
        """pgp_online_step's exchange points (include/preganplus.h
        PGP_COLL_*): the section's gradients (Disc, Gen: the GAN group, on the
        GAN stream; Transformer: the tuning group, on the main stream) or the
        state increments, summed over ranks in place."""
        import torch.distributed as dist
        try:
            tr, tun = self.tr, self.tun
            if which in (0, 1):
                sec, grp, st = ("disc" if which == 0 else "gen"), self.gan_group, self._streams[1]
                buf = tr.G[tr.sec_off[sec]:tr.sec_end[sec]]
            else:
                grp, st = tun.group, self._streams[0]
                buf = tr.G[tr.sec_off["transformer"]:tr.sec_end["transformer"]] if which == 2 else tun.inc
            with torch.cuda.stream(st):
                dist.all_reduce(buf, group=grp)
            return 0
        except BaseException as e:   # surfaced by run() after the C call returns
            self._err = e
            return -1

    def issue_worker(self, on: bool):
        """World size 1, two streams: issue the GAN stream's launches from the
        library's second host thread while this one issues the tuning backward
        (the default; off: one thread issues both)."""
        _native.check(self.tr._L.pgp_online_issue_worker(self._h, int(on)), "pgp_online_issue_worker")

    def timing(self, on: bool):
        """Record HIP events in the native steps that follow (stage_ms())."""
        _native.check(self.tr._L.pgp_online_timing(self._h, int(on)), "pgp_online_timing")
        self._timing = bool(on)

    def stage_ms(self) -> dict:
        """The last native step's spans in ms (ONLINE_STAGES)."""
        ms = (ctypes.c_float * len(ONLINE_STAGES))()
        _native.check(self.tr._L.pgp_online_stage_ms(self._h, ms), "pgp_online_stage_ms")
        return dict(zip(ONLINE_STAGES, list(ms)))

    def gan_step(self):
        """The step's GAN part alone on the current stream (pgp_online_gan_step:
        train_gan for the E environments from the last forward's detect rows,
        world size 1), as the native step runs it on its GAN stream."""
        st = torch.cuda.current_stream(self.tr.device)
        _native.check(self.tr._L.pgp_online_gan_step(self._h, ctypes.c_void_p(st.cuda_stream)),
                      "pgp_online_gan_step")

    def sync(self):
        """The step's AdamW step counts back into the Trainer's tensor records
        (native: from the library's counts, the prototype decoder's from the
        device) and the tuning state (prototypes, factor, counters) into the
        TuneState the step was built with.  Native steps do not advance the
        DPTuner's host bookkeeping, so its base is re-anchored at the synced
        counts: a later ``tun.sync(st)`` or Python-composed step continues from
        them instead of resetting them."""
        tun = self.tun
        if not self.native:
            tun.sync(self.st)
            return
        n = len(self._sel)
        out = (ctypes.c_double * n)()
        _native.check(self.tr._L.pgp_online_steps(self._h, out, n), "pgp_online_steps")
        cs = tun.cond_steps.cpu().numpy()
        tsel = tun.sel
        for t, v in zip(self._sel, out):
            t["step"] = float(cs[tun.cond.index(tsel.index(t))]) if v < 0 else float(v)
        self.st.from_device(tun.state)
        tun.base = [t["step"] for t in tun.sel]
        tun.n = 0

    def prep(self):
        """Host bookkeeping of the next step (AdamW rows).  Eager steps read
        the rows straight from the tables; a captured step reads the fixed
        buffers, so the rows are copied there (on the current stream)."""
        if self.graph is None:
            self._rows = (self.tun.next_row(), self.rows_d.next_row(), self.rows_g.next_row())
        else:
            self._rows = (self.tun.next_row(out=self.rowT), self.rows_d.next_row(self.rowD),
                          self.rows_g.next_row(self.rowG))

    def issue(self, stage=None, sub=None):
        if self.native:
            raise RuntimeError("native OnlineTrainStep: run() issues the step (construct with native=False "
                               "for the Python composition)")
        from .model import embedding
        tr, B, E = self.tr, self.B, self.E
        main = torch.cuda.current_stream(tr.device)
        side = self.side if self.side is not None else main
        rec = (lambda k: stage[k].record(main)) if stage is not None else (lambda k: None)
        rec(0)
        _, y, cls, _ = tune_dataset(tr, self.series, self.tmax, out=self.bufs)
        rec(1)

        gate = self._gate

        def detect_gan():   # once the forward is issued: beside the targets and the tuning backward
            gate.record(main)
            side.wait_event(gate)
            with torch.cuda.stream(side):
                if stage is not None:
                    stage[5].record(side)
                embedding(tr.logits[B:B + E], tr.protos[B:B + E], out=self.emb)
                if stage is not None:
                    stage[2].record(side)
                train_gan_batched(tr, self.sim, self.envs, self.emb, self.sched, out=self.sim_out,
                                  target=self.target, all_reduce=True, group=self.gan_group,
                                  rows=self._rows[1:])
                if stage is not None:
                    stage[3].record(side)

        self.tun.step(self.bufs[4], y, cls, mark=(lambda k: sub[k].record(main)) if sub is not None else None,
                      after_forward=detect_gan, row=self._rows[0])
        main.wait_stream(side)
        rec(4)

    def capture(self):
        """Record one step (the Python composition) as a HIP graph on the
        current (non-default) stream."""
        if self.native:
            raise RuntimeError("capture() records the Python composition (native=False)")
        main = torch.cuda.current_stream(self.tr.device)
        torch.cuda.synchronize(self.tr.device)
        g = torch.cuda.CUDAGraph()
        self._rows = (self.rowT, self.rowD, self.rowG)
        with torch.cuda.graph(g, stream=main):
            self.issue()
        torch.cuda.synchronize(self.tr.device)
        self.graph = g

    def run(self):
        if self.native:
            main = torch.cuda.current_stream(self.tr.device)
            side = self.side if self.side is not None else main
            self._streams = (main, side)
            rc = self.tr._L.pgp_online_step(self._h, ctypes.c_void_p(main.cuda_stream),
                                            ctypes.c_void_p(side.cuda_stream), self._cb, None)
            if self._err is not None:
                e, self._err = self._err, None
                raise RuntimeError("pgp_online_step: collective failed") from e
            _native.check(rc, "pgp_online_step")
            return
        self.prep()
        if self.graph is not None:
            self.graph.replay()
        else:
            self.issue()
