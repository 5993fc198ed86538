"""Offline training of PreGAN's FPE_16 encoder on MI355X (PreGAN.py:26-27,
39-49): with no FPE checkpoint the reference creates a new FPE_16 and trains it
for num_epochs (train.py:42-57 backprop + :94-109 accuracy over utils.py:36-42
load_dataset's series, AdamW lr 1e-4 weight decay 1e-5, models.py:14), saving
the checkpoint after every epoch; the encoder is then frozen.  The reference's
framework environment ships no FPE checkpoint, so this is the path it takes
there.

Every step runs on the device: ``pgp_fpe_train_step`` (forward, custom_loss /
triplet_loss bookkeeping on the device state in fp64, full backward, one
workgroup; csrc/pgp_fpetrain.hip) then ``pgp_adamw`` with torch's semantics.
The GRU state the reference draws inside every forward (torch.randn,
models.py:70) is drawn here by the same call in the same order (backprop's N,
then accuracy's N per epoch), so a seeded run reproduces the reference's."""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _native
from . import weights as W
from .train import PROTO_FACTOR_DECAY, PROTO_UPDATE_MIN, TuneState, _AdamTensor, accuracy_scores

FPE_LR = 1e-4          # FPE_16.lr (models.py:14)
COND = ("prototype_decoder.0.weight", "prototype_decoder.0.bias")   # no gradient without a positive label


class FPETrainer:
    """fp32 master weights, gradients and AdamW moments of FPE_16 on the device,
    in state_dict order (weights.fpe_shapes)."""

    def __init__(self, fpe: dict, device="cuda", state: dict | None = None, weight_decay=1e-5,
                 betas=(0.9, 0.999), eps=1e-8, H=16):
        self.H = H
        self.device = torch.device(device)
        L = _native.lib()
        self._L = L
        if not getattr(L, "_pgp_fpetrain_bound", False):
            vp, i32, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
            L.pgp_fpe_param_len.argtypes = [i32]
            L.pgp_fpe_param_len.restype = ctypes.c_size_t
            L.pgp_fpe_train_step.argtypes = [i32, i32] + [vp] * 7 + [dbl, dbl, vp, vp]
            L.pgp_fpe_train_step.restype = i32
            L.pgp_fpe_forward_many.argtypes = [i32, i32] + [vp] * 5 + [vp]
            L.pgp_fpe_forward_many.restype = i32
            L.pgp_adamw.argtypes = [vp] * 4 + [ctypes.c_float] * 5 + [ctypes.POINTER(_AdamTensor), i32, vp]
            L.pgp_adamw.restype = i32
            L._pgp_fpetrain_bound = True
        n = int(L.pgp_fpe_param_len(H))
        if n == 0:
            raise ValueError(f"FPE training: H={H} not supported (FPE_16 only)")
        shapes = W.fpe_shapes(H)
        self.tensors, off = [], 0
        for name, shp in shapes.items():
            cnt = int(np.prod(shp))
            self.tensors.append({"name": name, "shape": shp, "offset": off, "n": cnt, "step": 0.0})
            off += cnt
        assert off == n, (off, n)
        blob = np.concatenate([np.asarray(fpe[k], dtype=np.float64).reshape(-1) for k in shapes])
        f32 = torch.float32
        self.P = torch.tensor(blob, dtype=f32, device=self.device)
        self.G = torch.zeros_like(self.P)
        self.m = torch.zeros_like(self.P)
        self.v = torch.zeros_like(self.P)
        if state:   # AdamW state per parameter INDEX: a checkpoint's optimizer_state_dict["state"]
            m, v = self.m.cpu().numpy(), self.v.cpu().numpy()   # (torch's keys, as checkpoint() writes them)
            for idx, t in enumerate(self.tensors):
                s = state.get(idx)
                if s:
                    m[t["offset"]:t["offset"] + t["n"]] = np.asarray(s["exp_avg"]).reshape(-1)
                    v[t["offset"]:t["offset"] + t["n"]] = np.asarray(s["exp_avg_sq"]).reshape(-1)
                    t["step"] = float(s["step"])
            self.m.copy_(torch.tensor(m))
            self.v.copy_(torch.tensor(v))
        self.lr, self.wd, self.b1, self.b2, self.eps = FPE_LR, weight_decay, betas[0], betas[1], eps
        self.loss = torch.zeros(2, dtype=torch.float64, device=self.device)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def adam_step(self, positive: bool):
        """torch.optim.AdamW.step (utils.py:65); the prototype decoder had no
        gradient when the window has no positive label (torch skips it)."""
        arr = []
        for t in self.tensors:
            active = positive or t["name"] not in COND
            if active:
                t["step"] += 1
            st = max(t["step"], 1.0)
            arr.append(_AdamTensor(t["offset"], t["n"], int(active), self.lr / (1 - self.b1 ** st),
                                   math.sqrt(1 - self.b2 ** st)))
        desc = (_AdamTensor * len(arr))(*arr)
        _native.check(self._L.pgp_adamw(
            ctypes.c_void_p(self.P.data_ptr()), ctypes.c_void_p(self.G.data_ptr()),
            ctypes.c_void_p(self.m.data_ptr()), ctypes.c_void_p(self.v.data_ptr()),
            self.lr, self.wd, self.b1, self.b2, self.eps, desc, len(arr), self._stream()), "pgp_adamw")

    def backprop(self, st: TuneState, wins, h0s, anom, cls):
        """train.py:42-57 over the windows: one device step per window (forward,
        bookkeeping, backward) and its AdamW; the state (prototypes, factor,
        counters) lives on the device for the whole pass and is read back once.
        Returns the per-window (aloss, tloss)."""
        st.num_zero, st.num_ones = 1, 1
        n, H, dev = len(wins), self.H, self.device
        anom = np.asarray(anom).reshape(n, H)
        cls = np.asarray(cls).reshape(n, H)
        w = torch.as_tensor(np.asarray(wins), dtype=torch.float32).to(dev).contiguous()
        h = torch.as_tensor(np.asarray(h0s), dtype=torch.float32).reshape(n, 3).to(dev).contiguous()
        y = torch.as_tensor(anom, dtype=torch.int32).to(dev).contiguous()
        c = torch.as_tensor(np.clip(cls, 0, 2), dtype=torch.int32).to(dev).contiguous()
        state = torch.tensor(st.vector(), dtype=torch.float64, device=dev)
        K = st.protos.shape[0]
        losses = torch.zeros((n, 2), dtype=torch.float64, device=dev)
        positive = np.any(anom > 0, axis=1)
        for i in range(n):
            _native.check(self._L.pgp_fpe_train_step(
                H, K, w[i].data_ptr(), h[i].data_ptr(), y[i].data_ptr(), c[i].data_ptr(), self.P.data_ptr(),
                self.G.data_ptr(), state.data_ptr(), PROTO_UPDATE_MIN, PROTO_FACTOR_DECAY, losses[i].data_ptr(),
                self._stream()), "pgp_fpe_train_step")
            self.adam_step(bool(positive[i]))
        st.from_vector(state.cpu().numpy())
        return [tuple(r) for r in losses.cpu().numpy().tolist()]

    def forward_many(self, wins, h0s):
        """n independent forwards (accuracy(), train.py:94-109): probs, protos [n,H,2] fp64."""
        n, H, dev = len(wins), self.H, self.device
        w = torch.as_tensor(np.asarray(wins), dtype=torch.float32).to(dev).contiguous()
        h = torch.as_tensor(np.asarray(h0s), dtype=torch.float32).reshape(n, 3).to(dev).contiguous()
        out = torch.zeros((2, n, H, 2), dtype=torch.float64, device=dev)
        _native.check(self._L.pgp_fpe_forward_many(H, n, w.data_ptr(), h.data_ptr(), self.P.data_ptr(),
                                                    out[0].data_ptr(), out[1].data_ptr(), self._stream()),
                      "pgp_fpe_forward_many")
        o = out.cpu().numpy()
        return o[0], o[1]

    def accuracy(self, st: TuneState, wins, h0s, anom, cls):
        """train.py:94-109 on the FPE (its probabilities are what the reference
        takes the argmax of): (AScore, CScore)."""
        probs, protos = self.forward_many(wins, h0s)
        return accuracy_scores(probs, protos, anom, cls, st.protos)

    def weights_numpy(self) -> dict:
        p = self.P.detach().cpu().numpy().astype(np.float64)
        return {t["name"]: p[t["offset"]:t["offset"] + t["n"]].reshape(t["shape"]) for t in self.tensors}

    def checkpoint(self, epoch, accuracy_list, prototypes):
        """save_model's dict (utils.py:49-58) for the FPE: weights, prototypes,
        AdamW state per parameter index, epoch, accuracy_list."""
        w = self.weights_numpy()
        m, v = self.m.cpu().numpy(), self.v.cpu().numpy()
        state = {}
        for idx, t in enumerate(self.tensors):
            sl = slice(t["offset"], t["offset"] + t["n"])
            if t["step"] > 0:
                state[idx] = {"step": torch.tensor(float(t["step"])),
                              "exp_avg": torch.tensor(m[sl].astype(np.float64).reshape(t["shape"])),
                              "exp_avg_sq": torch.tensor(v[sl].astype(np.float64).reshape(t["shape"]))}
        return {"epoch": epoch,
                "model_state_dict": {k: torch.tensor(a) for k, a in w.items()},
                "model_prototypes": [torch.tensor(np.asarray(p, dtype=np.float64)) for p in prototypes],
                "optimizer_state_dict": {"state": state, "param_groups": [{
                    "lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps, "weight_decay": self.wd,
                    "amsgrad": False, "params": list(range(len(self.tensors)))}]},
                "accuracy_list": list(accuracy_list)}


def draw_h0(n, generator=None):
    """The GRU states n consecutive FPE forwards draw (models.py:70:
    torch.randn(1, 1, 3, dtype=torch.double) on the CPU generator), [n,3]."""
    return np.stack([torch.randn(1, 1, 3, dtype=torch.double, generator=generator).numpy().reshape(3)
                     for _ in range(n)])
