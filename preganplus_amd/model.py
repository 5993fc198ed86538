"""Batched PreGAN+ decision model on MI355X (host side of the C-ABI).

``DecisionModel.forward`` is one launch sequence of ``pgp_forward``: the
per-window part of ``PreGANPlusRecovery.run_model``
(``recovery/PreGANPlus.py:115-136``) for a whole batch of windows — encoder
(``models.py:376-416``), detect/embed (``PreGANPlus.py:119-131``),
``get_classes`` (``utils.py:102-109``), Gen/Disc (``models.py:118-151``) and the
decision tensors of ``recover_decision`` (``PreGANPlus.py:84-105``).

torch is only plumbing here (device memory, the stream); every FLOP runs in
``libpreganplus.so``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native
from . import weights as W


class DecisionModel:
    def __init__(self, n_hosts: int, weights: dict, device: str | torch.device = "cuda"):
        self.H = int(n_hosts)
        self.K = int(np.asarray(weights["prototypes"]).shape[0])
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("DecisionModel runs on the GPU only (no CPU fallback)")
        L = _native.lib()
        if self.H not in _native.supported_hosts():
            raise ValueError(f"H={self.H} not compiled in; supported {_native.supported_hosts()}")
        self._L = L
        h = ctypes.c_void_p()
        _native.check(L.pgp_create(self.H, self.K, ctypes.byref(h)), "pgp_create")
        self._h = h
        self.load_weights(weights)

    def load_weights(self, weights: dict):
        blob = W.pack_blob(weights, self.H)
        n = self._L.pgp_weight_blob_len(self.H, self.K)
        if n != blob.size:
            raise ValueError(f"blob length {blob.size} != {n}")
        torch.cuda.set_device(self.device)
        _native.check(self._L.pgp_load_weights(
            self._h, blob.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), blob.size),
            "pgp_load_weights")
        self.prototypes = np.asarray(weights["prototypes"], dtype=np.float64)

    def load_master(self, P: torch.Tensor, prototypes):
        """Rebuild the packed inference weights from device master weights
        (natural fp32 layout, preganplus_amd.train.Trainer.P)."""
        pr = np.ascontiguousarray(np.asarray(prototypes, dtype=np.float64))
        L = self._L
        L.pgp_load_weights_master.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        torch.cuda.synchronize(self.device)
        _native.check(L.pgp_load_weights_master(self._h, ctypes.c_void_p(P.data_ptr()),
                                                pr.ctypes.data_as(ctypes.POINTER(ctypes.c_double))),
                      "pgp_load_weights_master")
        self.prototypes = pr.copy()

    def repack_master(self, P: torch.Tensor, protos_dev: torch.Tensor, prototypes_host=None, stream=None,
                      sections: int = 3):
        """Rebuild the packed inference weights ON THE DEVICE (``pgp_repack_master``)
        from device master weights P (natural fp32) and device prototypes
        protos_dev [K,2] fp64: three launches on the stream, no host round trip,
        the same bits as load_master.  prototypes_host (optional) updates the
        host-side copy of the prototypes.  sections (``pgp_repack_master_sections``):
        1 the PreGAN+ encoder / decoders only, 2 the GAN only, 3 both."""
        if protos_dev.dtype != torch.float64 or protos_dev.numel() != 2 * self.K or not protos_dev.is_contiguous():
            raise ValueError(f"protos_dev must be contiguous float64 [{self.K},2] on the device")
        L = self._L
        L.pgp_repack_master_sections.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p]
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        _native.check(L.pgp_repack_master_sections(self._h, ctypes.c_void_p(P.data_ptr()),
                                                   ctypes.c_void_p(protos_dev.data_ptr()), int(sections),
                                                   ctypes.c_void_p(st.cuda_stream)), "pgp_repack_master_sections")
        if prototypes_host is not None:
            self.prototypes = np.array(prototypes_host, dtype=np.float64)

    def reserve(self, max_batch: int):
        _native.check(self._L.pgp_reserve(self._h, int(max_batch)), "pgp_reserve")

    def gan_split(self, on: bool):
        """K3 on split-bf16 MFMAs (True: the default where compiled, H = 16, 50) or
        on the fp32 MFMA (False); ``pgp_gan_split``."""
        _native.check(self._L.pgp_gan_split(self._h, int(bool(on))), "pgp_gan_split")

    def encoder_split(self, on: bool):
        """K2's feed-forward on split-bf16 MFMAs (True: the default where
        compiled, H = 50) or on the fp32 MFMA (False); ``pgp_encoder_split``."""
        _native.check(self._L.pgp_encoder_split(self._h, int(bool(on))), "pgp_encoder_split")

    def decoder_split(self, on: bool):
        """K2b on split-bf16 MFMAs (True: the default where compiled, H = 32 and
        50) or on the fp32 MFMA (False); ``pgp_decoder_split``."""
        _native.check(self._L.pgp_decoder_split(self._h, int(bool(on))), "pgp_decoder_split")

    def alloc_outputs(self, B: int, latent: bool = False, packed: bool = False):
        """Output tensors of forward().  packed=True places them all in one
        device buffer (every output is 4-byte) with a pinned host twin, so
        to_numpy() reads the whole result with ONE device-to-host copy (the
        batch-1 plugin path)."""
        dev, H = self.device, self.H
        f32, i32 = torch.float32, torch.int32
        spec = [("logits", f32, (B, H, 2)), ("protos", f32, (B, H, 2)), ("cls", i32, (B, H)), ("any", i32, (B,)),
                ("probs", f32, (B, 2)), ("keep", i32, (B,)), ("final_target", i32, (B, H)),
                ("gen_target", i32, (B, H))]
        if packed:
            n = sum(int(np.prod(s)) for _, _, s in spec)
            buf = torch.zeros(n, dtype=i32, device=dev)
            out, o = {}, 0
            for name, dt, shp in spec:
                k = int(np.prod(shp))
                out[name] = buf[o:o + k].view(dt).view(shp)
                o += k
            out["_buf"] = buf
            out["_hbuf"] = torch.zeros(n, dtype=i32).pin_memory()
        else:
            out = {name: torch.empty(shp, dtype=dt, device=dev) for name, dt, shp in spec}
        out["latent"] = torch.empty((B, 3 * H * H), dtype=f32, device=dev) if latent else None
        return out

    def _check_inputs(self, windows, sched):
        H = self.H
        B = windows.shape[0]
        if tuple(windows.shape) != (B, 3, 3 * H) or windows.dtype != torch.float32:
            raise ValueError(f"windows must be float32 [B,3,{3 * H}], got {tuple(windows.shape)} {windows.dtype}")
        if sched is not None and (tuple(sched.shape) != (B, H, H) or sched.dtype != torch.float32):
            raise ValueError(f"sched must be float32 [B,{H},{H}], got {tuple(sched.shape)} {sched.dtype}")
        for t in (windows, sched):
            if t is not None and (t.device != self.device or not t.is_contiguous()):
                raise ValueError("inputs must be contiguous tensors on the model's device")
        return B

    def forward(self, windows: torch.Tensor, sched: torch.Tensor, out: dict | None = None,
                latent: bool = False, stage: int = -1, stream=None) -> dict:
        """windows [B,3,3H] f32 (normalised), sched [B,H,H] f32, both on device."""
        B = self._check_inputs(windows, sched)
        if out is None:
            out = self.alloc_outputs(B, latent)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t: None if t is None else t.data_ptr()
        _native.check(self._L.pgp_forward_stage(
            self._h, int(stage), B, p(windows), p(sched), p(out["logits"]), p(out["protos"]),
            p(out["cls"]), p(out["any"]), p(out["probs"]), p(out["keep"]),
            p(out["final_target"]), p(out["gen_target"]), p(out.get("latent")),
            ctypes.c_void_p(st.cuda_stream)), "pgp_forward")
        return out

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.pgp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FPEDecisionModel(DecisionModel):
    """PreGAN's decision model (BASELINE config C4): ``FPE_16`` encoder
    (``models.py:10-115``) + detect/embed/``get_classes`` over K = 3 prototypes
    (``recovery/PreGAN.py:105-120``) + PreGAN's own Gen/Disc
    (``recover_decision``, ``PreGAN.py:73-77``), one ``pgp_forward_fpe`` call
    (K4 then K3).  The GRU initial state ``h0`` [B,3] is an input: the reference
    draws it with ``torch.randn`` inside ``encode`` (``models.py:70``)."""

    def __init__(self, n_hosts: int, weights: dict, device: str | torch.device = "cuda"):
        self.H = int(n_hosts)
        self.K = W.FPE_PROTOS
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("FPEDecisionModel runs on the GPU only (no CPU fallback)")
        L = _native.lib()
        self._L = L
        h = ctypes.c_void_p()
        _native.check(L.pgp_create_fpe(self.H, ctypes.byref(h)), "pgp_create_fpe")
        self._h = h
        self.load_weights(weights)

    def load_weights(self, weights: dict):
        if "fpe" not in weights:
            raise ValueError("FPE weights need an 'fpe' section (PreGAN FPE_16 state_dict)")
        blob = W.pack_blob(weights, self.H)
        n = self._L.pgp_fpe_weight_blob_len(self.H)
        if n != blob.size:
            raise ValueError(f"blob length {blob.size} != {n}")
        torch.cuda.set_device(self.device)
        _native.check(self._L.pgp_load_weights(
            self._h, blob.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), blob.size), "pgp_load_weights")
        self.prototypes = np.asarray(weights["prototypes"], dtype=np.float64)

    def load_master(self, P, prototypes):
        raise NotImplementedError("the PreGAN encoder is frozen (PreGAN.py:29); reload GAN weights with load_weights")

    def alloc_outputs(self, B: int, latent: bool = False):
        out = super().alloc_outputs(B, False)
        out["scores"] = out.pop("logits")
        return out

    def forward(self, windows: torch.Tensor, h0: torch.Tensor, sched: torch.Tensor, out: dict | None = None,
                stage: int = -1, stream=None) -> dict:
        """windows [B,3,3H], h0 [B,3], sched [B,H,H]; float32, contiguous, on device.
        stage: -1 both kernels, 0 K4 only, 1 K3 only (after a stage-0 call)."""
        B = self._check_inputs(windows, sched)
        if tuple(h0.shape) != (B, 3) or h0.dtype != torch.float32 or h0.device != self.device \
                or not h0.is_contiguous():
            raise ValueError(f"h0 must be contiguous float32 [B,3] on {self.device}")
        if out is None:
            out = self.alloc_outputs(B)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t: t.data_ptr()
        _native.check(self._L.pgp_forward_fpe_stage(
            self._h, int(stage), B, p(windows), p(h0), p(sched), p(out["scores"]), p(out["protos"]), p(out["cls"]),
            p(out["any"]), p(out["probs"]), p(out["keep"]), p(out["final_target"]), p(out["gen_target"]),
            ctypes.c_void_p(st.cuda_stream)), "pgp_forward_fpe")
        return out


def migrations(keep_orig: torch.Tensor, final_target: torch.Tensor, cur_host: torch.Tensor, stream=None,
               out=None):
    """recover_decision's per-container moves for a batch (K5, ``pgp_migrations``):
    int32 device tensors keep_orig [B], final_target [B,C], cur_host [B,C]
    (-1 = unplaced / None) -> (moves [B,C], hosts_from [B,C])."""
    B, C = final_target.shape
    for t, shp in ((keep_orig, (B,)), (final_target, (B, C)), (cur_host, (B, C))):
        if tuple(t.shape) != shp or t.dtype != torch.int32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("migrations: int32 contiguous device tensors keep [B], final_target/cur_host [B,C]")
    moves, hosts_from = out if out is not None else (torch.empty_like(final_target), torch.empty_like(final_target))
    st = stream if stream is not None else torch.cuda.current_stream(final_target.device)
    _native.check(_native.lib().pgp_migrations(
        C, B, keep_orig.data_ptr(), final_target.data_ptr(), cur_host.data_ptr(), moves.data_ptr(),
        hosts_from.data_ptr(), ctypes.c_void_p(st.cuda_stream)), "pgp_migrations")
    return moves, hosts_from


def embedding(logits: torch.Tensor, protos: torch.Tensor, out: torch.Tensor | None = None, stream=None):
    """run_model's embedding (PreGANPlus.py:129) for a batch (``pgp_embedding``):
    fp32 device [B,H,2] logits / protos -> protos where the host is flagged
    (argmax = 1, ties -> 0), else 0."""
    B, H = logits.shape[0], logits.shape[1]
    for t in (logits, protos):
        if tuple(t.shape) != (B, H, 2) or t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("embedding: fp32 contiguous device tensors logits / protos [B,H,2]")
    out = torch.empty_like(protos) if out is None else out
    st = stream if stream is not None else torch.cuda.current_stream(logits.device)
    _native.check(_native.lib().pgp_embedding(H, B, logits.data_ptr(), protos.data_ptr(), out.data_ptr(),
                                              ctypes.c_void_p(st.cuda_stream)), "pgp_embedding")
    return out


def assemble_decision(original_decision, moves_row, cur_host_row):
    """The returned list of recover_decision (PreGANPlus.py:96-105): the original
    decision's order, then overridden / new container keys in host-ascending,
    then container order (``np.concatenate(host_alloc)``)."""
    decision = dict(original_decision)
    moves_row = [int(v) for v in moves_row]
    cur = [int(v) for v in cur_host_row]
    order = sorted((h, c) for c, h in enumerate(cur) if h >= 0)
    for _, c in order:
        if moves_row[c] >= 0:
            decision[c] = moves_row[c]
    return list(decision.items())


def to_numpy(out: dict) -> dict:
    res = {}
    if "_buf" in out:   # packed outputs: one device-to-host copy, numpy views of the pinned twin
        hb = out["_hbuf"]
        hb.copy_(out["_buf"], non_blocking=True)
        torch.cuda.current_stream(out["_buf"].device).synchronize()
        a, o = hb.numpy(), 0
        for k, v in out.items():
            if k.startswith("_") or v is None or k == "latent":
                continue
            n = v.numel()
            x = a[o:o + n].view(np.float32 if v.dtype == torch.float32 else np.int32).reshape(tuple(v.shape)).copy()
            res[k] = x.astype(bool) if k in ("any", "keep") else x
            o += n
        if out.get("latent") is not None:
            res["latent"] = out["latent"].detach().cpu().numpy()
        return res
    for k, v in out.items():
        if v is None or k.startswith("_"):
            continue
        a = v.detach().cpu().numpy()
        if k in ("any", "keep"):
            a = a.astype(bool)
        res[k] = a
    return res
