"""GOBI on MI355X — the schedule producer upstream of the decision path.

Replaces the optimiser of ``GOBIScheduler.run_GOBI`` (``scheduler/GOBI.py:19-42``):
``opt()`` (``scheduler/BaGTI/src/opt.py:17-33``) over the ``energy_latency_16``
surrogate (``scheduler/BaGTI/src/models.py:8-27``), batched over independent
environments, one ``pgp_gobi_optimize`` launch (``csrc/pgp_gobi.hip``).  Its
result's allocation columns are ``env.scheduler.result_cache``, the schedule
input of ``PreGANPlusRecovery.run_model`` (``recovery/PreGANPlus.py:117``).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _native

H = 16
_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "gobi_energy_latency_16.npz")
_ORDER = ("find.0.weight", "find.0.bias", "find.2.weight", "find.2.bias", "find.4.weight", "find.4.bias",
          "find.6.weight", "find.6.bias")


def load_weights(path=_DATA):
    """The surrogate's state dict (fp32) and the dataset's max container IPS
    (scheduler/BaGTI/src/utils.py:61), as packaged from the reference checkpoint
    by tests/golden/make_golden_gobi.py."""
    z = np.load(path)
    return {k: np.asarray(z[k], dtype=np.float32) for k in _ORDER}, float(z["max_ips"])


class GOBIOptimizer:
    """Batched opt(): init [E,16,18] -> (result [E,16,18], iterations [E], fitness [E])."""

    def __init__(self, weights: dict | None = None, device="cuda"):
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("GOBIOptimizer runs on the GPU only (no CPU fallback)")
        if weights is None:
            weights, self.max_ips = load_weights()
        L = _native.lib()
        vp = ctypes.c_void_p
        L.pgp_gobi_weight_len.argtypes = [ctypes.c_int]
        L.pgp_gobi_weight_len.restype = ctypes.c_size_t
        L.pgp_gobi_create.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, ctypes.POINTER(vp)]
        L.pgp_gobi_optimize.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int, vp, vp]
        L.pgp_gobi_destroy.argtypes = [vp]
        L.pgp_gobi_last_error.argtypes = []
        L.pgp_gobi_last_error.restype = ctypes.c_char_p
        self._L = L
        blob = np.ascontiguousarray(np.concatenate([np.asarray(weights[k], np.float32).reshape(-1) for k in _ORDER]))
        if blob.size != L.pgp_gobi_weight_len(H):
            raise ValueError(f"GOBI weight blob {blob.size} != {L.pgp_gobi_weight_len(H)}")
        torch.cuda.set_device(self.device)
        h = vp()
        rc = L.pgp_gobi_create(H, blob.ctypes.data_as(vp), blob.size, ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"pgp_gobi_create: {rc} {L.pgp_gobi_last_error().decode()}")
        self._h = h

    def optimize(self, init, out=None, stream=None, max_iters=0, pre=None):
        """init: [E,16,18] float32 (device tensor or host array).  max_iters /
        pre [E,16,16]: test hooks (step limit, pre-projection values)."""
        x = torch.as_tensor(init, dtype=torch.float32).to(self.device).contiguous()
        if x.dim() != 3 or tuple(x.shape[1:]) != (H, H + 2):
            raise ValueError(f"init must be [E,{H},{H + 2}], got {tuple(x.shape)}")
        E = x.shape[0]
        if out is None:
            out = (torch.empty_like(x), torch.empty(E, dtype=torch.int32, device=self.device),
                   torch.empty(E, dtype=torch.float32, device=self.device))
        res, its, fit = out
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = self._L.pgp_gobi_optimize(self._h, E, x.data_ptr(), res.data_ptr(), its.data_ptr(), fit.data_ptr(),
                                       int(max_iters), None if pre is None else pre.data_ptr(),
                                       ctypes.c_void_p(st.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"pgp_gobi_optimize: {rc} {self._L.pgp_gobi_last_error().decode()}")
        return res, its, fit

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.pgp_gobi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Scheduler:
    """The scheduler plugin interface COSCO drives (scheduler/Scheduler.py:9-38):
    main.py:154-155 calls ``selection()``, ``placement(ids)`` and
    ``filter_placement(decision)``; Simulator.py:118, 173-174 call
    ``getMigrationFromHost`` / ``getMigrationToHost``.  Only these plugin methods
    are restated; the base class's host-selection heuristics (LR / MAD / IQR
    ..., :40-185) belong to the other schedulers, which are out of scope."""

    def __init__(self):
        self.env = None

    def setEnvironment(self, env):
        self.env = env

    def selection(self):
        return None

    def placement(self, containerlist):
        return None

    def filter_placement(self, decision):
        """Scheduler.py:20-25: drop decisions that keep a container in place."""
        return [(cid, hid) for cid, hid in decision if self.env.getContainerByID(cid).getHostID() != hid]

    def getMigrationFromHost(self, hostID, decision):
        """Scheduler.py:27-32."""
        return [cid for cid, _ in decision if self.env.getContainerByID(cid).getHostID() == hostID]

    def getMigrationToHost(self, hostID, decision):
        """Scheduler.py:34-38."""
        return [cid for cid, hid in decision if hid == hostID]


class GOBIScheduler(Scheduler):
    """The placement step of scheduler/GOBI.py:19-48 on the COSCO env interface
    (hostlist[i].getCPU(), containerlist[c].getApparentIPS() / getHostID() / id),
    a drop-in for the scheduler main.py builds (``GOBIScheduler('energy_latency_16')``)."""

    def __init__(self, data_type="energy_latency_16", device="cuda"):
        super().__init__()
        if data_type != "energy_latency_16":
            raise ValueError("only the energy_latency_16 surrogate ships with the reference")
        self.opt = GOBIOptimizer(device=device)
        self.max_container_ips = self.opt.max_ips
        self.data_type = data_type
        self.hosts = H
        self.result_cache = None

    def selection(self):
        """GOBI.py:44-45: GOBI re-places every container, it selects none."""
        return []

    def init_matrix(self, rng=np.random):
        """GOBI.py:20-32: [host cpu / 100, container ips / max, one-hot host];
        an unplaced container gets a random host, as the reference draws it."""
        cpu = np.array([[h.getCPU() / 100 for h in self.env.hostlist]]).T
        cpuc = np.array([[(c.getApparentIPS() / self.max_container_ips if c else 0) for c in self.env.containerlist]]).T
        alloc, prev = [], {}
        for c in self.env.containerlist:
            one = [0] * len(self.env.hostlist)
            if c:
                prev[c.id] = c.getHostID()
            if c and c.getHostID() != -1:
                one[c.getHostID()] = 1
            else:
                one[rng.randint(0, len(self.env.hostlist))] = 1
            alloc.append(one)
        return np.concatenate((cpu, cpuc, np.array(alloc)), axis=1), prev

    def run_GOBI(self):
        init, prev = self.init_matrix()
        res, _, _ = self.opt.optimize(init[None])
        result = res[0].cpu().numpy()
        self.result_cache = result[:, -self.hosts:]
        decision = []
        for cid in prev:  # GOBI.py:37-41
            one_hot = result[cid, -self.hosts:].tolist()
            new_host = one_hot.index(max(one_hot))
            if prev[cid] != new_host:
                decision.append((cid, new_host))
        return decision

    def placement(self, containerIDs):
        return self.run_GOBI()
