"""Batched ``Stats.runSimulation`` on MI355X — the GAN-label producer.

The reference scores a schedule for the GAN label (``PreGANPlus.py:65`` ->
``run_simulation`` ``PreGANSrc/src/utils.py:97-100`` -> ``Stats.runSimulation``
``stats/Stats.py:154-177``): move every placed container to its schedule row's
first argmax when the move is a change and ``getPlacementPossible``
(``simulator/Simulator.py:89-105``) admits it, then sum per-host apparent IPS and
price it with the host power model (``Host.getPowerFromIPS`` ``host/Host.py:25-26``,
``PM.powerFromCPU`` ``metrics/powermodels/PM.py:11-16``); score = 0.8 energy·interval
+ 0.2 latency (``PreGANSrc/src/constants.py:19-20``).

Here the environment's simulation inputs are packed once per interval into one
fp64 record per environment (``pack_env``), and ``pgp_simulate``
(``csrc/pgp_sim.hip``) scores the generator's and the original schedule of a
whole batch of environments on the device and writes the BCE target
``PreGANPlus.py:66`` uses — the label never visits the host.

Record layout (doubles, ``env_len(H) = 2 + 20 H``; C = H containers):
  [0] interval time   [1] latency term max(0, mean(avgresponsetime[-5:]))
  host[C] (-1: no container / unplaced)  base_ips[C]  ram_size[C]  disk_size[C]
  apparent_ips[C]  ips_available[H]  ram_available[H]  disk_available[H]
  ips_cap[H]  power_list[H][11]
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native

COEFF_ENERGY, COEFF_LATENCY = 0.8, 0.2  # PreGANSrc/src/constants.py:19-20
N_POWER = 11  # PM.powerlist: power at 0, 10, ..., 100 % cpu


def env_len(H: int) -> int:
    return 2 + 20 * H


def offsets(H: int) -> dict:
    """Field -> (start, length) inside one record."""
    o, out = 2, {"interval": (0, 1), "latency": (1, 1)}
    for name, n in (("host", H), ("base_ips", H), ("ram", H), ("disk", H), ("app_ips", H), ("ips_av", H),
                    ("ram_av", H), ("disk_av", H), ("ips_cap", H), ("power", H * N_POWER)):
        out[name] = (o, n)
        o += n
    assert o == env_len(H)
    return out


def latency_term(metrics) -> float:
    """Stats.py:177: max(0, mean of the last 5 intervals' avgresponsetime)."""
    last = [m["avgresponsetime"] for m in metrics[-5:]]
    return float(max(0, np.mean(last))) if last else 0.0  # max(0, nan) of an empty list is 0


def pack_env(env, metrics, out: np.ndarray | None = None) -> np.ndarray:
    """Read runSimulation's inputs from a COSCO environment (``Simulator`` or
    ``Framework``: ``hostlist``, ``containerlist``, ``intervaltime``) and the
    stats' ``metrics`` list, through the same getters the reference calls."""
    H = len(env.hostlist)
    if len(env.containerlist) != H:
        raise ValueError(f"runSimulation scores [containers={len(env.containerlist)}, hosts={H}] schedules; "
                         "the PreGAN+ path has one container slot per host")
    v = np.zeros(env_len(H)) if out is None else out
    o = offsets(H)
    v[0] = env.intervaltime
    v[1] = latency_term(metrics)
    f = {k: v[s:s + n] for k, (s, n) in o.items()}
    f["host"][:] = -1
    for i, c in enumerate(env.containerlist):
        if not c or c.getHostID() == -1:
            continue
        if c.id != i:
            raise ValueError("containerlist[i].id must be i (Stats.py:175 indexes containerlist by id)")
        f["host"][i] = c.getHostID()
        f["base_ips"][i] = c.getBaseIPS()
        f["ram"][i] = c.getRAM()[0]
        f["disk"][i] = c.getDisk()[0]
        f["app_ips"][i] = c.getApparentIPS()
    for h, host in enumerate(env.hostlist):
        f["ips_av"][h] = host.getIPSAvailable()
        f["ram_av"][h] = host.getRAMAvailable()[0]
        f["disk_av"][h] = host.getDiskAvailable()[0]
        f["ips_cap"][h] = host.ipsCap
        pl = host.powermodel.powerlist
        if len(pl) != N_POWER:
            raise ValueError(f"host {h}: power list of {len(pl)} points, expected {N_POWER}")
        f["power"][h * N_POWER:(h + 1) * N_POWER] = pl
    return v


class Simulation:
    """Device-side runSimulation over a batch of packed environments.

    ``score(envs, new_sched, orig_sched)``: envs [E, env_len(H)] fp64,
    schedules [E, H, H] fp32 (the generator's output as the GAN kernels write
    it, and the original schedule) -> (out [E, 4] fp64 = energy·interval and
    score of the new, then of the original schedule; target [E, 2] fp32, the
    BCE target of PreGANPlus.py:66)."""

    def __init__(self, H: int, device="cuda"):
        self.H = H
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("Simulation runs on the GPU only (no CPU fallback)")
        L = _native.lib()
        vp = ctypes.c_void_p
        L.pgp_sim_env_len.argtypes = [ctypes.c_int]
        L.pgp_sim_env_len.restype = ctypes.c_size_t
        L.pgp_simulate.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, vp]
        self._L = L
        if L.pgp_sim_env_len(H) != env_len(H):
            raise RuntimeError("libpreganplus record layout differs from simulate.env_len")

    def score(self, envs, new_sched, orig_sched, out=None, target=None, stream=None):
        dev = self.device
        envs = torch.as_tensor(envs, dtype=torch.float64).to(dev).contiguous()
        sn = torch.as_tensor(new_sched, dtype=torch.float32).to(dev).contiguous()
        so = torch.as_tensor(orig_sched, dtype=torch.float32).to(dev).contiguous()
        E, H = envs.shape[0], self.H
        if envs.shape != (E, env_len(H)) or tuple(sn.shape) != (E, H, H) or tuple(so.shape) != (E, H, H):
            raise ValueError(f"shapes: envs {tuple(envs.shape)}, new {tuple(sn.shape)}, orig {tuple(so.shape)}")
        out = torch.empty(E, 4, dtype=torch.float64, device=dev) if out is None else out
        target = torch.empty(E, 2, dtype=torch.float32, device=dev) if target is None else target
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        _native.check(self._L.pgp_simulate(H, E, envs.data_ptr(), sn.data_ptr(), so.data_ptr(), out.data_ptr(),
                                           target.data_ptr(), ctypes.c_void_p(st.cuda_stream)), "pgp_simulate")
        return out, target


def synth_envs(E: int, H: int, seed: int = 0) -> np.ndarray:
    """Synthetic records for benches and tests: hosts of 4-16 k IPS with
    monotone 11-point power curves, H container slots (~8 % empty/unplaced)
    on random hosts, current availabilities derived from the placement."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.zeros((E, env_len(H)))
    o = offsets(H)
    for i in range(E):
        v = out[i]
        f = {k: v[s:s + n] for k, (s, n) in o.items()}
        v[0], v[1] = 300.0, rng.uniform(0, 30)
        cap = rng.choice([4029.0, 8058.0, 16111.0], H)
        ramc = rng.choice([4295.0, 8192.0, 17180.0], H)
        diskc = np.full(H, 32212.0)
        host = rng.integers(0, H, H).astype(float)
        host[rng.uniform(size=H) < 0.08] = -1
        base = rng.uniform(50, 1500, H).round()
        ram = rng.uniform(20, 1500, H)
        disk = rng.uniform(10, 600, H)
        app = np.zeros(H)
        used = np.zeros((3, H))
        for c in np.nonzero(host >= 0)[0]:
            used[:, int(host[c])] += (base[c], ram[c], disk[c])
        for c in np.nonzero(host >= 0)[0]:
            h = int(host[c])
            n = int((host == h).sum())
            app[c] = min(base[c] * 3, base[c] + (cap[h] - used[0, h]) / n)
        placed = host >= 0
        f["host"][:] = host
        f["base_ips"][:] = np.where(placed, base, 0)
        f["ram"][:] = np.where(placed, ram, 0)
        f["disk"][:] = np.where(placed, disk, 0)
        f["app_ips"][:] = app
        f["ips_av"][:] = cap - used[0]
        f["ram_av"][:] = ramc - used[1]
        f["disk_av"][:] = diskc - used[2]
        f["ips_cap"][:] = cap
        p0 = rng.uniform(1, 90, H)
        f["power"][:] = (p0[:, None] + np.cumsum(np.concatenate(
            [np.zeros((H, 1)), rng.uniform(0.5, 12, (H, N_POWER - 1))], 1), 1)).round(2).reshape(-1)
    return out
