"""CPU restatement of ``Stats.runSimulation`` — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, smoke() and bench.py's CPU baseline, never by the
product.  Works on the packed record of ``preganplus_amd/simulate.py``
(``pack_env``) and restates, in Python doubles, exactly the reference's order of
operations:

* ``Stats.runSimulation`` (stats/Stats.py:154-177): host_alloc built in
  containerlist order; decisions for placed containers in concatenated
  host_alloc order whose row's first argmax (``list.index(max(list))``) differs
  from the current host; ``filter_placement`` (scheduler/Scheduler.py:22-27)
  keeps them all (each already differs from the container's host); a move is
  applied when ``getPlacementPossible`` (simulator/Simulator.py:89-105: base IPS,
  RAM size, disk size against the host's CURRENT availability) admits it, and
  the container is removed from its host's list and appended to the target's;
  per-host IPS summed in list order; energy = sum over hosts in order of
  ``getPowerFromIPS`` (simulator/host/Host.py:25-26) times the interval;
* ``PM.powerFromCPU`` (metrics/powermodels/PM.py:11-16) with Python's floor,
  float modulo and negative list indexing;
* ``run_simulation`` (recovery/PreGANSrc/src/utils.py:97-100):
  0.8 energy + 0.2 latency (constants.py:19-20); the label of PreGANPlus.py:66.

Pinned by tests/test_sim_oracle.py against tests/golden/sim_h16.npz / sim_h50.npz,
made by the reference's own runSimulation on the reference's own Host, Container
and power-model objects (tests/golden/make_golden_sim.py).
"""
from __future__ import annotations

import math

import numpy as np

COEFF_ENERGY, COEFF_LATENCY = 0.8, 0.2
N_POWER = 11


def fields(v, H):
    o, out = 2, {}
    for name, n in (("host", H), ("base_ips", H), ("ram", H), ("disk", H), ("app_ips", H), ("ips_av", H),
                    ("ram_av", H), ("disk_av", H), ("ips_cap", H), ("power", H * N_POWER)):
        out[name] = [float(x) for x in v[o:o + n]]
        o += n
    return float(v[0]), float(v[1]), out


def power_from_cpu(pl, cpu):
    """PM.py:11-16 (IndexError where the reference raises one)."""
    index = math.floor(cpu / 10)
    left = pl[index]
    right = pl[index + 1 if cpu % 10 != 0 else index]
    alpha = (cpu / 10) - index
    return alpha * right + (1 - alpha) * left


def run_simulation(v, sched, H):
    """Stats.py:154-177 on one record and one [H, H] schedule -> (energy, latency)."""
    interval, latency, f = fields(v, H)
    host = [int(h) for h in f["host"]]
    host_alloc = [[] for _ in range(H)]
    container_alloc = [-1] * H
    for c in range(H):
        if host[c] != -1:
            host_alloc[host[c]].append(c)
            container_alloc[c] = host[c]
    decision = []
    for hl in host_alloc:
        for cid in hl:
            row = [float(x) for x in sched[cid]]
            new_host = row.index(max(row))
            if container_alloc[cid] != new_host:
                decision.append((cid, new_host))
    for cid, hid in decision:
        possible = (f["base_ips"][cid] <= f["ips_av"][hid] and f["ram"][cid] <= f["ram_av"][hid]
                    and f["disk"][cid] <= f["disk_av"][hid])
        if possible and container_alloc[cid] != -1:
            host_alloc[container_alloc[cid]].remove(cid)
            host_alloc[hid].append(cid)
    energy = 0
    for hid, cids in enumerate(host_alloc):
        ips = 0
        for cid in cids:
            ips += f["app_ips"][cid]
        pl = f["power"][hid * N_POWER:(hid + 1) * N_POWER]
        energy += power_from_cpu(pl, min(100, 100 * (ips / f["ips_cap"][hid])))
    return energy * interval, latency


def score(v, sched, H):
    e, r = run_simulation(v, sched, H)
    return e, COEFF_ENERGY * e + COEFF_LATENCY * r


def simulate_batch(envs, new, orig, H):
    """-> out [E, 4] (energy, score of new; energy, score of orig), target [E, 2]."""
    E = len(envs)
    out = np.zeros((E, 4))
    target = np.zeros((E, 2), np.float32)
    for i in range(E):
        out[i, 0:2] = score(envs[i], new[i], H)
        out[i, 2:4] = score(envs[i], orig[i], H)
        target[i] = (0.0, 1.0) if out[i, 1] <= out[i, 3] else (1.0, 0.0)
    return out, target
