"""Golden fixtures for the GAN-label simulation, made by the
reference's own code, run here:

  stats/Stats.py:154-177             Stats.runSimulation
  scheduler/Scheduler.py:22-27       Scheduler.filter_placement (GOBIScheduler inherits it)
  simulator/Simulator.py:65-105      getContainersOfHost / getContainerByID / getHostByID / getPlacementPossible
  simulator/host/Host.py             getPowerFromIPS, getIPSAvailable, getRAMAvailable, getDiskAvailable
  simulator/container/Container.py   getBaseIPS, getApparentIPS, getRAM, getDisk (constant IPS/RAM/disk models)
  metrics/powermodels/*.py           PM.powerFromCPU and the shipped power lists
  simulator/environment/RPiEdge.py (H=16, main.py's datacenter), AzureFog.py (H=50): the hosts
  recovery/PreGANSrc/src/utils.py:97-100, constants.py:19-20  run_simulation's score

``stats/Stats.py`` and ``scheduler/Scheduler.py`` import plotting packages absent
from this image (``scienceplots``), so this script compiles just the two methods
above from those files' text (``ast``) and binds them to a minimal stats object
holding a real ``Simulator`` (built without its workload/scheduler wiring), real
``Host`` and ``Container`` objects and the real power models.  Run with ``python -B``
from /tmp (no bytecode written under /root/reference).

Writes tests/golden/sim_h16.npz and sim_h50.npz: the packed records (via the
product's ``preganplus_amd.simulate.pack_env`` reading those live objects), the
generator-like and original schedules (fp32 values), and the reference's
(energy, score) for each, plus the BCE target.
"""
import ast
import importlib.util
import os
import sys
import types
import warnings

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(OUT))


def method_from(path, cls, name, glb):
    tree = ast.parse(open(path).read())
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == cls:
            for fn in node.body:
                if isinstance(fn, ast.FunctionDef) and fn.name == name:
                    mod = ast.Module(body=[fn], type_ignores=[])
                    ns = dict(glb)
                    exec(compile(mod, path, "exec"), ns)
                    return ns[name]
    raise KeyError(f"{cls}.{name} not in {path}")


def function_from(path, name, glb):
    tree = ast.parse(open(path).read())
    for fn in tree.body:
        if isinstance(fn, ast.FunctionDef) and fn.name == name:
            ns = dict(glb)
            exec(compile(ast.Module(body=[fn], type_ignores=[]), path, "exec"), ns)
            return ns[name]
    raise KeyError(f"{name} not in {path}")


def main():
    sys.path.insert(0, REF)
    sys.path.insert(0, REPO)
    warnings.simplefilter("ignore")
    from simulator.Simulator import Simulator
    from simulator.host.Host import Host
    from simulator.container.Container import Container
    from simulator.container.IPSModels.IPSMConstant import IPSMConstant
    from simulator.container.RAMModels.RMConstant import RMConstant
    from simulator.container.DiskModels.DMConstant import DMConstant
    from simulator.environment.RPiEdge import RPiEdge
    from simulator.environment.AzureFog import AzureFog
    from preganplus_amd.simulate import pack_env

    spec = importlib.util.spec_from_file_location("pgp_ref_constants", f"{REF}/recovery/PreGANSrc/src/constants.py")
    K = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(K)
    run_sim = method_from(f"{REF}/stats/Stats.py", "Stats", "runSimulation", {"np": np})
    filt = method_from(f"{REF}/scheduler/Scheduler.py", "Scheduler", "filter_placement", {})
    run_simulation = function_from(f"{REF}/recovery/PreGANSrc/src/utils.py", "run_simulation",
                                   {"Coeff_Energy": K.Coeff_Energy, "Coeff_Latency": K.Coeff_Latency})

    rng = np.random.Generator(np.random.PCG64(77))
    for H, dc, E in ((16, RPiEdge, 96), (50, AzureFog, 48)):
        envs, news, origs, ref = [], [], [], []
        for e in range(E):
            sim = Simulator.__new__(Simulator)
            sim.hostlist, sim.containerlist, sim.inactiveContainers = [], [], []
            sim.intervaltime, sim.interval, sim.hostlimit, sim.containerlimit = 300, 0, H, H
            for i, (ips, ram, disk, bw, lat, pm) in enumerate(dc(H).generateHosts()):
                sim.hostlist.append(Host(i, ips, ram, disk, bw, lat, pm, sim))
            mode = e % 6  # 0: typical, 1: crowded hosts, 2: sparse, 3: heavy (overload), 4: one host, 5: all unplaced
            for c in range(H):
                if mode == 5 or (mode == 2 and rng.uniform() < 0.5) or rng.uniform() < 0.06:
                    sim.containerlist.append(None if rng.uniform() < 0.5 else "unplaced")
                    continue
                hid = int(rng.integers(0, 3)) if mode == 1 else (0 if mode == 4 else int(rng.integers(0, H)))
                base = float(rng.integers(50, 3000 if mode == 3 else 1200))
                if rng.uniform() < 0.05:
                    base = 0.0
                ipsm = IPSMConstant(base, base * float(rng.uniform(1.0, 4.0)), 10, 1.5)
                rm = RMConstant(float(rng.uniform(20, 2500 if mode == 3 else 900)), 0.0, 0.0)
                dm = DMConstant(float(rng.uniform(10, 600)), 0.0, 0.0)
                sim.containerlist.append(Container(c, c, 0, ipsm, rm, dm, sim, HostID=hid))
            for c in range(H):
                if sim.containerlist[c] == "unplaced":  # a live container not yet placed: hostid -1
                    sim.containerlist[c] = Container(c, c, 0, IPSMConstant(300.0, 600.0, 10, 1.5),
                                                     RMConstant(100.0, 0.0, 0.0), DMConstant(50.0, 0.0, 0.0), sim,
                                                     HostID=-1)
            n_met = int(rng.integers(0, 9)) if e % 11 else 0
            metrics = [{"avgresponsetime": float(rng.uniform(0, 40))} for _ in range(n_met)]
            stats = types.SimpleNamespace(env=sim, metrics=metrics,
                                          simulated_scheduler=types.SimpleNamespace(env=sim))
            stats.simulated_scheduler.filter_placement = types.MethodType(filt, stats.simulated_scheduler)
            stats.runSimulation = types.MethodType(run_sim, stats)

            # generator-like schedule: sigmoid-range values with injected ties, and the original (one-hot)
            new = rng.uniform(0, 1, (H, H)).astype(np.float32)
            for r in range(H):
                u = rng.uniform()
                if u < 0.1:
                    new[r, :] = np.float32(0.5)  # all tied: first column
                elif u < 0.25:
                    j = rng.choice(H, 2, replace=False)
                    new[r, j] = new[r].max()  # two-way tie at the max
            orig = np.zeros((H, H), np.float32)
            cur = [c.getHostID() if c else -1 for c in sim.containerlist]
            for r in range(H):
                orig[r, cur[r] if (cur[r] >= 0 and rng.uniform() < 0.6) else rng.integers(0, H)] = 1.0
            if e % 7 == 3:
                new = orig.copy()  # generator returns the original: equal scores -> label [0, 1]

            row = []
            for s in (new, orig):
                t = torch.tensor(s, dtype=torch.double)
                try:
                    en, lat = stats.runSimulation(t)
                    sc = run_simulation(stats, t)
                except IndexError:  # PM.powerFromCPU past its table: the reference raises
                    en, sc = float("nan"), float("nan")
                row += [float(en), float(sc)]
            envs.append(pack_env(sim, metrics))
            news.append(new)
            origs.append(orig)
            ref.append(row)
        ref = np.array(ref)
        target = np.where((ref[:, 1] <= ref[:, 3])[:, None], [0.0, 1.0], [1.0, 0.0]).astype(np.float32)
        np.savez_compressed(os.path.join(OUT, f"sim_h{H}.npz"), envs=np.stack(envs), new=np.stack(news),
                            orig=np.stack(origs), ref=ref, target=target)
        print(H, "envs", len(envs), "labels new<=orig:", int(target[:, 1].sum()), "nan:", int(np.isnan(ref).any(1).sum()))


if __name__ == "__main__":
    main()
