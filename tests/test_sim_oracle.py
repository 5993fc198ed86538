"""The runSimulation oracle (f4) against the reference's own outputs
(tests/golden/make_golden_sim.py), and the record packer on a duck-typed env."""
import os
import types

import numpy as np
import pytest

from oracle import sim_oracle as S
from preganplus_amd import simulate as SIM

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("H", [16, 50])
def test_oracle_bit_exact_vs_reference(H):
    z = np.load(os.path.join(GOLD, f"sim_h{H}.npz"))
    out, target = S.simulate_batch(z["envs"], z["new"], z["orig"], H)
    assert np.array_equal(out, z["ref"]), np.abs(out - z["ref"]).max()
    assert np.array_equal(target, z["target"])


@pytest.mark.parametrize("H", [16, 50])
def test_fixtures_cover_edge_cases(H):
    """Moves refused by capacity, overloaded hosts (cpu clamp at 100), negative
    apparent IPS, ties, unplaced/empty slots and both label outcomes occur."""
    z = np.load(os.path.join(GOLD, f"sim_h{H}.npz"))
    o = SIM.offsets(H)
    refused = over = neg = unplaced = 0
    for v, new in zip(z["envs"], z["new"]):
        _, _, f = S.fields(v, H)
        host = np.array(f["host"], int)
        unplaced += int((host == -1).sum())
        neg += int((np.array(f["app_ips"]) < 0).sum())
        for c in np.nonzero(host >= 0)[0]:
            nh = int(np.argmax(new[c]))
            if nh != host[c] and not (f["base_ips"][c] <= f["ips_av"][nh] and f["ram"][c] <= f["ram_av"][nh]
                                      and f["disk"][c] <= f["disk_av"][nh]):
                refused += 1
        ips = np.zeros(H)
        np.add.at(ips, host[host >= 0], np.array(f["app_ips"])[host >= 0])
        over += int((ips > np.array(f["ips_cap"])).sum())
    assert refused > 0 and over > 0 and unplaced > 0
    assert z["target"][:, 0].sum() > 0 and z["target"][:, 1].sum() > 0
    assert o["power"][0] + o["power"][1] == SIM.env_len(H)


def test_power_from_cpu_python_semantics():
    pl = [float(i) for i in range(11)]
    assert S.power_from_cpu(pl, 100) == 10.0
    assert S.power_from_cpu(pl, 0.0) == 0.0
    assert S.power_from_cpu(pl, 55.0) == 5.5
    assert S.power_from_cpu(pl, -5.0) == pytest.approx(0.5 * 0 + 0.5 * 10)  # pl[-1] wraps, as in the reference
    with pytest.raises(IndexError):
        S.power_from_cpu(pl, -150.0)


def _fake_env(H):
    class C:
        def __init__(s, i, h):
            s.id, s.h = i, h

        def getHostID(s):
            return s.h

        def getBaseIPS(s):
            return 100.0 + s.id

        def getRAM(s):
            return 10.0 * s.id, 0, 0

        def getDisk(s):
            return 5.0 * s.id, 0, 0

        def getApparentIPS(s):
            return 150.5 + s.id

    class Hst:
        def __init__(s, i):
            s.i, s.ipsCap = i, 4000 + i
            s.powermodel = types.SimpleNamespace(powerlist=[float(i + k) for k in range(11)])

        def getIPSAvailable(s):
            return 1000.0 + s.i

        def getRAMAvailable(s):
            return 2000.0 + s.i, 0, 0

        def getDiskAvailable(s):
            return 3000.0 + s.i, 0, 0

    cl = [C(i, i % 3) if i % 4 else (None if i % 8 else C(i, -1)) for i in range(H)]
    return types.SimpleNamespace(hostlist=[Hst(i) for i in range(H)], containerlist=cl, intervaltime=300)


def test_pack_env_layout():
    H = 8
    env = _fake_env(H)
    v = SIM.pack_env(env, [{"avgresponsetime": 3.0}, {"avgresponsetime": 5.0}])
    o = SIM.offsets(H)
    g = lambda k: v[o[k][0]:o[k][0] + o[k][1]]  # noqa: E731
    assert v[0] == 300 and v[1] == 4.0
    assert list(g("host")) == [-1, 1, 2, 0, -1, 2, 0, 1]
    assert g("base_ips")[1] == 101.0 and g("base_ips")[0] == 0.0
    assert g("ips_cap")[3] == 4003 and g("power")[11 * 2 + 4] == 6.0
    assert SIM.pack_env(env, [])[1] == 0.0  # max(0, mean([])) -> 0, as Stats.py:177
    with pytest.raises(ValueError):
        SIM.pack_env(types.SimpleNamespace(hostlist=env.hostlist, containerlist=env.containerlist[:4],
                                           intervaltime=300), [])
