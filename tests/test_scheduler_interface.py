"""GOBIScheduler honours the scheduler plugin interface COSCO drives
(scheduler/Scheduler.py:9-38 via main.py:154-155 and Simulator.py:118,
173-174), checked on CPU with a fake env and a stub placement (the GOBI kernel
itself is tested in test_gpu_gobi.py)."""
from preganplus_amd.gobi import GOBIScheduler, Scheduler


class _C:
    def __init__(self, cid, hid):
        self.id, self.h = cid, hid

    def getHostID(self):
        return self.h


class _Env:
    def __init__(self, hosts):
        self.containerlist = [_C(c, h) for c, h in enumerate(hosts)]

    def getContainerByID(self, cid):
        return self.containerlist[cid]


class _StubGOBI(GOBIScheduler):
    def __init__(self, decision):   # no device: the optimiser is not built
        Scheduler.__init__(self)
        self._decision = decision

    def run_GOBI(self):
        return list(self._decision)


def test_main_py_call_sequence():
    env = _Env([0, 1, 1, 2])
    s = _StubGOBI([(0, 0), (1, 2), (2, 1), (3, 0)])
    s.setEnvironment(env)
    selected = s.selection()                                        # main.py:154
    assert selected == []
    decision = s.filter_placement(s.placement(selected + [3]))      # main.py:155
    assert decision == [(1, 2), (3, 0)]
    assert s.getMigrationFromHost(1, decision) == [1]               # Simulator.py:173
    assert s.getMigrationToHost(0, decision) == [3]                 # Simulator.py:118, 174
    assert s.getMigrationToHost(1, decision) == []


def test_interface_methods_present():
    for m in ("setEnvironment", "selection", "placement", "filter_placement", "getMigrationFromHost",
              "getMigrationToHost", "run_GOBI"):
        assert callable(getattr(GOBIScheduler, m)), m
    assert issubclass(GOBIScheduler, Scheduler)
