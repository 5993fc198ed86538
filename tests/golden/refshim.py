"""Import shim for the reference PreGAN+ package (fixture generation ONLY).

Test infrastructure: used by ``make_golden.py`` in the build container, never by
the product, never on the GPU box (``/root/reference`` does not exist there).

The reference imports two third-party pieces that are absent from this image:

* ``dgl==0.7.2`` (pinned at reference ``README.md:42``).  The reference uses four
  of its primitives (``recovery/PreGANSrc/src/dlutils.py:7-8,319-346``,
  graph built at ``models.py:332-334``).  They are restated here from DGL's
  published API semantics:

  - ``dgl.graph((src, dst))``: a graph with ``edges()``, ``number_of_nodes()``,
    ``edata``/``ndata`` dicts and ``update_all``;
  - ``dgl.softmax_edges(g, 'e')``: DGL's *readout* softmax, i.e. a softmax of
    the edge feature over **all edges of the graph** (dim 0), independently for
    every trailing feature position (the graph-wise semantics SURVEY.md §0.3
    documents; the reference's inline comment claiming per-destination is not
    what the function does);
  - ``update_all(src_mul_edge('z','a','m'), sum('m','h'))``:
    ``h[v] = sum_{e: dst(e)=v} z[src(e)] * a[e]``;
  - ``dgl.nn.pytorch.GATConv``: imported but never instantiated by the path, a
    placeholder class suffices.

* ``scienceplots``/``seaborn`` via ``plotter.py`` (imported by ``train.py``):
  plotting side effects only, replaced with an inert module.

Checkpoints are loaded with ``torch.load(weights_only=True)``; the only extra
global allowlisted is the one the safe loader itself names for these files
(``numpy.core.multiarray.scalar``, used by numpy scalars inside
``accuracy_list``) — no code from the files is executed.
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"


def _install_dgl_standin():
    if "dgl" in sys.modules:
        return
    dgl = types.ModuleType("dgl")

    class _Graph:
        def __init__(self, src, dst):
            self._src = torch.as_tensor(src, dtype=torch.long)
            self._dst = torch.as_tensor(dst, dtype=torch.long)
            self._n = int(max(self._src.max(), self._dst.max())) + 1
            self.edata = {}
            self.ndata = {}

        def edges(self):
            return self._src, self._dst

        def number_of_nodes(self):
            return self._n

        def update_all(self, message, reduce):
            zk, ak, mk = message
            mk2, hk = reduce
            assert mk == mk2
            z = self.ndata[zk]
            a = self.edata[ak]
            m = z[self._src] * a
            out = torch.zeros((self._n,) + tuple(m.shape[1:]), dtype=m.dtype)
            out.index_add_(0, self._dst, m)
            self.ndata[hk] = out

    def graph(edges):
        src, dst = edges
        return _Graph(src, dst)

    def softmax_edges(g, key):
        return torch.softmax(g.edata[key], dim=0)

    fn = types.ModuleType("dgl.function")
    fn.src_mul_edge = lambda z, a, m: (z, a, m)
    fn.sum = lambda m, h: (m, h)

    nn_mod = types.ModuleType("dgl.nn")
    pt = types.ModuleType("dgl.nn.pytorch")

    class GATConv(torch.nn.Module):
        pass

    pt.GATConv = GATConv
    nn_mod.pytorch = pt
    dgl.graph = graph
    dgl.softmax_edges = softmax_edges
    dgl.function = fn
    dgl.nn = nn_mod
    sys.modules["dgl"] = dgl
    sys.modules["dgl.function"] = fn
    sys.modules["dgl.nn"] = nn_mod
    sys.modules["dgl.nn.pytorch"] = pt


def _install_plotter_standin():
    name = "recovery.PreGANSrc.src.plotter"
    if name in sys.modules:
        return
    m = types.ModuleType(name)

    class _Inert:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, _):
            return lambda *a, **k: None

    m.Model_Plotter = _Inert
    m.GAN_Plotter = _Inert
    sys.modules[name] = m


def import_reference():
    """Return (models, utils, train) modules of the reference package."""
    sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
    _install_dgl_standin()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    _install_plotter_standin()
    import recovery.PreGANSrc.src.models as models
    import recovery.PreGANSrc.src.utils as utils
    import recovery.PreGANSrc.src.train as train
    return models, utils, train


def safe_load_ckpt(path):
    sg = [(np._core.multiarray.scalar, "numpy.core.multiarray.scalar"), np.dtype,
          np.dtypes.Float64DType]
    with torch.serialization.safe_globals(sg):
        return torch.load(path, weights_only=True)


def ckpt_path(rel):
    return os.path.join(REF, "recovery/PreGANSrc", rel)
