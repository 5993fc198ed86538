"""Trainer.forward_context (the C3 detect beside the tuning step): a forward in
its own workspace gives the same outputs as the plain forward and leaves the
tuning step's activations alone (a backward after it equals one without it);
DPTuner.step(before_update=) orders the update after another stream's work."""
import numpy as np
import pytest
import torch

from preganplus_amd import train as TR
from preganplus_amd import weights as W

pytestmark = pytest.mark.gpu


def test_forward_context_is_independent():
    H, B, Bd = 50, 64, 16
    w = W.synth_weights(H, seed=0)
    rng = np.random.Generator(np.random.PCG64(5))
    x = torch.tensor(rng.uniform(0, 0.8, size=(B, 3, 3 * H)).astype(np.float32), device="cuda")
    xd = torch.tensor(rng.uniform(0, 0.8, size=(Bd, 3, 3 * H)).astype(np.float32), device="cuda")
    y = (rng.uniform(size=(B, H)) < 0.2).astype(np.int32)
    mult = rng.uniform(0.5, 2.0, size=(B, H)).astype(np.float32)
    tgt = rng.uniform(size=(B, H, 2)).astype(np.float32)
    grads, outs = [], []
    for with_ctx in (False, True):
        tr = TR.Trainer(H, w, max_batch=B)
        ctx = tr.forward_context(Bd)
        tr.tune_forward(x)
        if with_ctx:   # a detect forward between the tuning forward and its backward
            lg, pr = tr.tune_forward(xd, ctx=ctx)
            outs.append((lg.clone(), pr.clone()))
        tr.tune_backward(B, y, mult, tgt)
        grads.append(tr.G.clone())
    torch.testing.assert_close(grads[0], grads[1], rtol=0, atol=0)
    tr = TR.Trainer(H, w, max_batch=B)
    lg, pr = tr.tune_forward(xd)
    torch.testing.assert_close(outs[0][0], lg, rtol=0, atol=0)
    torch.testing.assert_close(outs[0][1], pr, rtol=0, atol=0)
