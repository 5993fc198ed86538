"""Trainer.adam_schedule_np (the vectorised AdamW table of the tuning graph)
against the per-step reference loop Trainer.adam_schedule: identical fp32
tables and step counts (CPU; the C-ABI's host-side size queries only)."""
import numpy as np

from preganplus_amd import weights as W


def test_adam_schedule_np_matches_loop():
    from preganplus_amd import train as TR
    w = W.synth_weights(16, seed=1)
    a = TR.Trainer(16, w, None, device="cpu", max_batch=1)
    b = TR.Trainer(16, w, None, device="cpu", max_batch=1)
    cond = ("prototype_decoder.0.weight", "prototype_decoder.0.bias")
    rng = np.random.default_rng(0)
    for call in range(4):
        pos = rng.random(10) < 0.6
        if call == 0:
            pos[:3] = False            # cond tensors at step 0 (bias correction at max(step, 1))
        _, ta = a.adam_schedule("transformer", [() if p else cond for p in pos])
        tb = b.adam_schedule_np("transformer", pos, cond)
        np.testing.assert_array_equal(ta, tb)
        assert [t["step"] for t in a.tensors] == [t["step"] for t in b.tensors]
