"""Multi-process (gloo, world_size 2, CPU) checks of the data-parallel paths.

* Tuning: each rank computes the gradients of its shard of
  windows; one flat all-reduce (sum) of the gradient buffer — the exact call
  Trainer.all_reduce_grads makes (RCCL on the GPU box, gloo here) — equals the
  gradient of the concatenated batch.  Gradients come from the torch training
  oracle (no GPU here).
* Inference sharding: bench.py gives every rank its own independent windows;
  the per-rank seeds differ and no collective touches the data path.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pregan_train_oracle as TO
from preganplus_amd import weights as W

H, B = 8, 4


def _batch_grads(w, x, y, mult, tgt):
    tw = TO.leaf_params(w["transformer"])
    logits, protos = TO.decode_t(tw, TO.encode_t(tw, torch.tensor(x)))
    ce = torch.nn.functional.cross_entropy(logits.reshape(-1, 2), torch.tensor(y.reshape(-1), dtype=torch.long),
                                           reduction="none").reshape(x.shape[0], H)
    loss = (ce * torch.tensor(mult)).sum() + (((protos - torch.tensor(tgt)) ** 2).mean(-1)
                                              * torch.tensor(y > 0)).sum()
    loss.backward()
    return torch.cat([tw[k].grad.reshape(-1) for k in tw if tw[k].grad is not None])


def _inputs():
    rng = np.random.Generator(np.random.PCG64(3))
    x = rng.uniform(0, 0.8, size=(B, 3, 3 * H))
    y = (rng.uniform(size=(B, H)) < 0.4).astype(np.int64)
    mult = rng.uniform(0.5, 2, size=(B, H))
    tgt = rng.uniform(0, 1, size=(B, H, 2))
    return x, y, mult, tgt


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = W.synth_weights(H, seed=1)
    x, y, mult, tgt = _inputs()
    sl = slice(rank * B // world, (rank + 1) * B // world)
    g = _batch_grads(w, x[sl], y[sl], mult[sl], tgt[sl])
    dist.all_reduce(g)  # Trainer.all_reduce_grads: one flat SUM all-reduce
    if rank == 0:
        q.put(g.numpy())
    dist.destroy_process_group()


def test_dp_gradient_allreduce_equals_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    g_dp = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    w = W.synth_weights(H, seed=1)
    g_full = _batch_grads(w, *_inputs()).numpy()
    np.testing.assert_allclose(g_dp, g_full, rtol=1e-10, atol=1e-12)


def test_trainer_allreduce_is_noop_without_process_group():
    """Single process: all_reduce_grads must not require torch.distributed."""
    from preganplus_amd import train as TR
    tr = TR.Trainer.__new__(TR.Trainer)
    tr.G = torch.arange(10, dtype=torch.float32)
    tr.sec_off, tr.sec_end = {"transformer": 0}, {"transformer": 10}
    tr.all_reduce_grads("transformer")
    assert tr.G.tolist() == list(range(10))
