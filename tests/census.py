"""Full-scale decision census — TEST INFRASTRUCTURE (checker only).

Runs the fp64 oracle over EVERY window of a full BASELINE launch and compares
the HIP outputs with it window by window (tests/decision_bounds.py).  The
oracle work is split into chunks over a pool of CPU worker processes (spawned
fresh: they import numpy and the oracle only, never torch or the GPU), one BLAS
thread each, so a 65,536-window H=50 census takes seconds of wall time.
"""
from __future__ import annotations

import multiprocessing as mp
import os

import numpy as np

from oracle import pregan_oracle as O
from tests import decision_bounds as DB

_W = None
_LIMITS = None


def _init(weights):
    global _W, _LIMITS
    from threadpoolctl import threadpool_limits
    _LIMITS = threadpool_limits(limits=1)
    _W = weights


def _envelope_ratio(g, r, atol, ok=None):
    g, r = np.asarray(g, np.float64), np.asarray(r, np.float64)
    if ok is not None:
        g, r = g[ok], r[ok]
    if g.size == 0:
        return 0.0
    return float((np.abs(g - r) / DB.envelope(r, atol)).max())


def _chunk(task):
    """One chunk: fp64 oracle forward of the chunk's windows, then the census
    and the worst |got - ref| / tolerance ratio of the continuous outputs."""
    x32, sidx, got = task
    B, H = sidx.shape
    s = np.zeros((B, H, H))
    s[np.arange(B)[:, None], np.arange(H)[None, :], sidx] = 1.0
    ref = O.forward(_W, x32.astype(np.float64), s)
    st = DB.compare(got, ref, _W, s)
    lr = ref["logits"]
    ok = ((got["logits"][..., 1] > got["logits"][..., 0]) == (lr[..., 1] > lr[..., 0])).all(axis=1)
    err = {"logits": _envelope_ratio(got["logits"], lr, DB.ATOL_LOGIT),
           "protos": _envelope_ratio(got["protos"], ref["protos"], DB.ATOL_PROB),
           "probs": _envelope_ratio(got["probs"], ref["probs"], DB.ATOL_PROB, ok),
           "logits_max_abs": float(np.abs(got["logits"] - lr).max()),
           "logits_max_rel": float((np.abs(got["logits"] - lr) / np.maximum(np.abs(lr), 1e-3)).max())}
    return st, err


def _chunk_fpe(task):
    """One chunk of the PreGAN (FPE) variant: the anomaly softmax plays the
    detect logits' role, the discriminator probs are 'probs'."""
    x32, h0, sidx, got = task
    B, H = sidx.shape
    s = np.zeros((B, H, H))
    s[np.arange(B)[:, None], np.arange(H)[None, :], sidx] = 1.0
    r = O.forward_fpe(_W, x32.astype(np.float64), h0.astype(np.float64), s)
    ref = dict(r, logits=r["probs"], probs=r["gprobs"])
    st = DB.compare(got, ref, _W, s)
    lr = ref["logits"]
    ok = ((got["logits"][..., 1] > got["logits"][..., 0]) == (lr[..., 1] > lr[..., 0])).all(axis=1)
    err = {"logits": _envelope_ratio(got["logits"], lr, DB.ATOL_PROB),
           "protos": _envelope_ratio(got["protos"], ref["protos"], DB.ATOL_PROB),
           "probs": _envelope_ratio(got["probs"], ref["probs"], DB.ATOL_PROB, ok),
           "logits_max_abs": float(np.abs(got["logits"] - lr).max()),
           "logits_max_rel": float((np.abs(got["logits"] - lr) / np.maximum(np.abs(lr), 1e-3)).max())}
    return st, err


def run(weights, x32, sidx, got, workers=None, chunk=2048, log=None, h0=None):
    """x32 [B,3,3H] float32 windows, sidx [B,C] int one-hot schedule columns,
    got: HIP outputs (numpy, full launch).  h0 [B,3]: the PreGAN (FPE)
    variant's GRU states (got['logits'] = its anomaly softmax).  Returns
    (census, worst error ratios)."""
    B = x32.shape[0]
    workers = workers or min(16, os.cpu_count() or 1)
    keys = ("logits", "protos", "probs", "cls", "any", "keep", "final_target", "gen_target")
    if h0 is None:
        fn = _chunk
        tasks = [(x32[i:i + chunk], sidx[i:i + chunk], {k: got[k][i:i + chunk] for k in keys})
                 for i in range(0, B, chunk)]
    else:
        fn = _chunk_fpe
        tasks = [(x32[i:i + chunk], h0[i:i + chunk], sidx[i:i + chunk], {k: got[k][i:i + chunk] for k in keys})
                 for i in range(0, B, chunk)]
    stats, errs = [], []
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers, initializer=_init, initargs=(weights,)) as pool:
        for i, (st, err) in enumerate(pool.imap(fn, tasks)):
            stats.append(st)
            errs.append(err)
            if log is not None and (i + 1) % 8 == 0:
                log(f"census: {min((i + 1) * chunk, B)}/{B} windows")
    worst = {k: max(e[k] for e in errs) for k in errs[0]}
    return DB.merge(stats), worst
