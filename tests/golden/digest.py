"""Compact, deterministic digests of large parameter / gradient tensors for the
H=50 training fixtures (the full H=50 decoders are 1.5 M values per snapshot).

A tensor with at most FULL values is stored whole.  A larger one is stored as
(i) a fixed sample of SAMPLE entries (indices drawn from a generator seeded by a
CRC of the tensor name, so the fixture generator and the tests draw the same
ones), (ii) its row sums and (iii) its column sums (2-D), in fp64.  Sums see every
entry, the sample pins individual values.
"""
import zlib

import numpy as np

FULL = 40000
SAMPLE = 20000


def sample_index(name, n):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    return np.sort(rng.choice(n, size=min(SAMPLE, n), replace=False))


def digest(name, a, key=None):
    """key: seeds the sample indices (default: name) — snapshots of one
    parameter (gradient, values after step 1 / 10) share a key, so their
    samples are the same entries."""
    a = np.asarray(a, dtype=np.float64)
    if a.size <= FULL:
        return {f"{name}/full": a.copy()}
    flat = a.reshape(-1)
    out = {f"{name}/sample": flat[sample_index(key or name, flat.size)]}
    m = a.reshape(a.shape[0], -1)
    out[f"{name}/rows"] = m.sum(axis=1)
    out[f"{name}/cols"] = m.sum(axis=0)
    out[f"{name}/rows_abs"] = np.abs(m).sum(axis=1)
    out[f"{name}/cols_abs"] = np.abs(m).sum(axis=0)
    return out


def parts(z, name):
    """Digest entries of `name` present in the npz-like mapping z."""
    return {k[len(name) + 1:]: z[k] for k in (f"{name}/full", f"{name}/sample", f"{name}/rows", f"{name}/cols")
            if k in z}


def check(z, name, got, cmp, sum_rel=None, key=None):
    """Digest `got` the way the fixture stored `name` and call
    cmp(got_part, want_part, label) for the full / sampled values; row and
    column sums are checked here, |got - want| <= sum_rel * (sum of |entries|)
    (sum_rel: the relative accuracy expected of single entries)."""
    want = parts(z, name)
    assert want, f"{name}: not in the fixture"
    mine = parts(digest(name, got, key), name)
    for k, v in want.items():
        if k in ("rows", "cols"):
            if sum_rel is None:
                continue
            tol = sum_rel * z[f"{name}/{k}_abs"] + 1e-300
            bad = np.abs(mine[k] - v) > tol
            assert not bad.any(), (f"{name}/{k}: {bad.sum()} of {bad.size} off, max err/tol "
                                   f"{(np.abs(mine[k] - v) / tol).max():.3g}")
        else:
            cmp(mine[k], v, f"{name}/{k}")
