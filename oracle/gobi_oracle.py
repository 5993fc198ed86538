"""CPU restatement of GOBI's schedule optimiser — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, smoke() and bench.py's CPU baseline, never by the
product.  Restates, in fp32 torch on the CPU (the reference's own dtype here:
GOBI builds its input with dtype=torch.float, scheduler/GOBI.py:33):

* the energy_latency_16 surrogate (scheduler/BaGTI/src/models.py:8-27):
  Linear(288,128) Softplus Linear(128,128) Softplus Linear(128,64) Tanhshrink
  Linear(64,2) Sigmoid, then z = 0.8 e + 0.2 l (Coeff_Energy/Latency,
  src/constants.py:6-7);
* opt() (scheduler/BaGTI/src/opt.py:17-33): torch.optim.AdamW(lr=0.8) with its
  defaults (betas 0.9/0.999, eps 1e-8, weight_decay 1e-2) on the input matrix,
  CosineAnnealingLR(T_max=10) stepped per iteration (torch's recursive form),
  then convertToOneHot (opt.py:9-15): each row's allocation part becomes the
  one-hot of its first argmax and the cpu columns are restored; stop when the
  allocation is unchanged for 31 consecutive steps, or after 200 iterations.
* run_GOBI's decision list (scheduler/GOBI.py:36-42).

Pinned by tests/test_gobi_oracle.py against tests/golden/gobi_h16.npz, made by
the reference's own opt() (tests/golden/make_golden_gobi.py): bit-identical.
"""
from __future__ import annotations

import math

import numpy as np
import torch

COEFF_ENERGY, COEFF_LATENCY = 0.8, 0.2
LR, T_MAX, WD, BETAS, EPS = 0.8, 10, 1e-2, (0.9, 0.999), 1e-8
MAX_IT, PATIENCE = 200, 30


def load(path):
    z = np.load(path)
    return {k: torch.tensor(z[k]) for k in z.files if k != "max_ips"}, float(z["max_ips"])


def surrogate(sd, x):
    """models.py:22-27 (forward on the flattened [C, 2+H] input)."""
    f = torch.nn.functional
    h = x.flatten()
    h = f.softplus(f.linear(h, sd["find.0.weight"], sd["find.0.bias"]))
    h = f.softplus(f.linear(h, sd["find.2.weight"], sd["find.2.bias"]))
    h = f.tanhshrink(f.linear(h, sd["find.4.weight"], sd["find.4.bias"]))
    o = torch.sigmoid(f.linear(h, sd["find.6.weight"], sd["find.6.bias"]))
    return COEFF_ENERGY * o[0] + COEFF_LATENCY * o[1]


def cosine_lrs(n=MAX_IT, base=LR, t_max=T_MAX):
    """lr used by the AdamW step of iteration i: CosineAnnealingLR's recursive
    update (torch/optim/lr_scheduler.py, eta_min 0), one scheduler.step() per
    iteration after optimizer.step()."""
    lrs, lr = [], base
    for epoch in range(n):
        lrs.append(lr)
        e = epoch + 1
        if (e - 1 - t_max) % (2 * t_max) == 0:
            lr = lr + base * (1 - math.cos(math.pi / t_max)) / 2
        else:
            lr = (1 + math.cos(math.pi * e / t_max)) / (1 + math.cos(math.pi * (e - 1) / t_max)) * lr
    return lrs


def adamw_constants(n=MAX_IT):
    """Per-iteration scalars of torch's single-tensor AdamW (step = i + 1):
    decay factor 1 - lr*wd, step size lr / (1 - b1^step), sqrt(1 - b2^step)."""
    out = []
    for i, lr in enumerate(cosine_lrs(n)):
        step = i + 1
        out.append((1 - lr * WD, lr / (1 - BETAS[0] ** step), math.sqrt(1 - BETAS[1] ** step)))
    return out


def opt(sd, init, hosts=16, max_it=MAX_IT, return_pre=False):
    """opt.py:17-33 on one init [C, 2+H] (numpy or tensor).  Returns
    (result [C, 2+H] float32, iterations, fitness) and, with return_pre, the
    last step's allocation values before the one-hot projection."""
    x = torch.tensor(np.asarray(init), dtype=torch.float32).clone().requires_grad_(True)
    m = torch.zeros_like(x)
    v = torch.zeros_like(x)
    consts = adamw_constants()
    equal, it, pre = 0, 0, None
    while it < max_it:
        cpu_old = x.data[:, :-hosts].clone()
        alloc_old = x.data[:, -hosts:].clone()
        z = surrogate(sd, x)
        x.grad = None
        z.backward()
        decay, step_size, bc2s = consts[it]
        g = x.grad
        with torch.no_grad():
            x.mul_(decay)
            m.lerp_(g, 1 - BETAS[0])
            v.mul_(BETAS[1]).addcmul_(g, g, value=1 - BETAS[1])
            denom = (v.sqrt() / bc2s).add_(EPS)
            x.addcdiv_(m, denom, value=-step_size)
            alloc = x.data[:, -hosts:]
            pre = alloc.clone()
            onehot = torch.zeros_like(alloc)
            onehot[torch.arange(alloc.shape[0]), first_argmax(alloc)] = 1.0
            x.data = torch.cat([cpu_old, onehot], dim=1)
        equal = equal + 1 if torch.all(alloc_old.eq(x.data[:, -hosts:])) else 0
        if equal > PATIENCE:
            break
        it += 1
    x.requires_grad_(False)
    if return_pre:
        return x.data.numpy(), it, float(surrogate(sd, x)), pre.numpy()
    return x.data.numpy(), it, float(surrogate(sd, x))


def first_argmax(a):
    """list.index(max(list)) per row (opt.py:12): the first maximal element."""
    mx = a.max(dim=1, keepdim=True).values
    idx = torch.arange(a.shape[1]).expand_as(a)
    return torch.where(a == mx, idx, a.shape[1]).min(dim=1).values


def decision(result, prev_alloc, hosts=16):
    """GOBI.py:37-41: (cid, new_host) for containers whose host changes."""
    out = []
    for cid, h in prev_alloc.items():
        row = list(np.asarray(result)[cid, -hosts:])
        new_host = row.index(max(row))
        if h != new_host:
            out.append((cid, new_host))
    return out
