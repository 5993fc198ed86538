"""CPU baseline of the decision path — TEST / BENCH INFRASTRUCTURE.

Imported only by bench.py's ``cpu_baseline`` leg (and its tests): the timed CPU
restatement of the reference, never the product.  Two modes, as BASELINE.md §4
asks:

1. ``reference_faithful``: one window at a time in fp64, in ``run_model``'s
   operation order and with its per-host Python loops —
   encoder forward (``models.py:376-416``), the per-host argmax loop that builds
   the embedding (``PreGANPlus.py:119-131``), ``get_classes``' per-(host,
   prototype) ``torch.mean`` loop (``utils.py:102-109``), Gen/Disc forward and
   the keep test (``PreGANPlus.py:84-87``), the per-container
   ``list.index(max(list))`` targets (``PreGANPlus.py:98-99``) and the
   generator proposal's row argmaxes (``stats/Stats.py:162-166``).  No training,
   plotting or checkpoint side effects.
2. ``batched_fp32``: the same math batched over windows in fp32 torch-CPU
   (oracle/pregan_train_oracle.py's forward pieces).

Threads: the CPUs this process may run on (``os.sched_getaffinity``), capped by
``OMP_NUM_THREADS`` when set (16 on the GPU box: the box's CPU share per GPU);
both are reported beside the count used.  Warm-up, median of 5 repeats.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import pregan_train_oracle as TO


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


THREADS_NOTE = ("threads = the CPUs in this process's affinity mask (os.sched_getaffinity), capped by "
                "OMP_NUM_THREADS when set (the box's CPU share per GPU); os.cpu_count() counts the whole host")


def affinity_cpus() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def host_threads() -> int:
    n = affinity_cpus()
    env = os.environ.get("OMP_NUM_THREADS")
    return min(n, int(env)) if env and env.isdigit() and int(env) > 0 else n


def thread_report() -> dict:
    """What the thread count was derived from (reported in every cpu_baseline)."""
    return {"threads": host_threads(), "affinity_cpus": affinity_cpus(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "host_cpus": os.cpu_count(),
            "threads_note": THREADS_NOTE}


def _tensors(weights, dtype):
    t = lambda sd: {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in sd.items()}
    return t(weights["transformer"]), t(weights["gen"]), t(weights["disc"])


def reference_faithful_window(tw, gw, dw, prototypes, win, s):
    """One window, fp64, run_model's forward order (see module docstring).
    win [1,3,3H], s [H,H] (fp64 tensors); prototypes: list of [2] tensors."""
    with torch.no_grad():
        logits, protos = TO.decode_t(tw, TO.encode_t(tw, win))
        H = logits.shape[1]
        embedding, anomaly = [], False
        for i in range(H):                                     # PreGANPlus.py:120-131
            if torch.argmax(logits[0, i]).item() == 1:
                anomaly = True
                embedding.append(protos[0, i])
            else:
                embedding.append(torch.zeros_like(protos[0, i]))
        emb = torch.stack(embedding)
        classes = []
        for e in emb:                                          # utils.py:102-109
            if torch.all(e == 0):
                classes.append(-1)
                continue
            d = [torch.mean((e - p) ** 2).item() for p in prototypes]
            classes.append(int(np.argmin(d)))
        ns = TO.gen_t(gw, emb[None], s[None])[0]
        probs = TO.disc_t(dw, s[None], ns[None])[0]
        keep = bool(probs[0] > probs[1])                      # PreGANPlus.py:87
        final = [row.index(max(row)) for row in s.tolist()]    # PreGANPlus.py:98-99
        gen = [row.index(max(row)) for row in ns.tolist()]     # Stats.py:164-166
    return anomaly, classes, keep, final, gen


def batched_fp32(tw, gw, dw, P, win, s):
    with torch.no_grad():
        logits, protos = TO.decode_t(tw, TO.encode_t(tw, win))
        anom = logits[..., 1] > logits[..., 0]
        emb = torch.where(anom[..., None], protos, torch.zeros_like(protos))
        dist = ((emb[:, :, None, :] - P[None, None]) ** 2).mean(-1)
        cls = torch.where(anom, dist.argmin(-1), torch.full_like(anom, -1, dtype=torch.long))
        ns = TO.gen_t(gw, emb, s)
        probs = TO.disc_t(dw, s, ns)
        return cls, probs[:, 0] > probs[:, 1], s.argmax(-1), ns.argmax(-1)


def measure(weights, windows, sched, per_window_n=256, batch_n=1024, repeats=5):
    """windows [N,3,3H], sched [N,H,H] (numpy, the GPU run's own inputs; N >=
    batch_n).  Returns the cpu_baseline object for bench.py (host-windows/s)."""
    H = windows.shape[2] // 3
    threads = host_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        tw, gw, dw = _tensors(weights, torch.float64)
        P64 = [torch.tensor(np.asarray(p, dtype=np.float64)) for p in weights["prototypes"]]
        xw = torch.tensor(np.asarray(windows[:per_window_n], np.float64))
        sw = torch.tensor(np.asarray(sched[:per_window_n], np.float64))
        reference_faithful_window(tw, gw, dw, P64, xw[:1], sw[0])          # warm-up
        pw = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            for i in range(per_window_n):
                reference_faithful_window(tw, gw, dw, P64, xw[i:i + 1], sw[i])
            pw.append(per_window_n * H / (time.perf_counter() - t0))
        tw32, gw32, dw32 = _tensors(weights, torch.float32)
        P32 = torch.tensor(np.asarray(weights["prototypes"]), dtype=torch.float32)
        xb = torch.tensor(np.asarray(windows[:batch_n], np.float32))
        sb = torch.tensor(np.asarray(sched[:batch_n], np.float32))
        batched_fp32(tw32, gw32, dw32, P32, xb[:64], sb[:64])                 # warm-up
        bt = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            batched_fp32(tw32, gw32, dw32, P32, xb, sb)
            bt.append(batch_n * H / (time.perf_counter() - t0))
    finally:
        torch.set_num_threads(prev)
    rf, bf = float(np.median(pw)), float(np.median(bt))
    return {
        "value": rf, "unit": "host-windows/s", "cores": threads, "kind": "port",
        "sample": (f"reference-faithful mode: {per_window_n} windows one at a time, fp64 torch-CPU in run_model's op "
                   f"order (per-host Python loops), median of {repeats}; the GPU run's own first windows (H={H})"),
        "modes": {"reference_faithful_fp64": {"value": rf, "windows_per_repeat": per_window_n,
                                              "repeats": [float(v) for v in pw]},
                  "batched_fp32": {"value": bf, "windows_per_repeat": batch_n,
                                   "repeats": [float(v) for v in bt]}},
        "cpu_model": cpu_model(), **thread_report(),
    }
