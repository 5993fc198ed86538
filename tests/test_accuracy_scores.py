"""train.accuracy_scores (vectorised) against a loop restatement of the
reference's anomaly_accuracy / class_accuracy accumulation (train.py:60-109):
identical floats on random logits / prototypes, ties included."""
import numpy as np

from preganplus_amd import train as TR


def _loop(lg, pr, anom, cls, P):
    n, H = lg.shape[:2]
    ac = cc = ct = 0
    for i in range(n):
        res = (lg[i, :, 1] > lg[i, :, 0]).astype(np.int64)
        ac += int(np.sum(res == anom[i])) / H
        if np.sum(anom[i]) > 0:
            ct += 1
            correct, total = 0, 1e-4
            for h in range(H):
                if anom[i, h] > 0:
                    total += 1
                    c = int(cls[i, h])
                    pos = float(np.mean((pr[i, h] - P[c]) ** 2))
                    negs = [float(np.mean((pr[i, h] - P[nc]) ** 2)) for nc in (0, 1, 2) if nc != c]
                    if pos <= negs[0] and pos <= negs[1]:
                        correct += 1
            cc += correct / total
    return ac / n, cc / ct


def test_accuracy_scores_match_loop():
    rng = np.random.default_rng(0)
    for t in range(200):
        n, H = 10, (16 if t % 2 else 50)
        lg = rng.normal(size=(n, H, 2))
        pr = rng.uniform(size=(n, H, 2))
        anom = (rng.random((n, H)) < 0.3).astype(int)
        anom[0, 0] = 1
        cls = rng.integers(0, 3, (n, H))
        P = rng.uniform(size=(H, 2))
        if t % 3 == 0:
            pr[..., 0] = P[cls, 0]          # distance ties
            lg[..., 1] = lg[..., 0]         # argmax ties -> class 0
        assert TR.accuracy_scores(lg, pr, anom, cls, P) == _loop(lg, pr, anom, cls, P)
