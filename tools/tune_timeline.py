"""Per-step timeline of a C3 run from a rocprofv3 kernel trace
(`rocprofv3 --kernel-trace --output-format csv`): the steps are cut at each
`tune_dataset_kernel`, and for every kernel of a step (in issue order) the
median start offset from the step start, median duration and queue are
printed, followed by the busy / idle split of the tuning path.
usage: python tools/tune_timeline.py <kernel_trace.csv> [skip_steps]"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np


def short(name):
    n = re.sub(r"^(void )?pgp::\(anonymous namespace\)::", "", name)
    n = re.sub(r"\(.*", "", n)
    return n[:48]


def main(path, skip=3):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        n = short(r["Kernel_Name"])
        if n.startswith("tune_dataset_kernel"):
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?")))
    steps = steps[skip:-1]
    if not steps:
        print("no complete steps")
        return
    spans = []
    table = defaultdict(list)
    for st in steps:
        t0 = st[0][1]
        spans.append((max(e for _, _, e, _ in st) - t0) / 1e3)
        seen = defaultdict(int)
        for n, s, e, q in st:
            k = (n, seen[n], q)
            seen[n] += 1
            table[k].append(((s - t0) / 1e3, (e - s) / 1e3))
    print(f"{len(steps)} steps, span median {np.median(spans):.1f} us (min {min(spans):.1f})")
    order = sorted(table, key=lambda k: np.median([a for a, _ in table[k]]))
    for k in order:
        v = np.array(table[k])
        s, d = np.median(v[:, 0]), np.median(v[:, 1])
        print(f"  q{k[2]:>3} {s:8.1f} +{d:7.1f} -> {s + d:8.1f}  {k[0]}#{k[1]}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
