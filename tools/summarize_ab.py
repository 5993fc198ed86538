"""Collapse an A/B study directory of bench JSON lines (one file per variant
and repeat, e.g. `k2_units/w12_c8.2.json`) into one SUMMARY.md table and
delete the per-run files: the numbers DESIGN.md quotes stay, the directory
stops holding dozens of near-duplicate artifacts.  Text notes
(*.txt, *.md) in the directory are kept.
usage: python tools/summarize_ab.py DIR [DIR ...]"""
import glob
import json
import os
import sys


def row(path):
    txt = open(path).read()
    i = txt.find("{")
    d = json.loads(txt[i:]) if i >= 0 else {}
    name = os.path.basename(path)[:-5]
    ms = d.get("ms_per_step")
    km = d.get("kernel_ms") or d.get("stage_ms") or {}
    frac = (d.get("roofline") or {}).get("frac")
    cfg = (d.get("config") or {}).get("workload", "")
    return name, ms, km, frac, cfg


def summarize(dirpath):
    files = sorted(glob.glob(os.path.join(dirpath, "*.json")))
    if not files:
        return 0
    rows = [row(f) for f in files]
    keys = []
    for r in rows:
        for k in r[2]:
            if k not in keys:
                keys.append(k)
    out = [f"# {os.path.basename(os.path.normpath(dirpath))}: A/B runs (one row per run file, collapsed by "
           f"tools/summarize_ab.py)", "",
           "| run | ms/step | " + " | ".join(f"{k} ms" for k in keys) + " | roofline frac | workload |",
           "|---|---|" + "---|" * len(keys) + "---|---|"]
    for name, ms, km, frac, cfg in rows:
        cells = [f"{km[k]:.4f}" if isinstance(km.get(k), (int, float)) else "" for k in keys]
        out.append(f"| {name} | {ms:.4f} | " if isinstance(ms, (int, float)) else f"| {name} | | ")
        out[-1] += " | ".join(cells) + f" | {frac:.4f} | " if isinstance(frac, float) else " | ".join(cells) + " | | "
        out[-1] += f"{cfg[:60]} |"
    with open(os.path.join(dirpath, "SUMMARY.md"), "w") as f:
        f.write("\n".join(out) + "\n")
    for fpath in files:
        os.remove(fpath)
    return len(files)


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(d, summarize(d))
