"""Per-kernel stall split from several rocprofv3 --pmc passes (one counter group
per run, MI355X_MICROARCH.md §PMC), merged by kernel name:
  parked       SQ_WAIT_ANY / SQ_WAVE_CYCLES        (waves waiting on a counter / barrier)
  issue-stall  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (waves ready but not issued)
  active       SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  lds-stall    SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  VALU / MFMA  SQ_INSTS_VALU / SQ_INSTS_MFMA (VALU counts include the MFMAs' AGPR moves)
  mfma-busy    SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / XCDs), when a pass
               holds GRBM_GUI_ACTIVE; else over (SIMDs x kernel ms x clock) with the
               durations of a kernel-stats csv (--stats, 2.4 GHz)
usage: python tools/pmc_split.py DIR... [--stats kernel_stats.csv] [--match SUBSTR]"""
import collections
import csv
import glob
import os
import re
import sys

N_SIMD, N_XCD, CLOCK_GHZ = 1024, 8, 2.4


def short(name):
    n = re.sub(r"^(void )?pgp::\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*", "", n)


def main(argv):
    stats, match, dirs = None, None, []
    it = iter(argv)
    for a in it:
        if a == "--stats":
            stats = next(it)
        elif a == "--match":
            match = next(it)
        else:
            dirs.append(a)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                per[(short(r["Kernel_Name"]), r.get("Dispatch_Id", ""))][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, _), cs in per.items():
                for c, v in cs.items():
                    acc[k][c].append(v)
    dur = {}
    if stats:
        for r in csv.DictReader(open(stats)):
            dur[short(r["Name"])] = float(r["AverageNs"]) * 1e-9
    for k in sorted(acc):
        if match and match not in k:
            continue
        d = {c: sum(v) / len(v) for c, v in acc[k].items()}
        wc = d.get("SQ_WAVE_CYCLES") or 0
        if not wc:
            continue
        f = lambda c: d.get(c, float("nan")) / wc
        line = (f"{k[:44]:44s} parked {f('SQ_WAIT_ANY'):5.2f} issue-stall {f('SQ_WAIT_INST_ANY'):5.2f} "
                f"active {f('SQ_ACTIVE_INST_ANY'):5.2f} lds-stall {f('SQ_WAIT_INST_LDS'):5.2f}")
        if d.get("SQ_INSTS_MFMA"):
            line += f" VALU/MFMA {d.get('SQ_INSTS_VALU', 0) / d['SQ_INSTS_MFMA']:5.2f}"
        busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if busy is not None:
            if d.get("GRBM_GUI_ACTIVE"):
                line += f" mfma-busy {busy / (N_SIMD * d['GRBM_GUI_ACTIVE'] / N_XCD):5.2f}"
            elif k in dur:
                line += f" mfma-busy {busy / (N_SIMD * dur[k] * CLOCK_GHZ * 1e9):5.2f} (from --stats)"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1:])
