"""Per-kernel stall breakdown from one rocprofv3 --pmc pass of
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (MI355X_MICROARCH.md §PMC):
fractions of wave cycles, MFMA pipe busy = MFMA_BUSY / (SIMDs x GUI_ACTIVE/XCDs).
usage: python tools/pmc_stalls.py <run_counter_collection.csv> [n_simd=1024] [n_xcd=8]"""
import collections
import csv
import sys


def main(path, n_simd=1024, n_xcd=8):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "pgp::" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        wc = d["SQ_WAVE_CYCLES"] or 1
        cyc = d["GRBM_GUI_ACTIVE"] / n_xcd
        print(f"{k[-40:]:40s} parked {d['SQ_WAIT_ANY'] / wc:5.2f}  issue-stall {d['SQ_WAIT_INST_ANY'] / wc:5.2f}  "
              f"active {d['SQ_ACTIVE_INST_ANY'] / wc:5.2f}  lds-stall {d['SQ_WAIT_INST_LDS'] / wc:5.2f}  "
              f"mfma-busy {d['SQ_VALU_MFMA_BUSY_CYCLES'] / (n_simd * cyc) if cyc else 0:5.2f}")


if __name__ == "__main__":
    main(sys.argv[1], *[int(x) for x in sys.argv[2:]])
