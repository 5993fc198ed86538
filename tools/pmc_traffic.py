"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Correction (MI355X_MICROARCH.md §HBM, which states it for 16 B/lane reads;
measured here for every width the kernels use, tools/micro/fetch_cal.hip,
profiles/r05/fetch_cal/ratios.json): on gfx950 FETCH_SIZE reports exactly 1/2
of the bytes of a coalesced streaming read at 4, 8, 12 and 16 B per lane, and
WRITE_SIZE exactly the bytes stored at each of those widths.  We report both the raw counters and the corrected figure
(2 x FETCH + WRITE), in bytes per launch, averaged over the dispatches.

Each kernel<H> of the run is written to profiles/pmc_<kernel>_h<H>.json,
stamped with the batch, the run it came from and the sha256 of that kernel's
instructions in the library the counters were taken with
(tools/isa_count.kernel_isa_hash; run this right after the GPU call, against
the same in-tree build): bench.py reports the traffic only while the loaded
library's kernel hashes the same, and tests/test_roofline_isa.py fails when a
committed file is stale.
usage: python tools/pmc_traffic.py gpurun_out/<tag> BATCH H [kernel ...]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_count  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    root, batch, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    only = set(sys.argv[4:])
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/*pmc*/run_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(.*$", "", row["Kernel_Name"].replace("void pgp::(anonymous namespace)::", ""))
            vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, d in sorted(vals.items()):
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        fe = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024
        wr = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
        print(f"{k:28s} FETCH {fe / 1e6:10.1f} MB  WRITE {wr / 1e6:10.1f} MB  corrected {(2 * fe + wr) / 1e6:10.1f} MB"
              f"  (n={len(d['FETCH_SIZE'])})")
        m = re.match(r"(\w+?)_kernel<(\d+)((?:, (?:\d+|true|false))*)>", k)
        if not m or int(m.group(2)) != H or (only and m.group(1) not in only):
            continue
        # integer and bool template arguments (encoder_kernel<50, true>: the split form)
        targs = ([H] + [x.strip() == "true" if x.strip() in ("true", "false") else int(x)
                        for x in m.group(3).split(",")[1:]] if m.group(3) else None)
        h = isa_count.kernel_isa_hash(m.group(1) + "_kernel", H, targs=targs)
        out = {"fetch_bytes_raw": fe, "write_bytes": wr, "hbm_bytes_per_launch": 2 * fe + wr, "batch": batch,
               "kernel": k, "dispatches": len(d["FETCH_SIZE"]), "isa_sha256": h, "template_args": targs,
               "source": os.path.relpath(root, ROOT),
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                         "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 read correction, the same 1/2 at 4, 8, 12 and 16 B "
                         "per lane: profiles/r05/fetch_cal/ratios.json)"}
        json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_{m.group(1)}_h{H}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
