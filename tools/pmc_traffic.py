"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports 1/2 of
the bytes of a wide (16 B/lane) coalesced read; WRITE_SIZE is exact for
16-B-per-lane stores.  We report both the raw counters and the corrected figure
(2 x FETCH + WRITE), in bytes per launch, averaged over the timed dispatches.
usage: python tools/pmc_traffic.py gpurun_out/<tag> BATCH [H]
"""
import csv, glob, json, re, sys, collections

root, batch = sys.argv[1], int(sys.argv[2])
H = int(sys.argv[3]) if len(sys.argv) > 3 else 50
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/pmc*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        name = re.sub(r"\(.*$", "", row["Kernel_Name"].replace("void pgp::(anonymous namespace)::", ""))
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, d in vals.items():
    if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
        continue
    fe = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024
    wr = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
    out[k] = {"fetch_bytes_raw": fe, "write_bytes": wr, "hbm_bytes_per_launch": 2 * fe + wr}
    print(f"{k:28s} FETCH {fe/1e6:10.1f} MB  WRITE {wr/1e6:10.1f} MB  corrected {(2*fe+wr)/1e6:10.1f} MB")
for k, v in out.items():
    m = re.match(r"(\w+?)_kernel<(\d+)>", k)
    if m and int(m.group(2)) == H:
        v.update({"batch": batch, "kernel": k,
                  "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                            "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 wide-read correction)"})
        json.dump(v, open(f"profiles/pmc_{m.group(1)}_h{H}.json", "w"), indent=1)
