"""Average PMC counter values per kernel over the dispatches of a rocprofv3 --pmc run."""
import csv, glob, re, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        short = re.sub(r"\(.*$", "", k.replace("void pgp::(anonymous namespace)::", "").replace("void (anonymous namespace)::", ""))
        acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    if not any(s in k for s in ("encdec", "encoder_kernel", "decoder_kernel", "gan_kernel", "gat_agg")):
        continue
    print(k)
    for c, v in sorted(d.items()):
        # several rows per dispatch (one per dimension instance) are already summed by rocprofv3
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
