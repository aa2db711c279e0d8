"""Summarise rocprofv3 --pmc csv passes per kernel (mean over dispatches)."""
import csv, glob, os, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = k.split("(")[0].replace("void vw::", "")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        # one row per (dispatch, counter) -> counters summed over dimensions already
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):16.4g}  (n={len(v)})")
