#!/usr/bin/env python3
"""HBM bytes per launch of each kernel family from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced
streaming reads, so it is doubled.  Output: JSON {family: {bytes_per_launch, fetch_bytes, write_bytes,
dispatches, kernels}} for bench.py's roofline.traffic.

    python tools/hbm_traffic.py gpurun_out/pmc > profiles/hbm_traffic_db4.json
"""
import collections
import csv
import glob
import json
import os
import sys


def family(kernel):
    k = kernel.split("(")[0].replace("void ", "").replace("vw::", "").strip()
    if k.startswith("k_forward_fused") or k.startswith("k_forward_persist"):
        return "forward"
    if k.startswith("k_inverse_fused") or k.startswith("k_inverse_seq") or k.startswith("k_inverse_db"):
        return "inverse"
    if k.startswith("k_forward_level"):
        return "forward_level"
    if k.startswith("k_inverse_level"):
        return "inverse_level"
    if k.startswith("k_noise_sigma"):
        return "sigma"
    return None


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    names = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "p*", "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            if fam is None:
                continue
            vals[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
            names[fam].add(r["Kernel_Name"].split("(")[0])
    out = {}
    for fam, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = 2.0 * 1024.0 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        write = 1024.0 * sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        out[fam] = {"bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
                    "dispatches": len(cs["FETCH_SIZE"]), "kernels": sorted(names[fam]),
                    "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KiB -> bytes"}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
