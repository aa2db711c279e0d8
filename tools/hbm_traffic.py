#!/usr/bin/env python3
"""HBM bytes per PASS (forward / inverse / sigma) from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced
streaming reads, so it is doubled.  A pass is every kernel launch of one forward (or inverse) call:
one fused kernel for short signals, a multi-level tile kernel plus column sweeps for long ones.
Output: JSON {pass: {bytes_per_launch (= per pass), fetch_bytes, write_bytes, dispatches, kernels}}
plus "captured_at" -- read by bench.py for roofline.traffic.

    python tools/hbm_traffic.py gpurun_out/pmc_db4 --passes 5 --commit <sha> > profiles/hbm_traffic_db4.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

MEMBERS = {
    "forward": ("k_forward_fused", "k_forward_persist", "k_forward_blk", "k_forward_level", "k_forward_multi", "k_forward_sweep",
                "k_forward_deep"),
    "inverse": ("k_inverse_fused", "k_inverse_seq", "k_inverse_db", "k_inverse_blk", "k_inverse_level", "k_inverse_multi",
                "k_inverse_sweep", "k_inverse_sweep2", "k_inverse_sweep3", "k_inverse_deep"),
    "sigma": ("k_noise_sigma",),
}


def pass_of(kernel):
    k = kernel.split("(")[0].replace("void ", "").replace("vw::", "").split("<")[0].strip()
    for p, names in MEMBERS.items():
        if k in names:
            return p
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--passes", type=int, default=0,
                    help="passes per family in the run (0: the launch count of the family's least-launched kernel, "
                         "i.e. every kernel of a pass runs at least once per pass)")
    ap.add_argument("--commit", default="")
    ap.add_argument("--rows", type=int, default=0, help="signals per pass (bench.py scales by its rank's rows)")
    a = ap.parse_args()
    # counter -> pass -> list of per-dispatch values (one csv row per dispatch and counter)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    names = collections.defaultdict(set)
    kcount = collections.defaultdict(collections.Counter)   # pass -> kernel -> FETCH_SIZE rows (dispatches)
    for f in sorted(glob.glob(os.path.join(a.root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            p = pass_of(r["Kernel_Name"])
            if p is None:
                continue
            vals[p][r["Counter_Name"]].append(float(r["Counter_Value"]))
            kn = r["Kernel_Name"].split("(")[0].replace("void ", "")
            names[p].add(kn)
            if r["Counter_Name"] == "FETCH_SIZE":
                kcount[p][kn] += 1
    out = {"captured_at": a.commit or None}
    if a.rows:
        out["rows"] = a.rows
    for p, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        n = a.passes or min(kcount[p].values())
        fetch = 2.0 * 1024.0 * sum(cs["FETCH_SIZE"]) / n
        write = 1024.0 * sum(cs["WRITE_SIZE"]) / n
        out[p] = {"bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
                  "dispatches": len(cs["FETCH_SIZE"]), "passes": n, "kernels": sorted(names[p]),
                  "launches_per_pass": {k: round(c / n, 3) for k, c in sorted(kcount[p].items())},
                  "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KiB -> bytes; per pass"}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
