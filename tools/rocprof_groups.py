#!/usr/bin/env python3
"""Per-launch-shape summary of a rocprofv3 --kernel-trace CSV.

rocprofv3's own --stats file averages every launch of a kernel name, so a run that launches the same
kernel over 2048-row (two-context) and 4096-row (one-context) batches reports a mean that belongs to no
launch.  This groups launches by (kernel, grid, workgroup, stream) instead, and prints count / avg / min /
median / max duration in ms per group -- the form profiles/ summaries are committed in.

    python3 tools/rocprof_groups.py gpurun_out/prof_1 [--commit SHA] [--cmd "bench.py ..."] > profiles/rNN/x.txt
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(name):
    n = name.split("(")[0].replace("void ", "").strip()
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--commit", default="")
    ap.add_argument("--cmd", default="")
    ap.add_argument("--min-launches", type=int, default=1)
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True))
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {a.root}")
    groups = collections.defaultdict(list)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
                       int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]),
                       r.get("Stream_Id", "?"))
                groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    print(f"# rocprofv3 --kernel-trace grouped per launch shape (kernel, grid threads, workgroup, stream)"
          + (f" at {a.commit}" if a.commit else "") + (f"; command: {a.cmd}" if a.cmd else ""))
    print("# kernel | grid | block | stream | launches | avg_ms | min_ms | median_ms | max_ms")
    for key in sorted(groups, key=lambda k: (k[0], k[1], k[3])):
        d = groups[key]
        if len(d) < a.min_launches:
            continue
        print(f"{key[0]} | {key[1]} | {key[2]} | {key[3]} | {len(d)} | {sum(d) / len(d):.5f} | {min(d):.5f} | "
              f"{statistics.median(d):.5f} | {max(d):.5f}")


if __name__ == "__main__":
    main()
