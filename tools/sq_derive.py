#!/usr/bin/env python3
"""Derived SQ metrics per kernel from a tools/pmc_ab.sh capture (pmc_summary-style means per dispatch).

cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs); per-CU rates divide by 256 CUs.
  valu_ipc   VALU wave-instructions per CU-cycle (4 SIMDs: <= 4)
  lds_ipc    LDS wave-instructions per CU-cycle
  lds_busy   SQ_LDS_IDX_ACTIVE per CU-cycle (LDS pipe occupancy, relative)
  conflict   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait       SQ_WAIT_ANY / SQ_WAVE_CYCLES (fraction of wave time waiting on a dependency / barrier)
  waves/CU   SQ_WAVE_CYCLES / (256 * cycles): average resident waves per CU
    python3 tools/sq_derive.py gpurun_out/pmcab_db8
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void vw::", "").replace("void ", "")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(f"{'kernel':48s} {'ms':>7s} {'valu_ipc':>8s} {'lds_ipc':>7s} {'lds_busy':>8s} {'conflict':>8s} {'wait':>6s} "
      f"{'waves/CU':>8s}")
for k, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    if not k.startswith("k_") or "GRBM_GUI_ACTIVE" not in m:
        continue
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    cu = 256 * cyc
    print(f"{k[:48]:48s} {cyc / 2.4e6:7.3f} {m.get('SQ_INSTS_VALU', 0) / cu:8.3f} {m.get('SQ_INSTS_LDS', 0) / cu:7.3f} "
          f"{m.get('SQ_LDS_IDX_ACTIVE', 0) / cu:8.3f} {m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, m.get('SQ_LDS_IDX_ACTIVE', 1)):8.3f} "
          f"{m.get('SQ_WAIT_ANY', 0) / max(1, m.get('SQ_WAVE_CYCLES', 1)):6.3f} {m.get('SQ_WAVE_CYCLES', 0) / cu:8.2f}")
