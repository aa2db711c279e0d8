#!/bin/bash
# Same-box A/B of the headline bench (driver command shape): this tree vs an older tree's package +
# bench copied to build/old_tree (its own libvectorwave_amd.so), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; : > gpurun_out/ab_builds.log
R=$(pwd)
for v in ${VARS:-head old head old}; do
  if [ $v = old ]; then d=build/old_tree; else d=.; fi
  (cd $d && timeout -k 10 120 python bench.py --no-cpu-baseline --no-alt --steps ${STEPS:-20} --warmup ${WARMUP:-5}) > gpurun_out/ab_cur.json 2>&1; rc=$?
  echo "$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1)" >> gpurun_out/ab_builds.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then break; fi
done
cat gpurun_out/ab_builds.log
