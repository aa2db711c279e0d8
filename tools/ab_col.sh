#!/bin/bash
# A/B of the deep-level column group (VW_COL*) on db8-stream; one bench line per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab_col.log
IFS=';' read -ra VARS <<< "${AB:-VW_COL=0;VW_COL=1;VW_COL=1 VW_COL_C=16 VW_COL_MIN=0;VW_COL=1 VW_COL_MIN=0 VW_COL_TK=170}"
for v in "${VARS[@]}"; do
  env $v timeout -k 10 200 python bench.py --config db8-stream --steps 10 --warmup 3 --settle 0.5 --no-cpu-baseline --no-alt > gpurun_out/ab_col_one.log 2>&1; rc=$?
  echo "$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_col_one.log) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_col_one.log)" >> gpurun_out/ab_col.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then break; fi
done
cat gpurun_out/ab_col.log
