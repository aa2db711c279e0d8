#!/bin/bash
# Small-batch (strong-scaling shard) A/B of env policies on the headline workload: --batch B rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; : > gpurun_out/ab_small.log
IFS=';' read -ra VARS <<< "${AB:-X=0;VW_FORCE_TILED=1 VW_MULTI_TILE=2048;VW_FORCE_TILED=1 VW_MULTI_TILE=1024;VW_NV=8;VW_INV_BUF=1;VW_FWD_PERSIST=0;VW_FWD_BUF=1}"
for b in ${BATCHES:-512 1024}; do
  for v in "${VARS[@]}"; do
    env $v timeout -k 10 120 python bench.py --batch $b --steps 200 --warmup 20 --no-cpu-baseline --no-alt > gpurun_out/ab_cur.json 2>&1; rc=$?
    echo "B=$b $v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1)" >> gpurun_out/ab_small.log
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then break 2; fi
  done
done
cat gpurun_out/ab_small.log
