#!/bin/bash
# Sweep of the multi-level tile (VW_MULTI_TILE) and reach bound (VW_MULTI_DIV) on the long-signal
# BASELINE config, one bench line each; stops at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sweep_multi.log
for t in ${TILES:-1024 2048 4096}; do
  for d in ${DIVS:-2 4 8}; do
    VW_MULTI_TILE=$t VW_MULTI_DIV=$d timeout -k 10 120 python bench.py --config ${CFG:-db8-stream} \
      --no-cpu-baseline --no-alt --steps ${CFG_STEPS:-10} --warmup 3 > gpurun_out/sweep_cur.json 2>&1
    rc=$?
    echo "tile=$t div=$d rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sweep_cur.json | head -1) \
$(grep -o '"kernels_ms": {[^}]*}' gpurun_out/sweep_cur.json | head -1)" >> gpurun_out/sweep_multi.log
    [ $rc -ne 0 ] && { cat gpurun_out/sweep_cur.json; exit $rc; }
  done
done
cat gpurun_out/sweep_multi.log
