#!/bin/bash
# A/B of the multi-level tile groups (VW_MULTI=1 default vs 0 = one launch per level) on the
# long-signal BASELINE config, one bench line each; stops at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab_multi.log
for v in ${AB_MULTI:-1 0}; do
  VW_MULTI=$v timeout -k 10 240 python bench.py --config ${CFG:-db8-stream} --no-cpu-baseline --no-alt \
    --steps ${CFG_STEPS:-10} --warmup 3 > gpurun_out/ab_multi_cur.json 2>&1
  rc=$?
  echo "VW_MULTI=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_multi_cur.json | head -1) \
$(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ab_multi_cur.json | head -1)" >> gpurun_out/ab_multi.log
  [ $rc -ne 0 ] && { cat gpurun_out/ab_multi_cur.json; break; }
done
cat gpurun_out/ab_multi.log
