#!/bin/bash
# A/B of experiment builds (tools/build_variant.sh) x env settings on the headline bench.
# VARS='base aux0'  ENVS='X=0;VW_INV_REV=1'  BARGS='--no-alt'
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; : > gpurun_out/ab.log
IFS=';' read -ra EV <<< "${ENVS:-X=0}"
for v in ${VARS:-base}; do
  for e in "${EV[@]}"; do
    env $e VW_LIB_PATH=build/var_$v/libvectorwave_amd.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-alt --steps ${STEPS:-300} ${BARGS:-} > gpurun_out/ab_cur.json 2>&1 || { cat gpurun_out/ab_cur.json; exit 3; }
    echo "$v $e $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1)" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
