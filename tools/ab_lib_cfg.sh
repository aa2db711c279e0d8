#!/bin/bash
# A/B of variant libraries (tools/build_variant.sh) on one config, same box, alternating:
# CFG=db8-stream VARS='ds1 ds2' REPS=2
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; OUT=gpurun_out/ab_lib_${CFG:-db4}.log; : > $OUT
for rep in $(seq ${REPS:-2}); do
  for v in ${VARS:-base}; do
    VW_LIB_PATH=build/var_$v/libvectorwave_amd.so timeout -k 10 200 python bench.py ${CFG:+--config $CFG} --no-cpu-baseline --no-alt --steps ${STEPS:-10} --warmup 3 > gpurun_out/ab_cur.json 2>&1 || { cat gpurun_out/ab_cur.json; exit 3; }
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1) ok=$(grep -o '"ok": [a-z]*' gpurun_out/ab_cur.json | head -1)" >> $OUT
  done
done
cat $OUT
