#!/bin/bash
# Round-3 A/B: chained inverse column sweeps on db8-stream -- triples + pairs (VW_SWEEP2=3), pairs only (2),
# one sweep per level (0); chunk length (VW_SWEEP2_UC) and residue-group width (VW_SWEEP2_R).  Same box,
# alternating; LIB = variant build.
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; OUT=gpurun_out/ab_r3c.log; : > $OUT
IFS=';' read -ra EV <<< "${ENVS:-VW_SWEEP2=3;VW_SWEEP2=2;VW_SWEEP2=0}"
for rep in 1 2; do
  for e in "${EV[@]}"; do
    env $e VW_LIB_PATH=${LIB:-build/var_p3/libvectorwave_amd.so} timeout -k 10 200 python bench.py --config ${CFG:-db8-stream} --no-cpu-baseline --no-alt --steps 10 --warmup 3 > gpurun_out/ab_cur.json 2>&1 || { cat gpurun_out/ab_cur.json; exit 3; }
    echo "$e $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1) ok=$(grep -o '"ok": [a-z]*' gpurun_out/ab_cur.json | head -1)" >> $OUT
  done
done
cat $OUT
