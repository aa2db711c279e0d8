#!/bin/bash
# A/B of runtime switches on one config, same box, alternating: CFG=sym8-denoise ENVS='VW_X=1;VW_X=0' REPS=2
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; OUT=gpurun_out/ab_env_${CFG:-db4}.log; : > $OUT
IFS=';' read -ra EV <<< "${ENVS:-X=0}"
for rep in $(seq ${REPS:-2}); do
  for e in "${EV[@]}"; do
    env $e timeout -k 10 200 python bench.py ${CFG:+--config $CFG} --no-cpu-baseline --no-alt --steps ${STEPS:-10} --warmup 3 > gpurun_out/ab_cur.json 2>&1 || { cat gpurun_out/ab_cur.json; exit 3; }
    echo "$e $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1) ok=$(grep -o '"ok": [a-z]*' gpurun_out/ab_cur.json | head -1)" >> $OUT
  done
done
cat $OUT
