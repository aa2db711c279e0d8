#!/bin/bash
# A/B of bench arguments on one config, same box, alternating: CFG=db8-stream ARGS='--contexts 1;--contexts 2' REPS=2
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; OUT=gpurun_out/ab_args_${CFG:-db4}.log; : > $OUT
IFS=';' read -ra AV <<< "${ARGS:---contexts 1}"
for rep in $(seq ${REPS:-2}); do
  for a in "${AV[@]}"; do
    timeout -k 10 200 python bench.py ${CFG:+--config $CFG} --no-cpu-baseline --no-alt --steps ${STEPS:-10} --warmup 3 $a > gpurun_out/ab_cur.json 2>&1 || { cat gpurun_out/ab_cur.json; exit 3; }
    echo "$a $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) ctx=$(grep -o '"contexts_per_gpu": [0-9]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1) ok=$(grep -o '"ok": [a-z]*' gpurun_out/ab_cur.json | head -1)" >> $OUT
  done
done
cat $OUT
