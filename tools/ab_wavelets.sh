#!/bin/bash
# Headline workload with other filter lengths (sensitivity of each kernel to tap count).
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; : > gpurun_out/abw.log
for w in ${WAVELETS:-haar db2 db4 db6 db8}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-alt --steps 200 --events separate --wavelet $w ${BARGS:-} > gpurun_out/abw_cur.json 2>&1 || { cat gpurun_out/abw_cur.json; exit 3; }
  echo "$w $(grep -o '"value": [0-9.]*' gpurun_out/abw_cur.json | head -1) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/abw_cur.json | head -1)" >> gpurun_out/abw.log
done
cat gpurun_out/abw.log
