#!/bin/bash
# Round-3 A/B: level-pair inverse sweeps (VW_SWEEP2) on db8-stream, wave-uniform blocked-inverse offsets
# (VW_BLK_SOFF builds s0 / s1) on sym8-denoise.  Same box, alternating runs.
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; : > gpurun_out/ab_r3b.log
one() {  # name lib env config
  env $3 VW_LIB_PATH=build/var_$2/libvectorwave_amd.so timeout -k 10 200 python bench.py --config $4 --no-cpu-baseline --no-alt --steps 10 --warmup 3 > gpurun_out/ab_cur.json 2>&1 || { cat gpurun_out/ab_cur.json; exit 3; }
  echo "$1 $4 $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1) $(grep -o '"check": \[[^]]*\]' gpurun_out/ab_cur.json | grep -o '"ok": [a-z]*')" >> gpurun_out/ab_r3b.log
}
for rep in 1 2; do
  one pair p2 VW_SWEEP2=1 db8-stream
  one single p2 VW_SWEEP2=0 db8-stream
  one pair16 p2 "VW_SWEEP2=1 VW_SWEEP2_KA=16" db8-stream
  one pairuc1k p2 "VW_SWEEP2=1 VW_SWEEP2_UC=1024" db8-stream
done
for rep in 1 2; do
  one soff1 s1 X=1 sym8-denoise
  one soff0 s0 X=1 sym8-denoise
done
cat gpurun_out/ab_r3b.log
