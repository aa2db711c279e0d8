cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out; : > gpurun_out/abc.log
for v in b16 a16 b16 a16; do
  VW_LIB_PATH=build/var_$v/libvectorwave_amd.so timeout -k 10 200 python bench.py --config sym8-denoise --no-cpu-baseline --no-alt --steps 10 --warmup 3 > gpurun_out/abc_cur.json 2>&1 || { cat gpurun_out/abc_cur.json; exit 3; }
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/abc_cur.json | head -1) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/abc_cur.json | head -1)" >> gpurun_out/abc.log
done
cat gpurun_out/abc.log
