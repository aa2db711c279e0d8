# coif5: compile-time-stride forward reads (fc) and 3 workgroups per CU (fcw6, VW_LONG_WAVES=6): parity, then A/B;
# then a 2-rank rehearsal of the overlapped-steps path (2 ranks on this one GPU, 512 rows each)
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for v in fc fcw6; do
  VW_LIB_PATH=build/var_$v/libvectorwave_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py \
    -m gpu -k "coif5 or COIF5 or config5" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { tail -30 gpurun_out/pytest_$v.log; exit 1; }
  tail -2 gpurun_out/pytest_$v.log
done
export AB_c5_V="|;VW_LIB_PATH=build/var_fc/libvectorwave_amd.so|;VW_LIB_PATH=build/var_fcw6/libvectorwave_amd.so|" AB_c5_REPS=2 AB_c5_STEPS=10 AB_c5_CFG=coif5-f32
bash tools/gpu_steps.sh ab:c5 || exit $?
VW_BENCH_DEVICE_MOD=1 timeout -k 10 300 python bench.py --gpus 2 --batch 1024 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rehearsal_2rank_overlap.json 2> gpurun_out/rehearsal_2rank_overlap.err || { tail -20 gpurun_out/rehearsal_2rank_overlap.err; exit 1; }
tail -c 700 gpurun_out/rehearsal_2rank_overlap.json
