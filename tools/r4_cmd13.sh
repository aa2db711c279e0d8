# sym8: the blocked NV = 8 forward (VW_BLK_FWD8=1) with kernel-argument taps (fk8 library: no spills) vs the fused forward
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
VW_BLK_FWD8=1 VW_LIB_PATH=build/var_fk8/libvectorwave_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_denoiser.py \
  -m gpu -k "sym8 or SYM8 or config3 or Symlet" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fk8.log 2>&1 || { tail -30 gpurun_out/pytest_fk8.log; exit 1; }
tail -2 gpurun_out/pytest_fk8.log
export AB_f8_V="|;VW_BLK_FWD8=1|;VW_BLK_FWD8=1 VW_LIB_PATH=build/var_fk8/libvectorwave_amd.so|" AB_f8_REPS=2 AB_f8_STEPS=10 AB_f8_CFG=sym8-denoise
bash tools/gpu_steps.sh ab:f8
