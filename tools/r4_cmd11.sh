# long-filter blocked kernels with their taps from the kernel arguments (SGPR operands, no LDS tap reads):
# kt = VW_FWD_KTAPS=1 VW_INV_KTAPS=1; kt6 = kt + VW_LONG_WAVES=6.  Parity first, then coif5 / sym8 A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
VW_LIB_PATH=build/var_kt/libvectorwave_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_denoiser.py \
  -m gpu -k "coif5 or COIF5 or config5 or sym8 or SYM8 or config3 or Symlet or Coiflet" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_kt.log 2>&1 || { tail -30 gpurun_out/pytest_kt.log; exit 1; }
tail -2 gpurun_out/pytest_kt.log
VW_LIB_PATH=build/var_kt6/libvectorwave_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -m gpu -k "coif5 or COIF5 or config5" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_kt6.log 2>&1 || { tail -30 gpurun_out/pytest_kt6.log; exit 1; }
tail -2 gpurun_out/pytest_kt6.log
export AB_k5_V="|;VW_LIB_PATH=build/var_kt/libvectorwave_amd.so|;VW_LIB_PATH=build/var_kt6/libvectorwave_amd.so|" AB_k5_REPS=2 AB_k5_STEPS=10 AB_k5_CFG=coif5-f32
export AB_k8_V="|;VW_LIB_PATH=build/var_kt/libvectorwave_amd.so|" AB_k8_REPS=2 AB_k8_STEPS=10 AB_k8_CFG=sym8-denoise
bash tools/gpu_steps.sh ab:k5 ab:k8
