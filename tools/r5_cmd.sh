# round-5: noise sigma with merged block reductions, 4 vs 8 waves per SIMD -- parity (denoise, medians,
# config 3), then same-box A/B on sym8-denoise against the round-4 kernels (ck0)
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
bash tools/gpu_steps.sh t:test_gpu_denoiser.py t:config3 t:median t:sigma || exit $?
export AB_sg_V="VW_LIB_PATH=vwvar/var_ck0/libvectorwave_amd.so|;VW_LIB_PATH=vwvar/var_sw4/libvectorwave_amd.so|;VW_LIB_PATH=vwvar/var_sw8/libvectorwave_amd.so|" AB_sg_STEPS=10 AB_sg_REPS=3 AB_sg_CFG=sym8-denoise
bash tools/gpu_steps.sh ab:sg
