# round-5: compile-time tap offsets in the deep forward (VW_DEEP_CK) and the inverse multi-level tiles (VW_MULTI_CK)
# -- parity on the product build, then same-box A/B: ck0 (both runtime), mck0 (deep only), ck1 (both)
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
bash tools/gpu_steps.sh t:test_gpu_deep.py t:config4 t:multilevel || exit $?
export AB_ck_V="VW_LIB_PATH=vwvar/var_ck0/libvectorwave_amd.so|;VW_LIB_PATH=vwvar/var_mck0/libvectorwave_amd.so|;VW_LIB_PATH=vwvar/var_ck1/libvectorwave_amd.so|" AB_ck_STEPS=10 AB_ck_REPS=3 AB_ck_CFG=db8-stream
bash tools/gpu_steps.sh ab:ck
