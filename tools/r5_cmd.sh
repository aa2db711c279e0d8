# round-5: deep forward output pairs (VW_DEEP_PAIR) -- parity on the product build, same-box A/B on db8-stream
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
bash tools/gpu_steps.sh t:test_gpu_deep.py t:config4 || exit $?
export AB_pr_V="VW_LIB_PATH=vwvar/var_pair0/libvectorwave_amd.so|;VW_LIB_PATH=vwvar/var_pair1/libvectorwave_amd.so|" AB_pr_STEPS=10 AB_pr_REPS=3 AB_pr_CFG=db8-stream
bash tools/gpu_steps.sh ab:pr
