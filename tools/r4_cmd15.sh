# bench step schedule for the long-signal configs: policy default vs explicit contexts
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export AB_s8_V="|;|--contexts 1;|--overlap-steps" AB_s8_REPS=2 AB_s8_STEPS=10 AB_s8_CFG=db8-stream
bash tools/gpu_steps.sh ab:s8
