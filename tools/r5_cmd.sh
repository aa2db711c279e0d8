# round-5: contexts per GPU for the long-signal configs (schedule policy check)
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export AB_c8_V="|;|--contexts 2;|--contexts 4" AB_c8_STEPS=10 AB_c8_REPS=2 AB_c8_CFG=db8-stream
export AB_cs_V="|;|--contexts 1;|--contexts 4" AB_cs_STEPS=10 AB_cs_REPS=2 AB_cs_CFG=sym8-denoise
export AB_cc_V="|;|--contexts 4" AB_cc_STEPS=10 AB_cc_REPS=2 AB_cc_CFG=coif5-f32
bash tools/gpu_steps.sh ab:c8 ab:cs ab:cc
