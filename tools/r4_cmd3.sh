export AB_xcd_V="|;VW_MULTI_XCD=64|;VW_MULTI_XCD=16|"
export AB_xcd_CFG=db8-stream AB_xcd_STEPS=10 AB_xcd_REPS=2
bash tools/gpu_steps.sh ab:xcd t:all "pmc:db4:--contexts 1 --settle 0" "prof:--steps 20 --warmup 5"
