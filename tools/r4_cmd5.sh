export AB_pol_V="VW_LIB_PATH=build/var_base/libvectorwave_amd.so|;VW_LIB_PATH=build/var_fst0/libvectorwave_amd.so|;VW_LIB_PATH=build/var_st0/libvectorwave_amd.so|;VW_LIB_PATH=build/var_ld0/libvectorwave_amd.so|"
export AB_pol_REPS=2 AB_pol_STEPS=20
export AB_def_V="|;|--batch 512;|--batch 1024;|--batch 2048"
export AB_def_REPS=2 AB_def_STEPS=20
bash tools/gpu_steps.sh t:all ab:def ab:pol
