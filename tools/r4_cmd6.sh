# forward-coefficient store policy across configs and batch sizes (library variants, tools/build_variant.sh)
b=build/var_base/libvectorwave_amd.so; f0=build/var_fst0/libvectorwave_amd.so
f1=build/var_fst1/libvectorwave_amd.so; f16=build/var_fst16/libvectorwave_amd.so
B3=build/var_base3/libvectorwave_amd.so; F3=build/var_fst0x/libvectorwave_amd.so
export AB_s4k_V="VW_LIB_PATH=$b|;VW_LIB_PATH=$f0|;VW_LIB_PATH=$f1|;VW_LIB_PATH=$f16|" AB_s4k_REPS=2
export AB_s512_V="VW_LIB_PATH=$b|--batch 512;VW_LIB_PATH=$f0|--batch 512;VW_LIB_PATH=$f1|--batch 512;VW_LIB_PATH=$f16|--batch 512" AB_s512_REPS=2
for c in sym8 db8 coif5; do
  export AB_${c}_V="VW_LIB_PATH=$B3|;VW_LIB_PATH=$F3|" AB_${c}_REPS=2 AB_${c}_STEPS=10
done
export AB_sym8_CFG=sym8-denoise AB_db8_CFG=db8-stream AB_coif5_CFG=coif5-f32
bash tools/gpu_steps.sh ab:s4k ab:s512 ab:sym8 ab:db8 ab:coif5
