# store policy, second box: forward sc1 with inverse nt / sc1 / write-back, several batch sizes
b=build/var_base/libvectorwave_amd.so; f0=build/var_fst0/libvectorwave_amd.so; f16=build/var_fst16/libvectorwave_amd.so
a=build/var_f16i16/libvectorwave_amd.so; c=build/var_f16i0/libvectorwave_amd.so
export AB_p4k_V="VW_LIB_PATH=$b|;VW_LIB_PATH=$f0|;VW_LIB_PATH=$f16|;VW_LIB_PATH=$a|;VW_LIB_PATH=$c|" AB_p4k_REPS=3
export AB_p512_V="VW_LIB_PATH=$b|--batch 512;VW_LIB_PATH=$f0|--batch 512;VW_LIB_PATH=$f16|--batch 512;VW_LIB_PATH=$a|--batch 512" AB_p512_REPS=3
export AB_pmid_V="VW_LIB_PATH=$b|--batch 1024;VW_LIB_PATH=$f16|--batch 1024;VW_LIB_PATH=$b|--batch 2048;VW_LIB_PATH=$f16|--batch 2048" AB_pmid_REPS=2
bash tools/gpu_steps.sh ab:p4k ab:p512 ab:pmid
