export AB_o2_V="|--batch 512;|--batch 512 --overlap-steps --launch direct;|--batch 512 --contexts 2;VW_DMA_NT=1|--batch 512;VW_DMA_NT=1|--batch 512 --overlap-steps --launch direct"
export AB_o2_STEPS=200 AB_o2_REPS=3
export AB_o4_V="|;|--overlap-steps --launch direct;|--rotate 4;|--rotate 1"
export AB_o4_STEPS=20 AB_o4_REPS=3
bash tools/gpu_steps.sh ab:o2 ab:o4
