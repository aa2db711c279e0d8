export AB_r4k_V="|;VW_DMA_NT=1|;VW_INV_PERSIST=1|;VW_INV_PERSIST=1 VW_DMA_NT=1|;|--rotate 1"
export AB_r512_V="|--batch 512;VW_DMA_NT=1|--batch 512;VW_INV_PERSIST=1|--batch 512;VW_INV_PERSIST=1 VW_DMA_NT=1|--batch 512;|--batch 512 --rotate 1"
export AB_r512_STEPS=200
export AB_ovl_V="|--batch 512;|--batch 512 --overlap-steps --rotate 32 --rotate-outputs"
export AB_ovl_STEPS=200 AB_ovl_REPS=2
bash tools/gpu_steps.sh ab:r4k ab:r512 ab:ovl t:test_gpu_configs.py
