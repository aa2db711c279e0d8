export AB_inv_V="|;VW_INV_PERSIST=1|;VW_INV_PERSIST=1 VW_INV_NV=2|;VW_INV_NV=2|"
export AB_inv512_V="|--batch 512;VW_INV_PERSIST=1|--batch 512;VW_INV_PERSIST=1 VW_INV_NV=2|--batch 512"
export AB_inv512_STEPS=200
export AB_rot_V="|;|--rotate 3;|--rotate 3 --rotate-outputs"
bash tools/gpu_steps.sh t:test_gpu_persist_inv.py t:test_gpu_multidevice.py t:test_gpu_graph.py ab:inv ab:inv512 ab:rot
