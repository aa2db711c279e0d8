export AB_db8_V="|;VW_FWD_STREAM=1|;VW_FWD_STREAM=1 VW_INV_STREAM=512|;VW_FWD_STREAM=1 VW_INV_STREAM=1024|;VW_MULTI_XCD=64|"
export AB_db8_CFG=db8-stream AB_db8_STEPS=10 AB_db8_REPS=2
export AB_fpf_V="|;VW_FWD_PF=1|;|--batch 512;VW_FWD_PF=1|--batch 512"
export AB_fpf_REPS=2 AB_fpf_STEPS=50
export AB_ovl_V="|--batch 512;|--batch 512 --overlap-steps;|--batch 1024;|--batch 1024 --overlap-steps;|;|--overlap-steps"
export AB_ovl_STEPS=100 AB_ovl_REPS=2
bash tools/gpu_steps.sh t:test_gpu_stream.py t:test_gpu_persist_inv.py ab:db8 ab:fpf ab:ovl
