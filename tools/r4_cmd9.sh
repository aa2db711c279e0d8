# cache policy on top of the sc1 forward stores: forward sc1+nt / sc0+sc1, inverse row loads sc1 / default
v() { echo "VW_LIB_PATH=build/var_$1/libvectorwave_amd.so"; }
export AB_q4k_V="$(v h16)|;$(v f18)|;$(v f17)|;$(v l16)|;$(v l0)|" AB_q4k_REPS=3
export AB_q512_V="$(v h16)|--batch 512;$(v f18)|--batch 512;$(v f17)|--batch 512;$(v l16)|--batch 512;$(v l0)|--batch 512" AB_q512_REPS=2
bash tools/gpu_steps.sh ab:q4k ab:q512
