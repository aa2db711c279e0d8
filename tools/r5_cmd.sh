set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out/r5b
bash tools/gpu_steps.sh t:test_gpu_pipeline.py t:test_gpu_graph.py t:test_gpu_multidevice.py || exit $?
export AB_p512_V="|--batch 512;|--batch 512 --contexts 1" AB_p512_STEPS=200 AB_p512_REPS=3
export AB_p4k_V="|" AB_p4k_STEPS=20 AB_p4k_REPS=2
bash tools/gpu_steps.sh ab:p512 ab:p4k "bench:--batch 512 --steps 200 --no-cpu-baseline --no-alt"
