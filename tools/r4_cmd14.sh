# final check after the blocked NV = 8 forward became the default: GPU suite, smoke, sym8 and the headline
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out/final3
bash tools/gpu_steps.sh t:all || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3/smoke.log 2>&1 || { cat gpurun_out/final3/smoke.log; exit 3; }
tail -1 gpurun_out/final3/smoke.log
for c in sym8-denoise db4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/final3/bench_$c.json 2> gpurun_out/final3/bench_$c.err || exit $?
  tail -c 200 gpurun_out/final3/bench_$c.json; echo
done
