# round-end evidence on one box: the GPU suite, smoke, the driver's bench command, rocprofv3 kernel trace of it,
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the headline passes, the other configs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/final
bash tools/gpu_steps.sh t:all || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { cat gpurun_out/final/smoke.log; exit 3; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench_20.json 2> gpurun_out/final/bench_20.err || exit $?
tail -c 400 gpurun_out/final/bench_20.json; echo
bash tools/gpu_steps.sh "prof:--steps 20 --warmup 5 --no-alt" "pmc:db4:--contexts 1 --settle 0" || exit $?
for c in sym8-denoise db8-stream coif5-f32; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/final/bench_$c.json 2> gpurun_out/final/bench_$c.err || exit $?
  tail -c 300 gpurun_out/final/bench_$c.json; echo
done
