# round-end check of the product library at HEAD: full GPU suite, smoke, the driver's bench command, the other configs
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out/final2
bash tools/gpu_steps.sh t:all || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 || { cat gpurun_out/final2/smoke.log; exit 3; }
tail -1 gpurun_out/final2/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final2/bench_20.json 2> gpurun_out/final2/bench_20.err || exit $?
tail -c 300 gpurun_out/final2/bench_20.json; echo
timeout -k 10 300 python bench.py --batch 512 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/final2/bench_512.json 2> gpurun_out/final2/bench_512.err || exit $?
for c in sym8-denoise coif5-f32 db8-stream; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/final2/bench_$c.json 2> gpurun_out/final2/bench_$c.err || exit $?
  tail -c 200 gpurun_out/final2/bench_$c.json; echo
done
