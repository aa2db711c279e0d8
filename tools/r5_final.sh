# round-5 evidence on one box: GPU suite, smoke, the driver's bench command, its rocprofv3 trace grouped per
# launch shape, PMC HBM traffic of db8-stream and sym8-denoise (kernels changed this round), the other configs, and the
# multi-rank launcher rehearsed with 2 and 8 ranks on this one GPU (VW_BENCH_DEVICE_MOD=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/final5
bash tools/gpu_steps.sh t:all || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final5/smoke.log 2>&1 || { cat gpurun_out/final5/smoke.log; exit 3; }
tail -1 gpurun_out/final5/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final5/bench_db4.json 2> gpurun_out/final5/bench_db4.err || exit $?
tail -c 300 gpurun_out/final5/bench_db4.json; echo
bash tools/gpu_steps.sh "grp:--steps 20 --warmup 5 --no-alt" "pmc:db8-stream:--contexts 1 --settle 0" \
  "pmc:sym8-denoise:--contexts 1 --settle 0" || exit $?
for c in sym8-denoise db8-stream coif5-f32; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/final5/bench_$c.json 2> gpurun_out/final5/bench_$c.err || exit $?
  tail -c 200 gpurun_out/final5/bench_$c.json; echo
done
for n in 2 8; do
  VW_BENCH_DEVICE_MOD=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 3 --no-cpu-baseline --no-alt \
    > gpurun_out/final5/bench_db4_${n}rank_rehearsal.json 2> gpurun_out/final5/bench_db4_${n}rank_rehearsal.err || exit $?
  tail -c 300 gpurun_out/final5/bench_db4_${n}rank_rehearsal.json; echo
done
