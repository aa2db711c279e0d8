# round-end evidence with sc1 forward stores (tools/r4_final.sh), then per-level pass times of the long filters
bash tools/r4_final.sh || exit $?
for a in "coif5 8192 65536 f32 6" "sym8 16384 16384 f64 8" "db4 4096 4096 f64 6 50"; do
  # shellcheck disable=SC2086
  timeout -k 10 240 python tools/level_probe.py $a >> gpurun_out/final/level_probe.log 2>&1 || exit $?
done
cat gpurun_out/final/level_probe.log
