#!/bin/bash
# Round-end evidence on one box, in the driver's order: the GPU suite, smoke, the driver's bench command
# (default flags), its rocprofv3 kernel trace grouped per launch shape, PMC HBM traffic (FETCH_SIZE /
# WRITE_SIZE passes) of the headline, the other BASELINE configs, and the multi-rank launcher rehearsed with
# 2 and 8 ranks on this one GPU.  Each step has its own time limit (tools/gpu_steps.sh); the first failure ends
# the run.  EVIDENCE_STEPS overrides the step list, e.g. EVIDENCE_STEPS="smoke: cfg:db4".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || exit $?
tail -c 400 gpurun_out/bench_driver.json; echo
# shellcheck disable=SC2086
bash tools/gpu_steps.sh ${EVIDENCE_STEPS:-t:all smoke: "grp:--steps 20 --warmup 5 --no-alt" \
  "pmc:db4:--contexts 1 --settle 0" cfg:sym8-denoise cfg:db8-stream cfg:coif5-f32 rehearse:2 rehearse:8}
