#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; a crash/abort/timeout (exit >= 124 or 134/139) stops the script, a plain test failure
# (exit 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 ${T_TESTS:-420} python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      tail -5 gpurun_out/pytest_gpu.log; echo "tests rc=$rc" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -3 gpurun_out/smoke.log; echo "smoke rc=$rc" ;;
    bench)
      timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
      tail -3 gpurun_out/bench.log; echo "bench rc=$rc" ;;
    ab)  # quick env variants (no CPU baseline, headline mode only; FMA=--exact selects exact accumulation)
      : > gpurun_out/ab.log
      IFS=';' read -ra VARS <<< "${AB:-X=1;FMA=--exact}"
      for v in "${VARS[@]}"; do
        env $v bash -c 'timeout -k 10 120 python bench.py --no-cpu-baseline --no-alt --steps 300 $FMA' >> gpurun_out/ab.log 2>&1; rc=$?
        echo "$v rc=$rc" >> gpurun_out/ab.log
        fatal $rc && break
      done
      grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}\|VW_NV.*' gpurun_out/ab.log ;;
    configs)  # the other BASELINE configs, one bench line each (no CPU baseline)
      : > gpurun_out/configs.log
      for c in ${CONFIGS:-sym8-denoise db8-stream coif5-f32}; do
        timeout -k 10 240 python bench.py --config $c --no-cpu-baseline --steps ${CFG_STEPS:-10} --warmup 3 >> gpurun_out/configs.log 2>&1; rc=$?
        echo "$c rc=$rc" >> gpurun_out/configs.log
        fatal $rc && break
      done
      grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}\|^[a-z0-9-]* rc=.*' gpurun_out/configs.log ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1; rc=$?
      tail -3 gpurun_out/prof.log; echo "prof rc=$rc" ;;
    traffic)  # HBM bytes per launch (PMC FETCH_SIZE / WRITE_SIZE, separate passes) -> gpurun_out/hbm_traffic_<cfg>.json
      rm -rf gpurun_out/pmc
      PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" BENCH_ARGS="${BENCH_ARGS:-}" bash tools/pmc.sh; rc=$?
      if [ $rc -eq 0 ]; then
        python3 tools/hbm_traffic.py gpurun_out/pmc > gpurun_out/hbm_traffic_${CFG:-db4}.json
        python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_traffic_${CFG:-db4}.txt
        cat gpurun_out/hbm_traffic_${CFG:-db4}.json
      fi
      echo "traffic rc=$rc" ;;
    *) echo "unknown step $s"; rc=0 ;;
  esac
  if fatal $rc; then echo "fatal rc=$rc at step $s, stopping"; exit $rc; fi
done
exit 0
