#!/bin/bash
# Run named GPU steps in order, each under its own time limit; stop at the first crash / abort / timeout
# (exit >= 124, 134, 139) and at a failing parity test.  Steps:
#   t:<pytest -k expr or file>   parity tests (file names under tests/ or a -k expression)
#   ab:<name>                    tools/ab.sh with V / STEPS / REPS / CFG / COMMON from AB_<name>_* env
#   bench:<args>                 one bench.py line into gpurun_out/bench_<n>.json
#   prof:<args>                  rocprofv3 --kernel-trace --stats of bench.py into gpurun_out/prof_<n>
#   pmc:<cfg>:<args>             FETCH_SIZE / WRITE_SIZE passes -> gpurun_out/hbm_traffic_<cfg>.json
#                                (one context: pass --contexts 1; VW_COMMIT=<sha> stamps captured_at)
#   grp:<args>                   prof:<args>, then the trace grouped per launch shape -> gpurun_out/prof_<n>_groups.txt
#   smoke:                       __graft_entry__.smoke() -> gpurun_out/smoke.log
#   cfg:<config>                 bench.py --config <config> (10 steps, no CPU leg) -> gpurun_out/bench_<config>.json
#   rehearse:<ranks>             the multi-rank launcher with <ranks> ranks on this one GPU (VW_BENCH_DEVICE_MOD=1)
#                                -> gpurun_out/bench_db4_<ranks>rank_rehearsal.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
n=0
for s in "$@"; do
  n=$((n + 1)); kind="${s%%:*}"; arg="${s#*:}"
  case "$kind" in
    t)
      if [ "$arg" = all ]; then sel=tests; elif [ -f "tests/$arg" ]; then sel="tests/$arg"; else sel="tests -k $arg"; fi
      # shellcheck disable=SC2086
      timeout -k 10 "${T_TESTS:-600}" python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread \
        > "gpurun_out/pytest_$n.log" 2>&1; rc=$?
      tail -3 "gpurun_out/pytest_$n.log"; echo "[$s] rc=$rc"
      [ $rc -ne 0 ] && exit $rc ;;
    ab)
      eval "V=\"\$AB_${arg}_V\" STEPS=\"\${AB_${arg}_STEPS:-20}\" REPS=\"\${AB_${arg}_REPS:-3}\" CFG=\"\${AB_${arg}_CFG:-}\" COMMON=\"\${AB_${arg}_COMMON:-}\""
      V="$V" STEPS="$STEPS" REPS="$REPS" CFG="$CFG" COMMON="$COMMON" OUT="gpurun_out/ab_$arg.log" bash tools/ab.sh > /dev/null; rc=$?
      cat "gpurun_out/ab_$arg.log"; echo "[$s] rc=$rc"
      fatal $rc && exit $rc ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 300 python bench.py $arg > "gpurun_out/bench_$n.json" 2> "gpurun_out/bench_$n.err"; rc=$?
      tail -c 600 "gpurun_out/bench_$n.json"; echo; echo "[$s] rc=$rc"
      [ $rc -ne 0 ] && { tail -5 "gpurun_out/bench_$n.err"; exit $rc; } ;;
    prof|grp)
      # shellcheck disable=SC2086
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$n" -o run -- \
        python3 bench.py --no-cpu-baseline $arg > "gpurun_out/prof_$n.log" 2>&1; rc=$?
      echo "[$s] rc=$rc"; fatal $rc && exit $rc
      if [ "$kind" = grp ] && [ $rc -eq 0 ]; then
        python3 tools/rocprof_groups.py "gpurun_out/prof_$n" --commit "${VW_COMMIT:-}" --cmd "bench.py --no-cpu-baseline $arg" \
          --min-launches 3 > "gpurun_out/prof_${n}_groups.txt"
        grep -E "k_(forward|inverse|noise)" "gpurun_out/prof_${n}_groups.txt" || true
      fi ;;
    pmc)
      cfg="${arg%%:*}"; bargs="${arg#*:}"
      rm -rf gpurun_out/pmc
      PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" BENCH_ARGS="--config $cfg $bargs" bash tools/pmc.sh; rc=$?
      if [ $rc -eq 0 ]; then
        case "$cfg" in db4) rows=4096 ;; sym8-denoise) rows=16384 ;; db8-stream) rows=256 ;; coif5-f32) rows=65536 ;; *) rows=0 ;; esac
        python3 tools/hbm_traffic.py gpurun_out/pmc --commit "${VW_COMMIT:-}" --rows "$rows" > "gpurun_out/hbm_traffic_$cfg.json"
        python3 tools/pmc_summary.py gpurun_out/pmc > "gpurun_out/pmc_traffic_$cfg.txt"
        cat "gpurun_out/hbm_traffic_$cfg.json"
      fi
      echo "[$s] rc=$rc"; fatal $rc && exit $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -2 gpurun_out/smoke.log; echo "[$s] rc=$rc"
      [ $rc -ne 0 ] && exit $rc ;;
    cfg)
      timeout -k 10 300 python bench.py --config "$arg" --no-cpu-baseline --steps 10 --warmup 3 \
        > "gpurun_out/bench_$arg.json" 2> "gpurun_out/bench_$arg.err"; rc=$?
      tail -c 300 "gpurun_out/bench_$arg.json"; echo; echo "[$s] rc=$rc"
      [ $rc -ne 0 ] && { tail -5 "gpurun_out/bench_$arg.err"; exit $rc; } ;;
    rehearse)
      VW_BENCH_DEVICE_MOD=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$arg" \
        --master-addr 127.0.0.1 --master-port $((29500 + arg)) bench.py --gpus "$arg" --steps 20 --warmup 3 \
        --no-cpu-baseline --no-alt > "gpurun_out/bench_db4_${arg}rank_rehearsal.json" \
        2> "gpurun_out/bench_db4_${arg}rank_rehearsal.err"; rc=$?
      tail -c 300 "gpurun_out/bench_db4_${arg}rank_rehearsal.json"; echo; echo "[$s] rc=$rc"
      [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
