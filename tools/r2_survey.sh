#!/bin/bash
# One GPU session of measurements (each step time-limited; a crash/timeout stops the script).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "fatal at $name"; exit $rc; fi
}
summ() { python3 - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
        r = d.get("roofline") or {}
        print(f.split("/")[-1], d["value"], d["ms_per_step"], json.dumps(d["config"].get("kernels")), r.get("frac"))
    except Exception as e:
        print(f, "parse error", e)
PY
}
for s in ${STEPS:-b512 configs pmc prof}; do
  case $s in
    b512)
      step b512_ev 120 python bench.py --batch 512 --steps 200 --warmup 20 --no-cpu-baseline --no-alt
      step b512_noev 120 python bench.py --batch 512 --steps 200 --warmup 20 --no-cpu-baseline --no-alt --events none
      step b1024_noev 120 python bench.py --batch 1024 --steps 200 --warmup 20 --no-cpu-baseline --no-alt --events none
      summ gpurun_out/b512_ev.log gpurun_out/b512_noev.log gpurun_out/b1024_noev.log ;;
    configs)
      for c in ${CONFIGS:-sym8-denoise db8-stream coif5-f32}; do
        step cfg_$c 240 python bench.py --config $c --steps ${CFG_STEPS:-10} --warmup 3 --settle 0.5 --no-cpu-baseline --no-alt
      done
      summ gpurun_out/cfg_*.log ;;
    pmc)
      CFG=${CFG:-db4}
      mkdir -p gpurun_out/pmc_$CFG
      i=0
      while read -r grp; do
        [ -z "$grp" ] && continue; i=$((i+1))
        step pmc_${CFG}_$i 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$CFG/p$i -o pmc -- python3 bench.py --config $CFG --launch direct --events none --settle 0 --no-cpu-baseline --no-alt --steps 3 --warmup 1 ${PMC_BATCH:+--batch $PMC_BATCH}
      done <<< "${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM}"
      python3 tools/pmc_summary.py gpurun_out/pmc_$CFG > gpurun_out/pmc_summary_$CFG.txt 2>&1
      python3 tools/hbm_traffic.py gpurun_out/pmc_$CFG --passes 5 --commit "${COMMIT:-}" > gpurun_out/hbm_traffic_$CFG.json 2>&1; cat gpurun_out/hbm_traffic_$CFG.json ;;
    prof)
      CFG=${CFG:-db4}
      step prof_$CFG 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o run -- python3 bench.py --config $CFG --no-cpu-baseline --no-alt --steps ${PROF_STEPS:-50} --warmup 5 --settle 0.5
      summ gpurun_out/prof_$CFG.log
      find gpurun_out/prof_$CFG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_$CFG.csv
      cut -d, -f1-8 gpurun_out/kernel_stats_$CFG.csv | head -12 ;;
  esac
done
exit 0
