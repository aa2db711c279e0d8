#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 invocation; no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PMC_DIR="${PMC_DIR:-gpurun_out/pmc}"
mkdir -p "$PMC_DIR"
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:-} --no-cpu-baseline --no-alt --steps 3 --warmup 1"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$PMC_DIR/p$i" -o pmc -- python3 bench.py $ARGS > "$PMC_DIR/p$i.log" 2>&1; rc=$?
  echo "group $i ($grp) rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done <<< "${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM}"
exit 0
