#!/bin/bash
# PMC A/B of env variants (LDS / VALU / wait counters), one summary per variant:
# AB="name:VAR=1 VAR2=2;name2:..." -> gpurun_out/pmcab_<name>.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -ra VARS <<< "$AB"
for v in "${VARS[@]}"; do
  name=${v%%:*}; envs=${v#*:}
  rm -rf gpurun_out/pmcab_$name
  env $envs PMC_DIR=gpurun_out/pmcab_$name PMC_GROUPS="${PMC_GROUPS:-SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY
GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES}" \
    bash tools/pmc.sh; rc=$?
  python3 tools/pmc_summary.py gpurun_out/pmcab_$name > gpurun_out/pmcab_$name.txt
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
