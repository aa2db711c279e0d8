#!/bin/bash
# PMC comparison of build/env variants: VARIANTS="name=ENV1=a,ENV2=b;name2=" (comma-separated env
# assignments per variant).  Writes gpurun_out/pmc_<name>.txt per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
IFS=';' read -ra VARS <<< "${VARIANTS:-base=}"
for spec in "${VARS[@]}"; do
  name="${spec%%=*}"
  envs="${spec#*=}"
  (
    IFS=',' read -ra KV <<< "$envs"
    for kv in "${KV[@]}"; do [ -n "$kv" ] && export "$kv"; done
    PMC_GROUPS="${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE}" bash tools/pmc.sh
  ) || exit $?
  python3 tools/pmc_summary.py > gpurun_out/pmc_$name.txt
  rm -rf gpurun_out/pmc
done
