#!/bin/bash
# Kernel resource summary (name, VGPRs, scratch bytes/lane) of the fused/tiled kernel units.
# usage: tools/usage.sh [DEV_TAPS]   e.g. tools/usage.sh 'X(8)'
cd "$(dirname "$0")/../vectorwave_amd/csrc" || exit 1
for ut in vw_fwd:double vw_inv:double vw_fwd:float vw_inv:float vw_lvl:double vw_lvl:float; do
  make -s usage U=${ut%%:*} T=${ut##*:} DEV_TAPS="${1:-X(8)}" 2>&1 |
    grep -o "Function Name: [^ ]*\|VGPRs: [0-9]*\|ScratchSize \[bytes/lane\]: [0-9]*" | paste - - - |
    sed 's/Function Name: _ZN2vw[0-9]*//; s/EEEvNS_.*IT_EE//' | awk '{printf "%-34s vgpr %4s scratch %4s\n", $1, $3, $6}'
done
