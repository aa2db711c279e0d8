#!/bin/bash
# A/B of env-var variants on the bench (headline config unless BENCH_ARGS says otherwise).
# AB="NAME1:VAR=1 VAR2=2;NAME2:..."  LIB=path/to/libvectorwave_amd.so (optional)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_env.log
IFS=';' read -ra VARS <<< "$AB"
for rep in ${REPS:-1}; do
for v in "${VARS[@]}"; do
  name=${v%%:*}; envs=${v#*:}
  env ${LIB:+VW_LIB_PATH=$LIB} $envs timeout -k 10 120 python bench.py --no-cpu-baseline --no-alt ${BENCH_ARGS:-} > gpurun_out/ab_one.log 2>&1; rc=$?
  grep "^{" gpurun_out/ab_one.log | tail -1 > gpurun_out/ab_one.json; echo -n "$name " | tee -a gpurun_out/ab_env.log
  python3 tools/bench_summary.py gpurun_out/ab_one.json | tee -a gpurun_out/ab_env.log || tail -c 600 gpurun_out/ab_one.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc"; exit $rc; fi
done
done
exit 0
