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
  python3 -c "
import json,sys
try:
    d=json.loads([l for l in open('gpurun_out/ab_one.log') if l.startswith('{')][-1])
    k=d['config'].get('kernels') or {}
    print('$name', d['value'], d['ms_per_step'], ' '.join(f'{a}={b[\"ms_per_launch\"]}' for a,b in k.items()))
except Exception as e:
    print('$name', 'FAILED', open('gpurun_out/ab_one.log').read()[-600:])
" | tee -a gpurun_out/ab_env.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc"; exit $rc; fi
done
done
exit 0
