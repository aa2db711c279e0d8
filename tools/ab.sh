#!/bin/bash
# Same-box A/B driver for bench.py variants, alternating REPS times (one fresh process per run).
# Library variants: VW_LIB_PATH=build/var_NAME/libvectorwave_amd.so in the env part (tools/build_variant.sh).
#   V='ENV=1 ENV2=x|--args;|--other args' CFG=db4 STEPS=20 REPS=3 OUT=gpurun_out/ab_x.log bash tools/ab.sh
# A variant is "<env assignments>|<bench arguments>" (either side may be empty).  Each run prints one
# log line: the variant, value, per-pass ms, check ok.  A crash / timeout stops the script (no retry).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
OUT="${OUT:-gpurun_out/ab_${CFG:-db4}.log}"
: > "$OUT"
IFS=';' read -ra VS <<< "${V:-|}"
for rep in $(seq "${REPS:-2}"); do
  for v in "${VS[@]}"; do
    envs="${v%%|*}"; args="${v#*|}"
    # shellcheck disable=SC2086
    env $envs timeout -k 10 "${TMO:-200}" python bench.py ${CFG:+--config $CFG} --no-cpu-baseline --no-alt \
      --steps "${STEPS:-20}" --warmup "${WARMUP:-3}" $COMMON $args > gpurun_out/ab_cur.json 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then cat gpurun_out/ab_cur.json; echo "[$v] rc=$rc" >> "$OUT"; exit $rc; fi
    echo "[$v] $(grep -o '"value": [0-9.]*' gpurun_out/ab_cur.json | head -1) $(grep -o '"passes_ms": {[^}]*}' gpurun_out/ab_cur.json | head -1) ctx=$(grep -o '"contexts_per_gpu": [0-9]*' gpurun_out/ab_cur.json | head -1 | grep -o '[0-9]*$') ok=$(grep -o '"ok": [a-z]*' gpurun_out/ab_cur.json | head -1 | grep -o '[a-z]*$')" >> "$OUT"
  done
done
cat "$OUT"
