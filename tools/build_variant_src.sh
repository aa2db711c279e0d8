#!/bin/bash
# Experiment build from the working tree with one source file replaced by its version at a git revision:
# tools/build_variant_src.sh NAME REV FILE 'EXTRA defines' [DEV_TAPS]  -> build/var_NAME/libvectorwave_amd.so
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; REV=$2; FILE=$3; EXTRA=$4; TAPS=${5:-X(8)}
D="$ROOT/build/var_$NAME"
mkdir -p "$D/src/csrc" "$D/include"
cp "$ROOT"/vectorwave_amd/csrc/* "$D/src/csrc/" 2>/dev/null || true
rm -f "$D"/src/csrc/*.o
cp "$ROOT"/include/*.h "$D/include/"
git -C "$ROOT" show "$REV:vectorwave_amd/csrc/$FILE" > "$D/src/csrc/$FILE"
make -C "$D/src/csrc" -j8 -s OUT="$D/libvectorwave_amd.so" EXTRA="$EXTRA" DEV_TAPS="$TAPS" > "$D/build.log" 2>&1
echo "$D/libvectorwave_amd.so"
