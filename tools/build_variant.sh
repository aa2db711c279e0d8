#!/bin/bash
# Experiment build: tools/build_variant.sh NAME 'EXTRA defines' [DEV_TAPS]
# -> build/var_NAME/libvectorwave_amd.so (load with VW_LIB_PATH=...).  Not the product build.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; EXTRA=$2; TAPS=${3:-X(8)}
D="$ROOT/${VARDIR:-build}/var_$NAME"
mkdir -p "$D/src/csrc" "$D/include"
cp "$ROOT"/vectorwave_amd/csrc/* "$D/src/csrc/" 2>/dev/null || true
rm -f "$D"/src/csrc/*.o
cp "$ROOT"/include/*.h "$D/include/"
# the Makefile's include path is ../../include relative to csrc
mkdir -p "$D/src/include" && cp "$ROOT"/include/*.h "$D/src/include/"
make -C "$D/src/csrc" -j8 -s OUT="$D/libvectorwave_amd.so" EXTRA="$EXTRA" DEV_TAPS="$TAPS" > "$D/build.log" 2>&1
echo "$D/libvectorwave_amd.so"
