#!/bin/bash
# Build the working tree's library with extra compile definitions into lib/libomega_<name>.so (A/B of
# build-time variants on one box: tools/ab.sh with AB_LIBS, tools/step_probe.py --lib ...).
#   tools/build_variant.sh p1 "-DOMEGA_PLAN_PAT=1"
set -eu -o pipefail
NAME=$1
DEFS=$2
REPO=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/omega_var.XXXXXX)
mkdir -p "$W/audio-analyzer-omega_amd" "$W/include"
cp -r "$REPO/audio-analyzer-omega_amd/csrc" "$REPO/audio-analyzer-omega_amd/Makefile" "$W/audio-analyzer-omega_amd/"
cp "$REPO/include/omega.h" "$W/include/"
make -C "$W/audio-analyzer-omega_amd" -j8 CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize $DEFS" >/dev/null
cp "$W/audio-analyzer-omega_amd/lib/libomega.so" "$REPO/audio-analyzer-omega_amd/lib/libomega_$NAME.so"
rm -rf "$W"
echo "lib/libomega_$NAME.so ($DEFS)"
