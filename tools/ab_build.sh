#!/bin/bash
# Build the library of another git revision (default HEAD) into lib/libomega_ab.so, for A/B runs of
# two builds on one GPU box (tools/step_probe.py --lib, tools/kernel_bench.py --lib, tools/dc_probe.py
# --lib). The working tree's lib/libomega.so is untouched.
set -eu -o pipefail
REV=${1:-HEAD}
OUTN=${2:-libomega_ab.so}
REPO=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/omega_ab.XXXXXX)
git -C "$REPO" archive "$REV" audio-analyzer-omega_amd/csrc audio-analyzer-omega_amd/Makefile include | tar -x -C "$W"
make -C "$W/audio-analyzer-omega_amd" -j8 >/dev/null
cp "$W/audio-analyzer-omega_amd/lib/libomega.so" "$REPO/audio-analyzer-omega_amd/lib/$OUTN"
rm -rf "$W"
echo "lib/$OUTN <- $(git -C "$REPO" rev-parse --short "$REV")"
