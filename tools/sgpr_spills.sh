#!/bin/bash
# SGPR spills (v_writelane) and SGPR / VGPR counts per kernel of one source file, from the device assembly.
# mt_vconv sits at the 100-SGPR limit: run this before and after any change that adds wave-uniform state, and A/B
# the two BUILDS (tools/ab_build.sh + tools/ab_run.sh) rather than a knob inside one build (experiments that lost).
# Usage: bash tools/sgpr_spills.sh matcha-tts_amd/csrc/mt_vconv.hip [extra hipcc flags]
set -o pipefail
SRC=${1:?source file}; shift
OUT=$(mktemp /tmp/sgpr_XXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --cuda-device-only -S -Imatcha-tts_amd/csrc "$@" "$SRC" -o "$OUT" 2>/dev/null || exit 1
awk '/^_ZN2mt.*:/{name=$1; wl=0; sg=""; vg=""} /v_writelane/{wl++} /amdhsa_next_free_sgpr/{sg=$2} /amdhsa_next_free_vgpr/{vg=$2}
     /\.end_amdhsa_kernel/{ if (name != "") printf "%4d spills  sgpr %4s  vgpr %4s  %s\n", wl, sg, vg, name; name="" }' "$OUT" | sort -rn
rm -f "$OUT"
