#!/bin/bash
# Timing-experiment builds (CPU, in this container): the in-tree objects with ONE source recompiled under extra
# defines, linked into matcha-tts_amd/ab/<name>.so (git-ignored; it travels to the GPU box). The experiment
# macros (VPAIR_EXP, VCONV_EXP) drop parts of a kernel's work, so such a library computes WRONG results: use it
# only with the timing tools (MT_LIB=...), never for tests.
#   bash tools/exp_build.sh NAME SOURCE.hip "-DVPAIR_EXP=1" [SOURCE2.hip "-D..."]...
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
M=$ROOT/matcha-tts_amd
name=$1; shift
make -s -C "$M" -j8 libmatcha_hip.so
mkdir -p "$M/ab" "$M/build_exp/$name"
objs=$(ls "$M"/build/*.o)
while [ $# -gt 0 ]; do
  src=$1; defs=$2; shift 2
  base=$(basename "$src")
  extra=""
  case "$base" in mt_rbfuse.hip|mt_rbconv.hip|mt_vpair.hip|mt_vpair32.hip|mt_vpair128.hip) extra="-mno-amdgpu-ieee -fno-honor-nans";; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $extra $defs \
    -c "$M/csrc/$base" -o "$M/build_exp/$name/$base.o"
  objs=$(echo "$objs" | sed "s#$M/build/$base.o#$M/build_exp/$name/$base.o#")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o "$M/ab/$name.so"
echo "$name: matcha-tts_amd/ab/$name.so"
