#!/bin/bash
# Builds tools/pairlab/pairlab (CPU, in this container; the binary travels to the GPU box with the tree).
# The pair kernels (mt_vpair / mt_vpair32 / mt_vpair128) are compiled several times, each in its own namespace:
#   mt_base   from git revision BASE (default HEAD): the reference for bit identity and timing;
#   mt        the working tree, as the library builds it;
#   mt_ts     the working tree with -DVPAIR_TS (phase stamps, mt_ts.h);
#   mt_<v>    one per VARIANTS entry "v:flags" (the working tree with extra -D flags), e.g.
#             VARIANTS="rd:-DVP_READS=1 both:-DVP_READS=1,-DVP_DMA=1" bash tools/pairlab/build.sh
# The lab times every build against mt_base in alternating blocks and checks each bit for bit against it.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
S=$ROOT/matcha-tts_amd/csrc
O=$ROOT/tools/pairlab/obj
rm -rf "$O"; mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result"
KF="-mno-amdgpu-ieee -fno-honor-nans"
B=$O/base_src
mkdir -p "$B"
git -C "$ROOT" archive "${BASE:-HEAD}" matcha-tts_amd/csrc | tar -x -C "$B"
# name|flags|source dir
builds=("base||$B/matcha-tts_amd/csrc" "mt||$S" "ts|-DVPAIR_TS|$S")
for v in ${VARIANTS:-}; do fl=${v#*:}; builds+=("${v%%:*}|${fl//,/ }|$S"); done  # flags: comma-separated
pids=()
inc=$O/variants.inc decl=$O/variants_decl.inc
: > "$inc"; : > "$decl"
for bspec in "${builds[@]}"; do
  IFS='|' read -r name flags dir <<< "$bspec"
  ns=$([ "$name" = mt ] && echo mt || echo "mt_$name")
  for f in mt_vpair mt_vpair32 mt_vpair128; do
    /opt/rocm/bin/hipcc $F -I"$dir" $KF $flags -Dmt=$ns -c "$dir/$f.hip" -o "$O/${f}_$name.o" & pids+=($!)
  done
  for f in mt_error mt_probe; do
    /opt/rocm/bin/hipcc $F -I"$dir" -x hip $flags -Dmt=$ns -c "$dir/$f.cpp" -o "$O/${f}_$name.o" & pids+=($!)
  done
  if [ "$name" != mt ] && [ "$name" != ts ] && [ "$name" != base ]; then
    echo "namespace $ns { struct VPairArgs; int launch_vpair(int, const VPairArgs&, hipStream_t); int launch_vpair32(int, const VPairArgs&, hipStream_t); int launch_vpair128(int, const VPairArgs&, hipStream_t); }" >> "$decl"
    echo "VARIANT($name, $ns)" >> "$inc"
  fi
done
/opt/rocm/bin/hipcc $F -I"$S" -I"$O" -x hip -c "$ROOT/tools/pairlab/pairlab.cpp" -o "$O/pairlab.o" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 "$O"/*.o -o "$ROOT/tools/pairlab/pairlab"
echo "built tools/pairlab/pairlab (variants: base mt ts ${VARIANTS:-})"
