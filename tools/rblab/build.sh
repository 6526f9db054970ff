#!/bin/bash
# Builds tools/rblab/rblab (CPU, in this container; the binary travels to the GPU box with the tree): the stage 1-2
# ResBlock conv kernel (mt_rbconv.hip) compiled several times, each in its own namespace, like tools/pairlab:
#   mt_base   from git revision BASE (default HEAD): the reference for bit identity and timing;
#   mt        the working tree, as the library builds it;
#   mt_ts     the working tree with -DVPAIR_TS (phase stamps, mt_ts.h);
#   mt_<v>    one per VARIANTS entry "v:flags" (comma-separated extra -D flags), e.g. VARIANTS="x4:-DRB_EXP=4"
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
S=$ROOT/matcha-tts_amd/csrc
O=$ROOT/tools/rblab/obj
rm -rf "$O"; mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result"
KF="-mno-amdgpu-ieee -fno-honor-nans"
B=$O/base_src
mkdir -p "$B"
git -C "$ROOT" archive "${BASE:-HEAD}" matcha-tts_amd/csrc | tar -x -C "$B"
builds=("base||$B/matcha-tts_amd/csrc" "mt||$S" "ts|-DVPAIR_TS|$S")
for v in ${VARIANTS:-}; do fl=${v#*:}; builds+=("${v%%:*}|${fl//,/ }|$S"); done
pids=()
inc=$O/variants.inc decl=$O/variants_decl.inc
: > "$inc"; : > "$decl"
for bspec in "${builds[@]}"; do
  IFS='|' read -r name flags dir <<< "$bspec"
  ns=$([ "$name" = mt ] && echo mt || echo "mt_$name")
  /opt/rocm/bin/hipcc $F -I"$dir" $KF $flags -Dmt=$ns -c "$dir/mt_rbconv.hip" -o "$O/mt_rbconv_$name.o" & pids+=($!)
  for f in mt_error mt_probe; do
    /opt/rocm/bin/hipcc $F -I"$dir" -x hip $flags -Dmt=$ns -c "$dir/$f.cpp" -o "$O/${f}_$name.o" & pids+=($!)
  done
  if [ "$name" != mt ] && [ "$name" != ts ] && [ "$name" != base ]; then
    echo "namespace $ns { struct VConvArgs; int launch_rbconv(int, const VConvArgs&, int, hipStream_t); }" >> "$decl"
    echo "VARIANT($name, $ns)" >> "$inc"
  fi
done
/opt/rocm/bin/hipcc $F -I"$S" -I"$O" -x hip -c "$ROOT/tools/rblab/rblab.cpp" -o "$O/rblab.o" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 "$O"/*.o -o "$ROOT/tools/rblab/rblab"
echo "built tools/rblab/rblab (variants: base mt ts ${VARIANTS:-})"
