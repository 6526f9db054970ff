#!/bin/bash
# Build-vs-build A/B, step 1 (CPU, in this container): build libmatcha_hip.so at git revisions, each from a clean
# `git worktree` checkout, into matcha-tts_amd/ab/<name>.so (git-ignored; it travels to the GPU box with the tree).
#   bash tools/ab_build.sh base=HEAD~1 new=WORKTREE
# REV "WORKTREE" is the current working tree (uncommitted edits included). Step 2 is tools/ab_run.sh on the box.
# Only the library is swapped (MT_LIB); the Python side is the working tree's, so both revisions must export the
# entry points the timing tools call (matcha_hip/_lib.py skips signatures an older build lacks).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/matcha-tts_amd/ab"
for spec in "$@"; do
  name=${spec%%=*}; rev=${spec#*=}
  if [ "$rev" = WORKTREE ]; then
    make -s -C "$ROOT/matcha-tts_amd" -j8
    cp "$ROOT/matcha-tts_amd/libmatcha_hip.so" "$ROOT/matcha-tts_amd/ab/$name.so"
  else
    wt=$(mktemp -d /tmp/ab_wt.XXXXXX)
    git -C "$ROOT" worktree add -q --detach "$wt" "$rev"
    make -s -C "$wt/matcha-tts_amd" -j8 libmatcha_hip.so
    cp "$wt/matcha-tts_amd/libmatcha_hip.so" "$ROOT/matcha-tts_amd/ab/$name.so"
    git -C "$ROOT" worktree remove --force "$wt"
  fi
  echo "$name <- $rev: matcha-tts_amd/ab/$name.so"
done
