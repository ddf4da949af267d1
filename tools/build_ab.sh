#!/bin/bash
# Build liblcclip.so from the native sources at a git revision (or the working tree: rev "WT")
# into lifelong-clip_amd/lcclip/ab/<name>.so for same-box A/Bs and diagnostic variants
# (LCCLIP_LIB=<path> selects it at run time; the .so travels with gpurun, git ignores it).
# usage: bash tools/build_ab.sh <rev|WT> <name> [EXTRA_FLAGS...]
set -e
REV=$1; NAME=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/ab_XXXX)
if [ "$REV" = "WT" ]; then
  mkdir -p "$TMP/lifelong-clip_amd"
  cp -r "$ROOT/lifelong-clip_amd/csrc" "$TMP/lifelong-clip_amd/" && cp -r "$ROOT/include" "$TMP/"
  rm -rf "$TMP/lifelong-clip_amd/csrc/build"*
else
  git -C "$ROOT" archive "$REV" lifelong-clip_amd/csrc include | tar -x -C "$TMP"
fi
mkdir -p "$ROOT/lifelong-clip_amd/lcclip/ab"
make -s -C "$TMP/lifelong-clip_amd/csrc" -j8 OUT="$ROOT/lifelong-clip_amd/lcclip/ab/$NAME.so" \
  EXTRA_FLAGS="$*" > /dev/null 2>&1
rm -rf "$TMP"
echo "$ROOT/lifelong-clip_amd/lcclip/ab/$NAME.so"
