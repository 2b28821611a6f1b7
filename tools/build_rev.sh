#!/bin/bash
# Build librmr.so of a git revision (or of the working tree with "WT") into OUT, for same-process
# A/B runs with tools/abrun.py lib:PATH (each library embeds its own hipRTC source).
#   tools/build_rev.sh REV OUT [EXTRA]      e.g. tools/build_rev.sh HEAD tools/librmr_base.so
set -e
REV=$1; OUT=$(realpath -m "$2"); EXTRA=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
if [ "$REV" = WT ]; then
  mkdir -p "$T/raymarchrenderer_amd"
  cp -r "$ROOT/raymarchrenderer_amd/csrc" "$T/raymarchrenderer_amd/"; cp -r "$ROOT/include" "$T/"
  rm -rf "$T"/raymarchrenderer_amd/csrc/build*
else
  git -C "$ROOT" archive "$REV" raymarchrenderer_amd/csrc include | tar -x -C "$T"
fi
TGT=$(grep -q "^lib:" "$T/raymarchrenderer_amd/csrc/Makefile" && echo lib || true)   # (older revisions: no lib target)
make -s -C "$T/raymarchrenderer_amd/csrc" -j8 $TGT BUILD="$T/build" OUT="$OUT" EXTRA="$EXTRA"
rm -rf "$T"
echo "built $OUT from $REV"
