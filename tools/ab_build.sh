#!/bin/bash
# Build the libraries of git revision REV (or the working tree: "-") into
# abtest/NAME/ for tools/ab.sh.  Usage: bash tools/ab_build.sh NAME [REV]
set -e
NAME=$1; REV=${2:--}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/abtest/$NAME
mkdir -p "$OUT"
if [ "$REV" = "-" ]; then
  make -s -C "$ROOT/broadway_amd/csrc"
  cp "$ROOT"/broadway_amd/lib/*.so "$ROOT"/broadway_amd/lib/h264mi_dec "$OUT/"
else
  TMP=$(mktemp -d)
  git -C "$ROOT" archive "$REV" broadway_amd/csrc include bindings | tar -x -C "$TMP"
  mkdir -p "$TMP/broadway_amd/lib"
  make -s -C "$TMP/broadway_amd/csrc" -j8
  cp "$TMP"/broadway_amd/lib/*.so "$TMP"/broadway_amd/lib/h264mi_dec "$OUT/"
  rm -rf "$TMP"
fi
ls -la "$OUT"
