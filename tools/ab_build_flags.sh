#!/bin/bash
# Build the working tree's libraries with extra compile flags (study
# switches, e.g. -DSTUDY_DEP_NOPOLL) into abtest/NAME/ for tools/ab.sh /
# tools/ab_env.sh.  Usage: bash tools/ab_build_flags.sh NAME "-DFLAG ..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/abtest/$NAME
mkdir -p "$OUT/obj"
make -s -C "$ROOT/broadway_amd/csrc" -j8 OUT="$OUT" OBJ="$OUT/obj" \
  HIPFLAGS="-O3 -fPIC --offload-arch=gfx950 -std=c++17 -Wno-unused-result $FLAGS" \
  "$OUT/libh264mi.so" "$OUT/h264mi_dec"
cp "$ROOT/broadway_amd/lib/libh264gen.so" "$OUT/"
rm -rf "$OUT/obj"
ls -la "$OUT"
