#!/bin/bash
# Build an A/B variant of libsldm_sage.so into ab/lib_<name>.so with extra
# compiler flags (e.g. -DSLDM_WSLN_PF=1); objects under ab/obj_<name>.
# Usage: tools/ab_build.sh <name> "<flags>"
set -e
NAME=${1:?name}; FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/ab"
make -s -C "$ROOT/sldm-gnn_amd/csrc" -j8 OBJDIR="$ROOT/ab/obj_$NAME" \
  LIB="$ROOT/ab/lib_$NAME.so" EXTRA="$FLAGS" "$ROOT/ab/lib_$NAME.so"
