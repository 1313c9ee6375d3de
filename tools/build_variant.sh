#!/bin/bash
# Build a variant of librevel_wal.so with extra device compile flags into
# build/ab/<name>.so (objects in build/ab/<name>/), for A/B runs:
#   tools/build_variant.sh <name> [-DMACRO=value ...]
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/build/ab"
make -s -C "$R/revel_amd/csrc" -j8 OUT="$R/build/ab/$name.so" BUILD="$R/build/ab/$name" XFLAGS="$*" \
    "$R/build/ab/$name.so"
echo "$R/build/ab/$name.so"
