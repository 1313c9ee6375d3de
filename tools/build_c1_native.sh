#!/bin/bash
# Builds tools/c1_native against the in-tree revel_amd/librevel_wal.so (build it first).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
g++ -O2 -std=c++17 -Wall -Wextra -I"$R/include" "$R/tools/c1_native.cpp" -L"$R/revel_amd" -lrevel_wal \
    -Wl,-rpath,'$ORIGIN/../revel_amd' -o "$R/tools/c1_native"
