#!/bin/bash
# A/B of two builds of librevel_wal.so on C2 (1 Mi full blocks), alternating
# processes; each process also times the streaming-read ceiling (variant 100,
# experiments library) so every run carries its own reference:
#   tools/ab_c2.sh <tag> A.so B.so [rounds]
set -u
tag=$1; A=$2; B=$3; n=${4:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab2_$tag
mkdir -p "$O"
for i in $(seq 1 "$n"); do
  for L in "$A" "$B"; do
    "$R/tools/box_step.sh" 300 "$O/run_${i}_$(basename "$L").log" \
        python3 "$R/tools/variants.py" --lib "$L" --variants 100,0 --rounds 3 --iters 3 || exit 99
  done
done
for L in "$A" "$B"; do
  echo "== $(basename "$L")"
  grep -h '"variant": 0' "$O"/run_*_"$(basename "$L")".log
  grep -h '"variant": 100' "$O"/run_*_"$(basename "$L")".log
done | tee "$O/summary.txt"
