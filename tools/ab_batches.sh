#!/bin/bash
# A/B of two builds on tools/bench_batches.py (fill1 / fill100 replay in HBM), alternating processes:
#   tools/ab_batches.sh <tag> A.so B.so [rounds]
set -u
tag=$1; A=$2; B=$3; n=${4:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_$tag
mkdir -p "$O"
for i in $(seq 1 "$n"); do
  for L in "$A" "$B"; do
    "$R/tools/box_step.sh" 300 "$O/run_${i}_$(basename "$L").log" python3 "$R/tools/bench_batches.py" --lib "$L" --iters 5 || exit 99
  done
done
