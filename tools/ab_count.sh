#!/bin/bash
# GPU suite on the in-tree build, then count+scan A/B of two builds on the C3 image:
#   tools/ab_count.sh <tag> A.so B.so [rounds]
set -u
tag=$1; A=$2; B=$3; n=${4:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_$tag; mkdir -p $O
"$R/tools/box_step.sh" 600 "$O/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 --timeout-method thread || exit 99
grep -q " passed" "$O/pytest.log" && ! grep -q "failed" "$O/pytest.log" || { tail -30 "$O/pytest.log"; exit 1; }
for i in $(seq 1 "$n"); do
  for L in "$A" "$B"; do
    "$R/tools/box_step.sh" 300 "$O/run_${i}_$(basename "$L").log" python3 "$R/tools/bench_c3.py" --lib "$L" --variants 0 --rounds 2 --iters 5 --keep-tail || exit 99
  done
done
