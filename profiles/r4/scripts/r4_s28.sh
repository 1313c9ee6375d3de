#!/bin/bash
# Round 4, session 28: 2-rank rehearsal of the driver's multi-GPU bench command
# on one GPU (ranks share it), with the round-4 legs (c3 steady state, c3_small).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s28; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 600 $O/bench_gpus2_share.log python3 $R/bench.py --gpus 2 --share-gpus --steps 5 --warmup 1 --e2e-gib 1 --c3-gib 1 --c3-small-gib 1
echo done > $O/DONE
