#!/bin/bash
# Kernel traces of the c3_small leg on a 192 MiB image (resident in the 256 MiB
# Infinity Cache across back-to-back calls) vs the 4 GiB one: per-byte cost of
# the count pass and dense2 when their reads hit on-die.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mall
mkdir -p $O
for g in 0.1875 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t_$g -o run -- python3 $R/tools/c3_legs.py --shapes small,zipf --gib $g --iters 20 >> $O/legs_$g.log 2>&1
done
