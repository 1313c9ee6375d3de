#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s0; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 300 $O/bench.log python3 $R/bench.py --no-cpu
step 300 $O/tl.log rocprofv3 --kernel-trace -d $O/tl -o tl -- python3 $R/bench.py --blocks 65536 --steps 3 --warmup 1 --no-cpu --e2e-gib 0
python3 $R/tools/kernel_timeline.py $O/tl --after k_count_hist > $O/timeline.txt 2>&1
echo done > $O/DONE
