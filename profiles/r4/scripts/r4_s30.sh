#!/bin/bash
# Round 4, session 30: the driver's bench command twice more on the final build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s30; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 400 $O/bench1.log python3 $R/bench.py
step 400 $O/bench2.log python3 $R/bench.py
echo done > $O/DONE
