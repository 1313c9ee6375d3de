#!/bin/bash
# Round 4, session 23: per-wave end times of the rows kernel with priority rotation.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s23; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 300 $O/wavetime_prio.log python3 $R/tools/rows_wavetime.py --lib $R/build/ab/rwt.so --shape zipf
echo done > $O/DONE
