#!/bin/bash
# Round 4, session 17: load balance of k_verify_rows (per-wave start / end
# times of a probe build) on bench.py's Zipf image.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s17; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 300 $O/wavetime_zipf.log python3 $R/tools/rows_wavetime.py --lib $A/wavetime.so --shape zipf
step 300 $O/wavetime_small.log python3 $R/tools/rows_wavetime.py --lib $A/wavetime.so --shape zipf --gib 1
echo done > $O/DONE
