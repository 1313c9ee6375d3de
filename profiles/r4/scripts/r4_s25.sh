#!/bin/bash
# Round 4, session 25: the XCD-weighted C2 split, longer A/B (8 rounds) and
# per-wave end times by XCD with and without it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s25; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 300 $O/wt_base.log python3 $R/tools/c2_wavetime.py --lib $A/c2wt.so
step 300 $O/wt_xcd80.log python3 $R/tools/c2_wavetime.py --lib $A/xcd80wt.so
$R/tools/ab_c2.sh r4s25 8 $R/revel_amd/librevel_wal.so $A/xcd80.so $A/xcd120.so || exit 99
echo done > $O/DONE
