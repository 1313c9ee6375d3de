#!/bin/bash
# Round 4, session 18: k_verify_rows taking list positions from a counter
# (dyn) after the wave-slot analysis of session 17 (older waves finish first:
# 511 / 576 / 640 / 723 us by slot group).  Parity, A/B on the Zipf and small
# images, per-wave end times of the dyn build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s18; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
REVEL_LIB=$A/dyn.so step 400 $O/pytest_dyn.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or expander or append or replay or reader or golden or guard or unmapped"
ok $O/pytest_dyn.log || { echo "dyn tests failed"; tail -40 $O/pytest_dyn.log; exit 1; }
step 300 $O/wavetime_dyn.log python3 $R/tools/rows_wavetime.py --lib $A/dynwt.so --shape zipf
$R/tools/ab_dev.sh r4s18 4 zipf $A/base.so $A/dyn.so || exit 99
$R/tools/ab_dev.sh r4s18 2 small $A/base.so $A/dyn.so || exit 99
echo done > $O/DONE
