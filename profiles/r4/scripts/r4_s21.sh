#!/bin/bash
# Round 4, session 21: C2 with wave priorities rotated per block (s_setprio
# (age + blocks done) & 3) against the in-tree build; per-wave end times.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s21; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
REVEL_LIB=$A/c2prio.so step 400 $O/pytest_c2prio.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "full_blocks or synth or c2"
ok $O/pytest_c2prio.log || { echo "c2prio tests failed"; tail -40 $O/pytest_c2prio.log; exit 1; }
step 300 $O/c2_wavetime_prio.log python3 $R/tools/c2_wavetime.py --lib $A/c2priowt.so
$R/tools/ab_c2.sh r4s21 4 $R/revel_amd/librevel_wal.so $A/c2prio.so || exit 99
echo done > $O/DONE
