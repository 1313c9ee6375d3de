#!/bin/bash
# Round 4, session 24: C2 with the even-index workgroups taking 4 % / 8 % more
# blocks than the odd ones (XCD-weighted halves), parity then A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s24; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
REVEL_LIB=$A/xcd80.so step 400 $O/pytest_xcd80.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_fullsize.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "full_blocks or synth or c2"
ok $O/pytest_xcd80.log || { echo "xcd80 tests failed"; tail -40 $O/pytest_xcd80.log; exit 1; }
$R/tools/ab_c2.sh r4s24 5 $R/revel_amd/librevel_wal.so $A/xcd40.so $A/xcd80.so || exit 99
echo done > $O/DONE
