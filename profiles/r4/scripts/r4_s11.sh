#!/bin/bash
# Round 4, session 11: C2 with the blocks visited in a scrambled order
# (sigma(i) = i * amul mod n) -- parity of the C2 tests on it, then A/B against
# the in-tree build on bench.py's C2 leg (alternating processes).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s11; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
REVEL_LIB=$A/c2scr.so step 400 $O/pytest_c2scr.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_fullsize.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "full_blocks or synth or c2"
ok $O/pytest_c2scr.log || { echo "c2scr tests failed"; tail -40 $O/pytest_c2scr.log; exit 1; }
$R/tools/ab_c2.sh r4s11 4 $R/revel_amd/librevel_wal.so $A/c2scr.so || exit 99
echo done > $O/DONE
