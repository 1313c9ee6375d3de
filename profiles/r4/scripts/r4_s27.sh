#!/bin/bash
# Round 4, session 27: dense loads a lane does not need masked off by EXEC
# instead of addressed out of range (exm): parity, A/B on the small image.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s27; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
REVEL_LIB=$A/exm.so step 300 $O/pytest_exm.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or dense or small or guard or unmapped"
ok $O/pytest_exm.log || { echo "exm tests failed"; tail -40 $O/pytest_exm.log; exit 1; }
$R/tools/ab_dev.sh r4s27 4 small $A/base.so $A/exm.so || exit 99
echo done > $O/DONE
