#!/bin/bash
# Round 4, session 16: the walk experiment after its RowsState fix; the rows
# kernel loading a block's header entries by its record lanes only (epred),
# parity + A/B against the current build on bench.py's Zipf image.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s16; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
step 300 $O/pytest_experiments.log python3 -u -m pytest $R/tests/test_experiments_gpu.py -m experiment -q --timeout 120 --timeout-method thread -p no:cacheprovider
REVEL_LIB=$A/epred.so step 400 $O/pytest_epred.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or expander"
ok $O/pytest_epred.log || { echo "epred tests failed"; tail -40 $O/pytest_epred.log; exit 1; }
$R/tools/ab_dev.sh r4s16 4 zipf $A/base.so $A/epred.so || exit 99
echo done > $O/DONE
