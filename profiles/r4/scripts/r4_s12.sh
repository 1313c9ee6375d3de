#!/bin/bash
# Round 4, session 12: the product suite on the current build (dense loads
# past a lane's stream addressed out of range); C2 scrambled order vs in-tree,
# 6 alternating rounds; c3 / c3_small of the current build vs the previous
# commit (prev.so).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s12; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
step 600 $O/pytest_product.log python3 -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
ok $O/pytest_product.log || { echo "product tests failed"; tail -40 $O/pytest_product.log; exit 1; }
$R/tools/ab_c2.sh r4s12 6 $R/revel_amd/librevel_wal.so $A/c2scr.so || exit 99
$R/tools/ab_dev.sh r4s12 2 small $A/prev.so $R/revel_amd/librevel_wal.so || exit 99
echo done > $O/DONE
