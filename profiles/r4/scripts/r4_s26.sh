#!/bin/bash
# Round 4, session 26: priority rotation at a finer grain -- per 32-word chunk
# in the dense kernel (dp2), per 8-row part in the rows kernel (rp2).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s26; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
for L in dp2 rp2; do
  REVEL_LIB=$A/$L.so step 300 $O/pytest_$L.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify_paths or dense or small or expander"
  ok $O/pytest_$L.log || { echo "$L tests failed"; tail -40 $O/pytest_$L.log; exit 1; }
done
$R/tools/ab_dev.sh r4s26 3 small $A/base.so $A/dp2.so || exit 99
$R/tools/ab_dev.sh r4s26 4 zipf $A/base.so $A/rp2.so || exit 99
echo done > $O/DONE
