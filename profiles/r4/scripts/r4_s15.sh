#!/bin/bash
# Round 4, session 15: the session-14 dense changes one at a time (3-input xor
# in absorb; pad fixup by LDS table; last word after the loop with grouped
# break checks), A/B on the small-record image; parity of each on the dense tests.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s15; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
for L in x3 pad lw; do
  REVEL_LIB=$A/$L.so step 300 $O/pytest_$L.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dense or small or verify_paths"
  ok $O/pytest_$L.log || { echo "$L tests failed"; tail -40 $O/pytest_$L.log; exit 1; }
done
$R/tools/ab_dev.sh r4s15 3 small $A/base.so $A/x3.so $A/pad.so $A/lw.so || exit 99
echo done > $O/DONE
