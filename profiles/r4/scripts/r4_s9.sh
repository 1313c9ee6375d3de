#!/bin/bash
# Round 4, session 9: captures carried across blocks (REVEL_CAP_CARRY: flushes
# only of full groups, at batch flushes and for 64-record blocks): parity of
# the verify tests on it, then A/B against the same source without it (base)
# and the previous commit (prev) on bench.py's Zipf image; timelines.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s9; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
REVEL_LIB=$A/carry.so step 400 $O/pytest_carry.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or dense or expander or guard or unmapped or replay or reader or golden or append"
ok $O/pytest_carry.log || { echo "carry tests failed"; tail -40 $O/pytest_carry.log; exit 1; }
REVEL_LIB=$A/carry.so step 300 $O/pytest_carry_full.log python3 -u -m pytest $R/tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
ok $O/pytest_carry_full.log || { echo "carry fullsize failed"; tail -40 $O/pytest_carry_full.log; exit 1; }
$R/tools/ab_dev.sh r4s9 4 zipf $A/prev.so $A/base.so $A/carry.so || exit 99
for L in base carry; do
  step 300 $O/tl_$L.log rocprofv3 --kernel-trace -d $O/tl_$L -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/$L.so --iters 5
  python3 $R/tools/kernel_timeline.py $O/tl_$L --after k_count_hist | tail -6 > $O/timeline_$L.txt 2>&1
done
echo done > $O/DONE
