#!/bin/bash
# Round 4, session 14: dense verify absorbing whole words only in its chunk
# loop (last word after it, pad fixup by LDS table, 3-input xor in absorb,
# break checks every 4 words): parity, then A/B against the current build on
# bench.py's small-record image; timelines.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s14; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
REVEL_LIB=$A/lastw.so step 400 $O/pytest_lastw.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or dense or guard or unmapped or replay or reader or golden or append"
ok $O/pytest_lastw.log || { echo "lastw tests failed"; tail -40 $O/pytest_lastw.log; exit 1; }
REVEL_LIB=$A/lastw.so step 300 $O/pytest_lastw_full.log python3 -u -m pytest $R/tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
ok $O/pytest_lastw_full.log || { echo "lastw fullsize failed"; tail -40 $O/pytest_lastw_full.log; exit 1; }
$R/tools/ab_dev.sh r4s14 3 small $A/base.so $A/lastw.so || exit 99
for L in base lastw; do
  step 300 $O/tl_$L.log rocprofv3 --kernel-trace -d $O/tl_$L -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/$L.so --shape small --iters 5
  python3 $R/tools/kernel_timeline.py $O/tl_$L --after k_count_hist | tail -6 > $O/timeline_$L.txt 2>&1
done
echo done > $O/DONE
