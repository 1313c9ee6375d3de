#!/bin/bash
# Round 4, session 6: count pass with a self-prefetch of the line after the
# next window from hop 4 / 8 / 16 on (A/B on bench.py's images), parity first.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s6; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
REVEL_LIB=$A/pf8.so step 300 $O/pytest_pf8.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or count"
$R/tools/ab_dev.sh r4s6 3 zipf $A/base.so $A/pf4.so $A/pf8.so $A/pf16.so || exit 99
$R/tools/ab_dev.sh r4s6 2 small $A/base.so $A/pf8.so || exit 99
for L in base pf8; do
  step 300 $O/tl_$L.log rocprofv3 --kernel-trace -d $O/tl_$L -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/$L.so --iters 5
  python3 $R/tools/kernel_timeline.py $O/tl_$L --after k_count_hist | tail -6 > $O/timeline_$L.txt 2>&1
done
echo done > $O/DONE
