#!/bin/bash
# Round 4, session 29: count pass touching the other 64-B half of each hop's
# 128-B line (so a next header in the same line hits L2), A/B on both images.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s29; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
$R/tools/ab_dev.sh r4s29 3 small $A/base.so $A/cline.so || exit 99
$R/tools/ab_dev.sh r4s29 3 zipf $A/base.so $A/cline.so || exit 99
for L in base cline; do
  step 300 $O/tl_$L.log rocprofv3 --kernel-trace -d $O/tl_$L -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/$L.so --shape small --iters 3
  python3 $R/tools/kernel_timeline.py $O/tl_$L --after k_count_hist | tail -6 > $O/timeline_$L.txt 2>&1
done
echo done > $O/DONE
