#!/bin/bash
# Round 4, session 2: where the c3 pipeline's time goes on bench.py's image
# (timing-probe builds in build/ab, wrong results except base), alternating
# processes, then a kernel trace of each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s2; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
$R/tools/ab_dev.sh r4s2 3 zipf $A/base.so $A/ctl16384.so $A/nocap.so $A/nofin.so $A/rowsonly.so $A/hop16.so $A/hop8.so || exit 99
for L in base hop16 hop8 rowsonly; do
  $R/tools/box_step.sh 300 $O/tl_$L.log rocprofv3 --kernel-trace -d $O/tl_$L -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/$L.so --iters 3 || exit 99
  python3 $R/tools/kernel_timeline.py $O/tl_$L --after k_count_hist | tail -8 > $O/timeline_$L.txt 2>&1
done
echo done > $O/DONE
