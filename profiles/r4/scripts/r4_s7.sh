#!/bin/bash
# Round 4, session 7: where the count pass's time goes -- kernel timelines of
# builds whose walk stops after 1/2/4/8/16 hops (timing only: their counts are
# wrong) against the product build, on bench.py's Zipf and small images; the
# c3 legs timed both ways (isolated calls, calls queued back to back).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s7; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
for shp in zipf small; do
  for L in base mh1 mh2 mh4 mh8 mh16; do
    step 300 $O/tl_${shp}_$L.log rocprofv3 --kernel-trace -d $O/tl_${shp}_$L -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/$L.so --shape $shp --iters 5
    python3 $R/tools/kernel_timeline.py $O/tl_${shp}_$L --after k_count_hist | tail -6 > $O/timeline_${shp}_$L.txt 2>&1
    grep '^{' $O/tl_${shp}_$L.log >> $O/timeline_${shp}_$L.txt
  done
done
step 300 $O/c3dev_zipf.log python3 $R/tools/bench_c3dev.py --shape zipf --iters 9 --rounds 2
step 300 $O/c3dev_small.log python3 $R/tools/bench_c3dev.py --shape small --iters 9 --rounds 2
echo done > $O/DONE
