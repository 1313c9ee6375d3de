#!/bin/bash
# Round 4, session 4: the VMM probe one mode per process; dense2 parity
# (walk2 verify paths, guard module with the fused paths); the small-record
# image: count-pass pipeline vs fused + dense2, kernel timelines of both
# pipelines on both images.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s4; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
for m in nosync sync keepva keepphys plain; do
  step 200 $O/vmm_$m.log python3 -u $R/tools/vmm_probe.py --iters 20 --modes $m
done
step 300 $O/pytest_walk2.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "walk2 or dense"
step 300 $O/pytest_guard.log python3 -u -m pytest $R/tests/test_gpu_guard.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider
for shp in small zipf; do
  for w in 0 1 3; do
    step 300 $O/tl_${shp}_$w.log rocprofv3 --kernel-trace -d $O/tl_${shp}_$w -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/base.so --shape $shp --walk $w --iters 3
    python3 $R/tools/kernel_timeline.py $O/tl_${shp}_$w --after k_count_hist | tail -8 > $O/timeline_${shp}_$w.txt 2>&1
    python3 $R/tools/kernel_timeline.py $O/tl_${shp}_$w --after k_verify_walk | tail -8 >> $O/timeline_${shp}_$w.txt 2>&1
    grep '^{' $O/tl_${shp}_$w.log >> $O/timeline_${shp}_$w.txt
  done
done
echo done > $O/DONE
