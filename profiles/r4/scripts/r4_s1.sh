#!/bin/bash
# Round 4, session 1: product GPU suite on this build, the VMM diagnosis
# probe, the guard module alone, and bench.py's c3 / c3_small legs.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s1; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 600 $O/pytest_gpu.log python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step 300 $O/vmm_probe.log python3 -u $R/tools/vmm_probe.py --iters 20
step 300 $O/pytest_guard.log python3 -u -m pytest $R/tests/test_gpu_guard.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider
step 300 $O/c3dev_zipf.log python3 $R/tools/bench_c3dev.py --shape zipf --rounds 2
step 300 $O/c3dev_small.log python3 $R/tools/bench_c3dev.py --shape small --gib 1
step 300 $O/tl_small.log rocprofv3 --kernel-trace -d $O/tl_small -o tl -- python3 $R/tools/bench_c3dev.py --shape small --gib 1 --iters 3
python3 $R/tools/kernel_timeline.py $O/tl_small --after k_count_hist > $O/timeline_small.txt 2>&1
echo done > $O/DONE
