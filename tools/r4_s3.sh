#!/bin/bash
# Round 4, session 3: the fused pipeline (verify_walk.inc) -- parity of the
# verify tests on every path, then an alternating A/B of the fused pipeline
# against the count pass in the same library on bench.py's images, then the
# VMM diagnosis probe and the guard module.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s3; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 400 $O/pytest_verify.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or expander or rfc3720"
grep -q " passed" $O/pytest_verify.log && ! grep -q -E "[0-9]+ failed|error" $O/pytest_verify.log || { echo "verify tests failed"; tail -30 $O/pytest_verify.log; exit 1; }
$R/tools/ab_dev.sh r4s3 3 zipf $R/build/ab/base.so:0 $R/build/ab/base.so:1 || exit 99
$R/tools/ab_dev.sh r4s3 2 small $R/build/ab/base.so:0 $R/build/ab/base.so:1 $R/build/ab/base.so:3 || exit 99
step 300 $O/tl_walk.log rocprofv3 --kernel-trace -d $O/tl_walk -o tl -- python3 $R/tools/bench_c3dev.py --walk 1 --iters 3
python3 $R/tools/kernel_timeline.py $O/tl_walk --after k_verify_walk | tail -12 > $O/timeline_walk.txt 2>&1
step 300 $O/vmm_probe.log python3 -u $R/tools/vmm_probe.py --iters 20
step 300 $O/pytest_guard.log python3 -u -m pytest $R/tests/test_gpu_guard.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider
echo done > $O/DONE
