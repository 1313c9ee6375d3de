#!/bin/bash
# Round 4, session 3: the fused pipeline (verify_walk.inc) -- parity of the
# verify tests on every path (in-tree build and the per-sub-row capture
# build), then an alternating A/B on bench.py's images (fused pipeline vs the
# count pass in the same library, ring depth, capture placement, dense2),
# then the VMM diagnosis probe and the guard module.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s3; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
step 400 $O/pytest_verify.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or expander or rfc3720"
ok $O/pytest_verify.log || { echo "verify tests failed"; tail -40 $O/pytest_verify.log; exit 1; }
REVEL_LIB=$A/capsub.so step 400 $O/pytest_verify_capsub.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or expander"
$R/tools/ab_dev.sh r4s3 3 zipf $A/base.so:0 $A/base.so:1 $A/walk16.so:1 $A/capsub.so:0 $A/capsub.so:1 || exit 99
$R/tools/ab_dev.sh r4s3 2 small $A/base.so:0 $A/base.so:1 $A/base.so:3 || exit 99
step 300 $O/tl_walk.log rocprofv3 --kernel-trace -d $O/tl_walk -o tl -- python3 $R/tools/bench_c3dev.py --walk 1 --iters 3
python3 $R/tools/kernel_timeline.py $O/tl_walk --after k_verify_walk | tail -12 > $O/timeline_walk.txt 2>&1
step 300 $O/vmm_probe.log python3 -u $R/tools/vmm_probe.py --iters 20
step 300 $O/pytest_guard.log python3 -u -m pytest $R/tests/test_gpu_guard.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider
echo done > $O/DONE
