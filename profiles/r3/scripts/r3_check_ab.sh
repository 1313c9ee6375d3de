#!/bin/bash
# GPU product tests on the in-tree build, then an alternating-process A/B of
# builds on the C3 image: tools/r3_check_ab.sh <tag> <rounds> <A.so> <B.so> [more.so ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; n=$2; shift 2
O=$R/gpurun_out/$tag; mkdir -p "$O"
"$R/tools/box_step.sh" 600 "$O/pytest_product.log" python3 -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 \
    --timeout-method thread --ignore="$R/tests/test_experiments_gpu.py" || exit 99
tail -2 "$O/pytest_product.log"
grep -q " passed" "$O/pytest_product.log" && ! grep -q "failed\|error" "$O/pytest_product.log" || { echo "tests failed"; exit 1; }
"$R/tools/ab_c3.sh" "$tag" "$n" "$@"
