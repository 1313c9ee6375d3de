#!/bin/bash
# Round-3 GPU check: smoke, the GPU test suite (product tests, then the
# experiment arms separately), a 2-rank bench rehearsal on one GPU.
# usage: tools/r3_gpu_suite.sh <outdir>   (stops at the first fault-class status)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
S=$R/tools/box_step.sh
$S 180 "$O/smoke.log" python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" || exit 99
$S 900 "$O/pytest_product.log" python3 -u -m pytest "$R/tests" -m gpu -x -v --timeout 300 --timeout-method thread \
    --ignore="$R/tests/test_experiments_gpu.py" || exit 99
$S 300 "$O/pytest_experiments.log" python3 -u -m pytest "$R/tests/test_experiments_gpu.py" -m gpu -q --timeout 120 \
    --timeout-method thread || exit 99
$S 400 "$O/rehearsal2.log" python3 "$R/bench.py" --gpus 2 --share-gpus --steps 5 --warmup 1 --blocks 65536 \
    --e2e-gib 0.5 --c3-gib 0.5 || exit 99
grep -h "passed\|failed\|error" "$O"/pytest_*.log | tail -4
