#!/bin/bash
# Round-5 evidence, part A: GPU suite, smoke, bench.py and its rocprofv3 kernel trace, experiment arms.
set -u
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev5_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 600 "$O/pytest_product.log" python3 -u -m pytest "$R/tests" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
step 120 "$O/smoke.log" python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()"
step 420 "$O/bench.log" python3 "$R/bench.py"
step 420 "$O/bench_trace.log" rocprofv3 --kernel-trace --stats -d "$O/bench_trace" -o bench -f csv -- python3 "$R/bench.py"
step 300 "$O/pytest_experiments.log" python3 -u -m pytest "$R/tests/test_experiments_gpu.py" -m experiment -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider
echo done > "$O/DONE_A"
