#!/bin/bash
# Round-2 (session 4) evidence on the current build: GPU suite, smoke, bench,
# rocprofv3 kernel trace of bench.py and of the C3 bench.
# usage: tools/evidence_r2b.sh <tag>
set -u
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 600 "$O/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -q --timeout 300 --timeout-method thread
step 120 "$O/smoke.log" python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()"
step 300 "$O/bench.log" python3 "$R/bench.py"
step 300 "$O/bench_trace.log" rocprofv3 --kernel-trace --stats -d "$O/bench_trace" -o bench -f csv -- python3 "$R/bench.py"
step 300 "$O/c3_trace.log" rocprofv3 --kernel-trace --stats -d "$O/c3_trace" -o c3 -f csv -- \
    python3 "$R/tools/bench_c3.py" --variants 0 --iters 3
step 300 "$O/c3.log" python3 "$R/tools/bench_c3.py" --variants 0 --rounds 3 --iters 5
echo done > "$O/DONE"
