#!/bin/bash
# Round 4, session 32: the experiment arms against the final sources, and smoke().
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s32; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 300 $O/pytest_experiments.log python3 -u -m pytest $R/tests/test_experiments_gpu.py -m experiment -q --timeout 120 --timeout-method thread -p no:cacheprovider
step 120 $O/smoke.log python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()"
echo done > $O/DONE
