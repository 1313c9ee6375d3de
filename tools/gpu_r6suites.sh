#!/bin/bash
# Round 6: smoke, the product GPU suite and the experiment suite on the current tree.
set -o pipefail
O=gpurun_out/${1:-r6suites}; mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 700 python3 -u -m pytest tests/test_experiments_gpu.py -m experiment -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_experiments.log 2>&1 || { tail -30 $O/pytest_experiments.log; exit 1; }
tail -2 $O/pytest_experiments.log
