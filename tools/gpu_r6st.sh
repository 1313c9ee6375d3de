#!/bin/bash
# Round 6: the staged dense kernels (x_verify_dense_staged.inc): parity on the
# experiment verify tests, then the same-process A/B against dense2 on bench.py's images.
set -o pipefail
O=gpurun_out/${1:-r6st1}; mkdir -p $O
timeout -k 10 420 python3 -u -m pytest tests/test_experiments_gpu.py -m experiment -q -x --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "${2:-long_records or golden or zipf_and or partial_last}" \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 420 python3 -u tools/dense_staged_ab.py --rounds ${3:-3} --arms ${4:-4,5,6,7} > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.log
