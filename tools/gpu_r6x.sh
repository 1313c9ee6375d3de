set -o pipefail
O=gpurun_out/r6x1; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_experiments_gpu.py -m experiment -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_experiments.log 2>&1; echo "rc=$?" >> $O/pytest_experiments.log
tail -3 $O/pytest_experiments.log
