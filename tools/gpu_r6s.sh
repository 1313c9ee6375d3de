set -o pipefail
O=gpurun_out/r6s1; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 bash tools/ab_libs_c3.sh r6s1/ab 3 d3=product d2=build/ab/d2.so > $O/ab.log 2>&1; echo "ab rc=$?"; cat $O/ab.log
