cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5d
timeout -k 10 420 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5d/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r5d/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 200 python -u tools/fused_phases.py --lib build/ab/phases.so --shape small > gpurun_out/r5d/phases_small.log 2>&1 && \
  timeout -k 10 200 python -u tools/fused_phases.py --lib build/ab/phases.so --shape zipf > gpurun_out/r5d/phases_zipf.log 2>&1 && \
  timeout -k 10 300 python -u tools/ab_fused.py --rounds 3 > gpurun_out/r5d/ab_fused.log 2>&1
  echo "rc=$?"; tail -n 2 gpurun_out/r5d/phases_small.log gpurun_out/r5d/phases_zipf.log; tail -n 1 gpurun_out/r5d/ab_fused.log
fi
