cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5a
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/r5a/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u tools/ab_fused.py --rounds 3 > gpurun_out/r5a/ab_fused.log 2>&1
  echo "ab rc=$?"
  tail -4 gpurun_out/r5a/ab_fused.log
fi
