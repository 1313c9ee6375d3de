cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5h
timeout -k 10 480 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5h/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r5h/pytest_gpu.log
if [ $rc -eq 0 ]; then
  timeout -k 10 400 python -u tools/ab_fused.py --hook revel_debug_set_dense_quad --rounds 4 > gpurun_out/r5h/ab_dense_quad.log 2>&1
  echo "rc=$?"; tail -n 1 gpurun_out/r5h/ab_dense_quad.log
fi
