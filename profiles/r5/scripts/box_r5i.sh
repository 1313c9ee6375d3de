cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5i
timeout -k 10 480 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5i/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r5i/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 200 python -u tools/fused_phases.py --kernel fused2 --lib build/ab/phases.so --shape small > gpurun_out/r5i/phases_fused2_small.log 2>&1 && \
  timeout -k 10 200 python -u tools/fused_phases.py --kernel fused2 --lib build/ab/phases.so --shape zipf > gpurun_out/r5i/phases_fused2_zipf.log 2>&1 && \
  timeout -k 10 400 python -u tools/ab_fused.py --hook revel_debug_set_fused --on 2 --rounds 3 > gpurun_out/r5i/ab_fused2.log 2>&1
  echo "rc=$?"; tail -n 1 gpurun_out/r5i/phases_fused2_small.log gpurun_out/r5i/phases_fused2_zipf.log; tail -n 1 gpurun_out/r5i/ab_fused2.log
fi
