cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5g
timeout -k 10 480 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5g/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r5g/pytest_gpu.log
if [ $rc -eq 0 ]; then
  timeout -k 10 200 python -u tools/fused_phases.py --kernel chunks --lib build/ab/phases.so --shape small > gpurun_out/r5g/phases_chunks_small.log 2>&1 && \
  timeout -k 10 300 python -u tools/ab_fused.py --hook revel_debug_set_dense_chunks --rounds 3 --shapes small > gpurun_out/r5g/ab_dense_chunks.log 2>&1
  echo "rc=$?"; tail -n 1 gpurun_out/r5g/phases_chunks_small.log; tail -n 1 gpurun_out/r5g/ab_dense_chunks.log
fi
